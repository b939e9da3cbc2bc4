/*
 * tools/mqgen.h — deterministic synthetic workload generator (bench/test
 * infrastructure, not part of the product library).
 *
 * Produces subscription filters (with client, QoS and MQTT 5 options) and
 * publish topics shaped like SURVEY.md §B / BASELINE.json configs: per-depth
 * Zipf token vocabularies, '+' / '#' wildcard mix, '$SHARE/<group>/' shared
 * filters, a few '$'-rooted topics, and topics that either instantiate a
 * filter (uniformly, or Zipf-skewed over filter rank for fan-out hubs) or are
 * drawn fresh from the vocabularies.  Everything derives from splitmix64(seed)
 * so a (params) tuple names one workload exactly.
 */
#ifndef MQGEN_H
#define MQGEN_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint64_t seed;
  uint64_t n_filters;
  uint64_t n_topics;
  uint32_t max_depth;       /* levels per filter/topic, <= 32                     */
  uint32_t n_clients;       /* 0 => ceil(n_filters / 4)                           */
  double p_plus;            /* P(filter has >= 1 '+'); two '+' w.p. p_plus^2      */
  double p_hash;            /* P(filter ends in '#'), depth >= 2                   */
  double p_shared;          /* P(filter is $SHARE/g{0..15}/...)                    */
  double p_dollar_topic;    /* P(topic is rooted at a '$' token)                   */
  double p_instantiate;     /* P(topic instantiates a filter)                      */
  double topic_zipf_s;      /* 0 => instantiate filters uniformly; else Zipf(s)    */
  double token_zipf_s;      /* Zipf exponent of per-depth token choice             */
  uint32_t vocab[8];        /* tokens per depth 0..7 (deeper levels use vocab[7])  */
  double depth_w[32];       /* unnormalised weight of filter depth m = i+1         */
  uint32_t n_root_hash;     /* explicit count of root '#' filters                  */
  uint32_t pad_;
  uint64_t client_lo;       /* keep only filters whose client index is in           */
  uint64_t client_hi;       /*   [client_lo, client_hi) (a subscriber shard);       */
                            /*   0, 0 => all.  Topics are drawn from every filter.  */
} mqgen_params;

typedef struct {
  uint64_t n;
  char *bytes;              /* concatenated strings                               */
  uint64_t *offs;           /* n + 1 offsets                                      */
} mqgen_strings;

typedef struct {
  mqgen_strings filters;
  mqgen_strings clients;    /* client name per filter                              */
  uint32_t *client_ids;     /* dense client index per filter                       */
  uint8_t *qos;
  uint8_t *no_local;
  uint8_t *rap;
  uint8_t *rh;
  int32_t *ident;
  mqgen_strings topics;
} mqgen_workload;

/* fills p with the defaults for config 1..5 (SURVEY.md §8d seeds) */
void mqgen_default_params(int config, mqgen_params *p);
int mqgen_generate(const mqgen_params *p, mqgen_workload *out);
void mqgen_free(mqgen_workload *w);

#ifdef __cplusplus
}
#endif
#endif
