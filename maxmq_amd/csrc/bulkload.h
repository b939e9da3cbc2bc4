// maxmq_amd/csrc/bulkload.h — decoder of persisted storage.Subscription
// records (vendor/github.com/mochi-co/mqtt/v2/hooks/storage/storage.go:151-161)
// for the bulk reload path (server.go:1377-1393).  See bulkload.cpp.
#pragma once
#include <stdint.h>

#include <functional>
#include <string>

namespace mqm {

struct SubscriptionRecord {  // the fields loadSubscriptions copies (server.go:1379-1386)
  int64_t identifier = 0;
  uint8_t qos = 0, retain_handling = 0;
  bool retain_as_published = false, no_local = false;
};

// returns false to stop the load (parse_subscription_records then returns -2)
using RecordSink = std::function<bool(const std::string &client, const std::string &filter,
                                      const SubscriptionRecord &r)>;

// Decode a JSON array of records, or records concatenated / one per line,
// calling sink for each in order.  Returns 0, -1 at the first record
// encoding/json would reject, -2 when sink stopped the load (the records
// before have been delivered; *n_records counts them).
int parse_subscription_records(const char *data, size_t len, const RecordSink &sink, uint64_t *n_records);

}  // namespace mqm
