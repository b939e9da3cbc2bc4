// maxmq_amd/csrc/bulkload.cpp — bulk load of persisted subscriptions
// (SURVEY.md §8f row 4).
//
// A storage hook persists every subscription as the JSON encoding of
// storage.Subscription (vendor/github.com/mochi-co/mqtt/v2/hooks/storage/
// storage.go:151-161: t, id, client, filter, identifier, retain_handling,
// qos, retain_as_pub, no_local) and Server.readStore replays them through
// loadSubscriptions (server.go:1377-1393): one TopicsIndex.Subscribe per
// record, in order.  parse_subscription_records decodes a blob of such records
// (a JSON array, or concatenated / newline-separated objects as a key-value
// store dumps them) with encoding/json's rules for these field types:
//   - keys match the struct tags exactly or case-insensitively (Go's fold,
//     incl. U+017F ~ 's' and U+212A ~ 'k'); unknown keys are skipped; the last
//     duplicate wins; null leaves the zero value;
//   - qos / retain_handling are Go bytes (integer literal 0..255),
//     identifier a Go int (integer literal, int64 range), the flags booleans;
//   - strings decode \uXXXX (surrogate pairs; a lone surrogate -> U+FFFD) and
//     replace invalid UTF-8 bytes with U+FFFD.
// A record that encoding/json would reject fails the load (-1) after the
// records before it, like readStore returning the hook's error.
#include "bulkload.h"

#include <cctype>
#include <cstring>
#include <string_view>

namespace mqm {

namespace {

bool is_lit_char(char c) { return std::isalnum((unsigned char)c) || c == '-' || c == '+' || c == '.'; }

bool number_ok(std::string_view s) {  // the JSON number grammar
  size_t i = 0;
  if (i < s.size() && s[i] == '-') i++;
  if (i >= s.size()) return false;
  if (s[i] == '0') {
    i++;
  } else if (s[i] >= '1' && s[i] <= '9') {
    while (i < s.size() && std::isdigit((unsigned char)s[i])) i++;
  } else {
    return false;
  }
  if (i < s.size() && s[i] == '.') {
    const size_t d = ++i;
    while (i < s.size() && std::isdigit((unsigned char)s[i])) i++;
    if (i == d) return false;
  }
  if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
    i++;
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) i++;
    const size_t d = i;
    while (i < s.size() && std::isdigit((unsigned char)s[i])) i++;
    if (i == d) return false;
  }
  return i == s.size();
}

void put_utf8(std::string &o, uint32_t cp) {
  if (cp < 0x80) {
    o += (char)cp;
  } else if (cp < 0x800) {
    o += (char)(0xC0 | (cp >> 6));
    o += (char)(0x80 | (cp & 0x3F));
  } else if (cp < 0x10000) {
    o += (char)(0xE0 | (cp >> 12));
    o += (char)(0x80 | ((cp >> 6) & 0x3F));
    o += (char)(0x80 | (cp & 0x3F));
  } else {
    o += (char)(0xF0 | (cp >> 18));
    o += (char)(0x80 | ((cp >> 12) & 0x3F));
    o += (char)(0x80 | ((cp >> 6) & 0x3F));
    o += (char)(0x80 | (cp & 0x3F));
  }
}

// length of the valid UTF-8 sequence at q (utf8.DecodeRune's rules), 0 if invalid
int utf8_len(const unsigned char *q, const unsigned char *e) {
  const unsigned c = q[0];
  if (c < 0x80) return 1;
  int n;
  unsigned lo = 0x80, hi = 0xBF;
  if (c >= 0xC2 && c <= 0xDF) {
    n = 2;
  } else if (c >= 0xE0 && c <= 0xEF) {
    n = 3;
    if (c == 0xE0) lo = 0xA0;
    if (c == 0xED) hi = 0x9F;  // surrogates are invalid
  } else if (c >= 0xF0 && c <= 0xF4) {
    n = 4;
    if (c == 0xF0) lo = 0x90;
    if (c == 0xF4) hi = 0x8F;
  } else {
    return 0;
  }
  if (e - q < n || q[1] < lo || q[1] > hi) return 0;
  for (int i = 2; i < n; i++)
    if (q[i] < 0x80 || q[i] > 0xBF) return 0;
  return n;
}

struct Parser {
  const char *p, *end;

  void ws() {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++;
  }
  bool eat(char c) {
    ws();
    if (p < end && *p == c) {
      p++;
      return true;
    }
    return false;
  }
  bool peek(char c) {
    ws();
    return p < end && *p == c;
  }
  std::string_view literal() {  // number / true / false / null
    ws();
    const char *q = p;
    while (q < end && is_lit_char(*q)) q++;
    const std::string_view lit(p, (size_t)(q - p));
    p = q;
    return lit;
  }
  bool hex4(uint32_t *v) {
    if (end - p < 4) return false;
    uint32_t x = 0;
    for (int i = 0; i < 4; i++) {
      const char c = p[i];
      x <<= 4;
      if (c >= '0' && c <= '9')
        x |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f')
        x |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F')
        x |= (uint32_t)(c - 'A' + 10);
      else
        return false;
    }
    p += 4;
    *v = x;
    return true;
  }

  bool string(std::string *out) {
    if (!eat('"')) return false;
    out->clear();
    while (p < end) {
      const unsigned char c = (unsigned char)*p;
      if (c == '"') {
        p++;
        return true;
      }
      if (c < 0x20) return false;  // control characters must be escaped
      if (c != '\\') {
        const int n = utf8_len((const unsigned char *)p, (const unsigned char *)end);
        if (n == 0) {  // invalid byte -> U+FFFD
          put_utf8(*out, 0xFFFD);
          p++;
        } else {
          out->append(p, (size_t)n);
          p += n;
        }
        continue;
      }
      if (++p >= end) return false;
      const char e = *p++;
      switch (e) {
        case '"': *out += '"'; break;
        case '\\': *out += '\\'; break;
        case '/': *out += '/'; break;
        case 'b': *out += '\b'; break;
        case 'f': *out += '\f'; break;
        case 'n': *out += '\n'; break;
        case 'r': *out += '\r'; break;
        case 't': *out += '\t'; break;
        case 'u': {
          uint32_t cp;
          if (!hex4(&cp)) return false;
          if (cp >= 0xD800 && cp < 0xDC00) {  // high surrogate: a low one must follow
            const char *save = p;
            uint32_t lo = 0;
            if (end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
              p += 2;
              if (hex4(&lo) && lo >= 0xDC00 && lo < 0xE000) {
                put_utf8(*out, 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00));
                break;
              }
            }
            p = save;  // the next escape is decoded on its own
            cp = 0xFFFD;
          } else if (cp >= 0xDC00 && cp < 0xE000) {
            cp = 0xFFFD;
          }
          put_utf8(*out, cp);
          break;
        }
        default:
          return false;
      }
    }
    return false;
  }

  bool skip_value(int depth = 0) {  // t, id and unknown keys
    ws();
    if (p >= end || depth > 64) return false;
    const char c = *p;
    if (c == '"') {
      std::string tmp;
      return string(&tmp);
    }
    if (c == '{' || c == '[') {
      const char close = c == '{' ? '}' : ']';
      p++;
      if (eat(close)) return true;
      for (;;) {
        if (c == '{') {
          std::string k;
          if (!string(&k) || !eat(':')) return false;
        }
        if (!skip_value(depth + 1)) return false;
        if (eat(',')) continue;
        return eat(close);
      }
    }
    const std::string_view lit = literal();
    return lit == "true" || lit == "false" || lit == "null" || number_ok(lit);
  }

  // a Go integer field: strconv.ParseInt of the number literal's text
  bool integer(int64_t lo, int64_t hi, int64_t *out, bool *is_null) {
    if (peek('"')) return false;  // a string into a number field
    const std::string_view lit = literal();
    if (lit == "null") {
      *is_null = true;
      return true;
    }
    if (!number_ok(lit)) return false;
    size_t i = lit[0] == '-' ? 1 : 0;
    unsigned __int128 v = 0;
    for (; i < lit.size(); i++) {
      if (!std::isdigit((unsigned char)lit[i])) return false;  // fraction / exponent: not an integer
      v = v * 10 + (unsigned)(lit[i] - '0');
      if (v > ((unsigned __int128)1 << 64)) return false;
    }
    const __int128 sv = lit[0] == '-' ? -(__int128)v : (__int128)v;
    if (sv < lo || sv > hi) return false;
    *out = (int64_t)sv;
    return true;
  }

  bool boolean(bool *out, bool *is_null) {
    const std::string_view lit = literal();
    if (lit == "true")
      *out = true;
    else if (lit == "false")
      *out = false;
    else if (lit == "null")
      *is_null = true;
    else
      return false;
    return true;
  }

  bool nullable_string(std::string *out) {
    if (peek('n')) return literal() == "null";
    return string(out);
  }
};

// encoding/json's key match: the exact tag, else a case-insensitive one with
// Go's simple folding (bytes.EqualFold: U+017F 'ſ' ~ 's', U+212A 'K' ~ 'k')
bool key_is(std::string_view key, std::string_view tag) {
  if (key == tag) return true;
  size_t i = 0, j = 0;
  while (i < key.size() && j < tag.size()) {
    const unsigned char c = (unsigned char)key[i];
    const char t = tag[j];
    if (c < 0x80) {
      if ((char)std::tolower(c) != t) return false;
      i++;
    } else if (t == 's' && key.substr(i, 2) == "\xC5\xBF") {
      i += 2;
    } else if (t == 'k' && key.substr(i, 3) == "\xE2\x84\xAA") {
      i += 3;
    } else {
      return false;
    }
    j++;
  }
  return i == key.size() && j == tag.size();
}

}  // namespace

int parse_subscription_records(const char *data, size_t len, const RecordSink &sink, uint64_t *n_records) {
  Parser ps{data ? data : "", data ? data + len : nullptr};
  if (!data) ps.end = ps.p;
  uint64_t n = 0;
  if (n_records) *n_records = 0;
  const bool array = ps.eat('[');
  std::string key, client, filter;
  for (;;) {
    if (array) {
      if (ps.eat(']')) {
        ps.ws();
        return ps.p == ps.end ? 0 : -1;
      }
      if (n > 0 && !ps.eat(',')) return -1;
    } else {
      ps.ws();
      if (ps.p >= ps.end) return 0;
    }
    SubscriptionRecord r{};
    client.clear();
    filter.clear();
    if (ps.peek('n')) {  // a null element decodes to the zero record
      if (ps.literal() != "null") return -1;
    } else {
      if (!ps.eat('{')) return -1;
      if (!ps.eat('}')) {
        for (;;) {
          if (!ps.string(&key) || !ps.eat(':')) return -1;
          bool is_null = false, b = false;
          int64_t v = 0;
          bool ok;
          if (key_is(key, "client")) {
            ok = ps.nullable_string(&client);
          } else if (key_is(key, "filter")) {
            ok = ps.nullable_string(&filter);
          } else if (key_is(key, "identifier")) {
            ok = ps.integer(INT64_MIN, INT64_MAX, &v, &is_null);
            if (ok && !is_null) r.identifier = v;
          } else if (key_is(key, "retain_handling")) {
            ok = ps.integer(0, 255, &v, &is_null);
            if (ok && !is_null) r.retain_handling = (uint8_t)v;
          } else if (key_is(key, "qos")) {
            ok = ps.integer(0, 255, &v, &is_null);
            if (ok && !is_null) r.qos = (uint8_t)v;
          } else if (key_is(key, "retain_as_pub")) {
            ok = ps.boolean(&b, &is_null);
            if (ok && !is_null) r.retain_as_published = b;
          } else if (key_is(key, "no_local")) {
            ok = ps.boolean(&b, &is_null);
            if (ok && !is_null) r.no_local = b;
          } else {
            ok = ps.skip_value();
          }
          if (!ok) return -1;
          if (ps.eat(',')) continue;
          if (ps.eat('}')) break;
          return -1;
        }
      }
    }
    if (!sink(client, filter, r)) return -2;
    if (n_records) *n_records = ++n;
  }
}

}  // namespace mqm
