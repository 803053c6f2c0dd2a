// bitcoin.cpp -- see bitcoin.hpp: the Message type and its encoding/json
// wire form (no GPU here; bitcoin::Hash and the miner loop, which call
// libp1hip.so, are in miner_gpu.cpp).
#include "bitcoin.hpp"

#include <inttypes.h>
#include <stdio.h>

#include <cctype>
#include <cstring>

#include "gojson.hpp"

namespace bitcoin {

using gojson::json_string;

Message NewRequest(const std::string& data, uint64_t lower, uint64_t upper) {
  Message m;
  m.Type = Request;
  m.Data = data;
  m.Lower = lower;
  m.Upper = upper;
  return m;
}

Message NewResult(uint64_t hash, uint64_t nonce) {
  Message m;
  m.Type = Result;
  m.Hash = hash;
  m.Nonce = nonce;
  return m;
}

Message NewJoin() { return Message(); }

std::string Message::String() const {
  char buf[96];
  switch (Type) {
    case Request:
      snprintf(buf, sizeof buf, " %" PRIu64 " %" PRIu64 "]", Lower, Upper);
      return "[Request " + Data + buf;
    case Result:
      snprintf(buf, sizeof buf, "[Result %" PRIu64 " %" PRIu64 "]", Hash, Nonce);
      return buf;
    case Join:
      return "[Join]";
  }
  return "";
}

std::string Marshal(const Message& m) {
  char buf[160];
  std::string o = "{\"Type\":" + std::to_string(m.Type) + ",\"Data\":";
  json_string(o, m.Data);
  snprintf(buf, sizeof buf, ",\"Lower\":%" PRIu64 ",\"Upper\":%" PRIu64 ",\"Hash\":%" PRIu64 ",\"Nonce\":%" PRIu64 "}",
           m.Lower, m.Upper, m.Hash, m.Nonce);
  return o + buf;
}

int UnmarshalStatus(const std::string& json, Message* out) {
  Message m = *out;  // a syntax error leaves *out untouched
  const gojson::Status st = gojson::decode_struct(json, [&](const std::string& key, const gojson::Value& v) {
    using gojson::key_matches;
    if (key_matches(key, "Type")) return gojson::assign_int(v, &m.Type);
    if (key_matches(key, "Data")) return gojson::assign_string(v, &m.Data);
    if (key_matches(key, "Lower")) return gojson::assign_uint(v, &m.Lower);
    if (key_matches(key, "Upper")) return gojson::assign_uint(v, &m.Upper);
    if (key_matches(key, "Hash")) return gojson::assign_uint(v, &m.Hash);
    if (key_matches(key, "Nonce")) return gojson::assign_uint(v, &m.Nonce);
    return gojson::kSet;  // unknown key: skipped
  });
  if (st != gojson::kSyntaxError) *out = m;
  return st;
}

bool Unmarshal(const std::string& json, Message* out) { return UnmarshalStatus(json, out) == gojson::kOk; }

}  // namespace bitcoin
