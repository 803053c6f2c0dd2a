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

using gojson::ieq;
using gojson::json_string;
using gojson::Parser;

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
  std::string o = "{\"Type\":" + std::to_string((int)m.Type) + ",\"Data\":";
  json_string(o, m.Data);
  snprintf(buf, sizeof buf, ",\"Lower\":%" PRIu64 ",\"Upper\":%" PRIu64 ",\"Hash\":%" PRIu64 ",\"Nonce\":%" PRIu64 "}",
           m.Lower, m.Upper, m.Hash, m.Nonce);
  return o + buf;
}

bool Unmarshal(const std::string& json, Message* out) {
  Parser P{json.data(), json.data() + json.size()};
  Message m = *out;
  P.ws();
  if (P.p >= P.e || *P.p != '{') return false;
  ++P.p;
  P.ws();
  if (P.p < P.e && *P.p == '}') { ++P.p; *out = m; return true; }
  for (;;) {
    P.ws();
    std::string key;
    if (!P.str(&key)) return false;
    P.ws();
    if (P.p >= P.e || *P.p++ != ':') return false;
    P.ws();
    if (P.lit("null")) {
      // Go leaves the field unchanged
    } else if (ieq(key, "Type")) {
      uint64_t v;
      if (!P.u64(&v, true)) return false;
      m.Type = (MsgType)(int)(int64_t)v;
    } else if (ieq(key, "Data")) {
      if (!P.str(&m.Data)) return false;
    } else if (ieq(key, "Lower")) {
      if (!P.u64(&m.Lower, false)) return false;
    } else if (ieq(key, "Upper")) {
      if (!P.u64(&m.Upper, false)) return false;
    } else if (ieq(key, "Hash")) {
      if (!P.u64(&m.Hash, false)) return false;
    } else if (ieq(key, "Nonce")) {
      if (!P.u64(&m.Nonce, false)) return false;
    } else if (!P.skip()) {
      return false;
    }
    P.ws();
    if (P.p < P.e && *P.p == ',') { ++P.p; continue; }
    if (P.p < P.e && *P.p == '}') { ++P.p; break; }
    return false;
  }
  P.ws();
  if (P.p != P.e) return false;
  *out = m;
  return true;
}

}  // namespace bitcoin
