// lsp_message.cpp -- see lsp_message.hpp.
#include "lsp_message.hpp"

#include <inttypes.h>
#include <stdio.h>

#include "gojson.hpp"

namespace lsp {

Message NewConnect() { return Message(); }

Message NewData(int64_t connID, int64_t seqNum, int64_t size, const std::string& payload) {
  Message m;
  m.Type = MsgData;
  m.ConnID = connID;
  m.SeqNum = seqNum;
  m.Size = size;
  m.Payload.assign(payload.begin(), payload.end());
  m.PayloadNil = false;
  return m;
}

Message NewAck(int64_t connID, int64_t seqNum) {
  Message m;
  m.Type = MsgAck;
  m.ConnID = connID;
  m.SeqNum = seqNum;
  return m;
}

std::string Message::String() const {
  std::string name, payload;
  switch (Type) {
    case MsgConnect: name = "Connect"; break;
    case MsgData:
      name = "Data";
      payload = " " + std::string(Payload.begin(), Payload.end());
      break;
    case MsgAck: name = "Ack"; break;
    default: break;
  }
  char buf[64];
  snprintf(buf, sizeof buf, " %" PRId64 " %" PRId64, ConnID, SeqNum);
  return "[" + name + buf + payload + "]";
}

static const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

std::string Base64Encode(const std::vector<uint8_t>& b) {
  std::string o;
  o.reserve((b.size() + 2) / 3 * 4);
  size_t i = 0;
  for (; i + 3 <= b.size(); i += 3) {
    const uint32_t v = (uint32_t)b[i] << 16 | (uint32_t)b[i + 1] << 8 | b[i + 2];
    o += kB64[v >> 18]; o += kB64[(v >> 12) & 63]; o += kB64[(v >> 6) & 63]; o += kB64[v & 63];
  }
  if (b.size() - i == 1) {
    const uint32_t v = (uint32_t)b[i] << 16;
    o += kB64[v >> 18]; o += kB64[(v >> 12) & 63]; o += "==";
  } else if (b.size() - i == 2) {
    const uint32_t v = (uint32_t)b[i] << 16 | (uint32_t)b[i + 1] << 8;
    o += kB64[v >> 18]; o += kB64[(v >> 12) & 63]; o += kB64[(v >> 6) & 63]; o += '=';
  }
  return o;
}

// Go's base64.StdEncoding.DecodeString: padding required, '\r' and '\n'
// skipped, trailing bits after the last full byte must be zero (Go 1.4 did not
// check that; neither does this).
bool Base64Decode(const std::string& s, std::vector<uint8_t>* out) {
  std::string t;
  for (char c : s)
    if (c != '\r' && c != '\n') t.push_back(c);
  if (t.size() % 4) return false;
  std::vector<uint8_t> o;
  o.reserve(t.size() / 4 * 3);
  for (size_t i = 0; i < t.size(); i += 4) {
    uint32_t v = 0;
    int pad = 0;
    for (int j = 0; j < 4; ++j) {
      const char c = t[i + j];
      const char* q = c ? strchr(kB64, c) : nullptr;
      if (c == '=') {
        if (i + 4 != t.size() || j < 2) return false;
        ++pad;
        v <<= 6;
        continue;
      }
      if (!q || pad) return false;
      v = v << 6 | (uint32_t)(q - kB64);
    }
    o.push_back((uint8_t)(v >> 16));
    if (pad < 2) o.push_back((uint8_t)(v >> 8));
    if (pad < 1) o.push_back((uint8_t)v);
  }
  *out = std::move(o);
  return true;
}

std::string Marshal(const Message& m) {
  char buf[128];
  snprintf(buf, sizeof buf, "{\"Type\":%" PRId64 ",\"ConnID\":%" PRId64 ",\"SeqNum\":%" PRId64 ",\"Size\":%" PRId64
           ",\"Payload\":", m.Type, m.ConnID, m.SeqNum, m.Size);
  std::string o = buf;
  if (m.PayloadNil) o += "null";
  else o += "\"" + Base64Encode(m.Payload) + "\"";
  return o + "}";
}

bool Unmarshal(const std::string& json, Message* out) {
  gojson::Parser P{json.data(), json.data() + json.size()};
  Message m = *out;
  P.ws();
  if (P.p >= P.e || *P.p != '{') return false;
  ++P.p;
  P.ws();
  if (P.p < P.e && *P.p == '}') {
    ++P.p;
  } else {
    for (;;) {
      P.ws();
      std::string key;
      if (!P.str(&key)) return false;
      P.ws();
      if (P.p >= P.e || *P.p++ != ':') return false;
      P.ws();
      if (P.lit("null")) {
        if (gojson::ieq(key, "Payload")) {  // null into a slice sets it to nil
          m.Payload.clear();
          m.PayloadNil = true;
        }
      } else if (gojson::ieq(key, "Type")) {
        if (!P.i64(&m.Type)) return false;
      } else if (gojson::ieq(key, "ConnID")) {
        if (!P.i64(&m.ConnID)) return false;
      } else if (gojson::ieq(key, "SeqNum")) {
        if (!P.i64(&m.SeqNum)) return false;
      } else if (gojson::ieq(key, "Size")) {
        if (!P.i64(&m.Size)) return false;
      } else if (gojson::ieq(key, "Payload")) {
        std::string b64;
        if (!P.str(&b64) || !Base64Decode(b64, &m.Payload)) return false;
        m.PayloadNil = false;
      } else if (!P.skip()) {
        return false;
      }
      P.ws();
      if (P.p < P.e && *P.p == ',') { ++P.p; continue; }
      if (P.p < P.e && *P.p == '}') { ++P.p; break; }
      return false;
    }
  }
  P.ws();
  if (P.p != P.e) return false;
  *out = m;
  return true;
}

}  // namespace lsp
