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

// Go's d.array into a []byte: each element decoded as a uint8 (a failed
// element keeps the byte already at that index), the length set to the
// element count, never nil
static gojson::Assign assign_byte_array(const gojson::Value& v, Message* m) {
  gojson::Reader R{v.b + 1, v.e};
  gojson::Assign st = gojson::kSet;
  size_t i = 0;
  for (;;) {
    R.ws();
    if (*R.p == ']') break;
    const gojson::Value x = R.value();
    if (i >= m->Payload.size()) m->Payload.push_back(0);
    uint64_t b = 0;
    if (x.kind == gojson::kNumber && gojson::parse_uint(x, &b) && b <= 255) m->Payload[i] = (uint8_t)b;
    else if (x.kind == gojson::kNumber) st = gojson::kSkip;  // ParseUint / OverflowUint
    else if (x.kind != gojson::kNull) st = gojson::kSkip;   // string / bool / array / object into uint8
    ++i;
    R.ws();
    if (*R.p == ',') ++R.p;
  }
  m->Payload.resize(i);
  m->PayloadNil = false;
  return st;
}

static gojson::Assign assign_payload(const gojson::Value& v, Message* m) {
  switch (v.kind) {
    case gojson::kNull:  // null into a slice sets it to nil
      m->Payload.clear();
      m->PayloadNil = true;
      return gojson::kSet;
    case gojson::kString: {
      std::vector<uint8_t> b;
      if (!Base64Decode(gojson::unquote(v), &b)) return gojson::kSkip;
      m->Payload = std::move(b);
      m->PayloadNil = false;
      return gojson::kSet;
    }
    case gojson::kArray: return assign_byte_array(v, m);
    case gojson::kNumber: return gojson::kAbort;
    default: return gojson::kSkip;
  }
}

int UnmarshalStatus(const std::string& json, Message* out) {
  Message m = *out;  // a syntax error leaves *out untouched
  const gojson::Status st = gojson::decode_struct(json, [&](const std::string& key, const gojson::Value& v) {
    using gojson::key_matches;
    if (key_matches(key, "Type")) return gojson::assign_int(v, &m.Type);
    if (key_matches(key, "ConnID")) return gojson::assign_int(v, &m.ConnID);
    if (key_matches(key, "SeqNum")) return gojson::assign_int(v, &m.SeqNum);
    if (key_matches(key, "Size")) return gojson::assign_int(v, &m.Size);
    if (key_matches(key, "Payload")) return assign_payload(v, &m);
    return gojson::kSet;  // unknown key: skipped
  });
  if (st != gojson::kSyntaxError) *out = m;
  return st;
}

bool Unmarshal(const std::string& json, Message* out) { return UnmarshalStatus(json, out) == gojson::kOk; }

}  // namespace lsp
