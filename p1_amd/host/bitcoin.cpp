// bitcoin.cpp -- see bitcoin.hpp.  Host code only: every hash is computed
// by libp1hip.so on the GPU.
#include "bitcoin.hpp"

#include <inttypes.h>
#include <stdio.h>

#include <cctype>
#include <cstring>

#include "../../include/p1hip.h"

namespace bitcoin {

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

static void check(int rc) {
  if (rc != P1HIP_OK) throw HipError(rc, std::string("p1hip: ") + p1hip_last_error());
}

uint64_t Hash(const std::string& msg, uint64_t nonce) {
  uint64_t h = 0;
  check(p1hip_hash(reinterpret_cast<const uint8_t*>(msg.data()), msg.size(), nonce, &h));
  return h;
}

// ---------------------------------------------------------------- JSON out
// Go 1.4 encoding/json string escaping (escapeHTML on): ", \, \n, \r, \t
// short forms; other control bytes and < > & as \u00XX; U+2028/2029 escaped;
// invalid UTF-8 bytes become �.
static size_t utf8_decode(const unsigned char* s, size_t n, uint32_t* cp) {
  const unsigned char c = s[0];
  size_t len;
  uint32_t v, min;
  if (c < 0x80) { *cp = c; return 1; }
  if ((c & 0xE0) == 0xC0) { len = 2; v = c & 0x1F; min = 0x80; }
  else if ((c & 0xF0) == 0xE0) { len = 3; v = c & 0x0F; min = 0x800; }
  else if ((c & 0xF8) == 0xF0) { len = 4; v = c & 0x07; min = 0x10000; }
  else return 0;
  if (len > n) return 0;
  for (size_t i = 1; i < len; ++i) {
    if ((s[i] & 0xC0) != 0x80) return 0;
    v = (v << 6) | (s[i] & 0x3F);
  }
  if (v < min || v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) return 0;
  *cp = v;
  return len;
}

static void json_string(std::string& o, const std::string& s) {
  static const char* hex = "0123456789abcdef";
  o.push_back('"');
  const unsigned char* p = reinterpret_cast<const unsigned char*>(s.data());
  size_t i = 0, n = s.size();
  while (i < n) {
    const unsigned char c = p[i];
    if (c < 0x80) {
      if (c >= 0x20 && c != '"' && c != '\\' && c != '<' && c != '>' && c != '&') o.push_back((char)c);
      else if (c == '"' || c == '\\') { o.push_back('\\'); o.push_back((char)c); }
      else if (c == '\n') o += "\\n";
      else if (c == '\r') o += "\\r";
      else if (c == '\t') o += "\\t";
      else { o += "\\u00"; o.push_back(hex[c >> 4]); o.push_back(hex[c & 15]); }
      ++i;
      continue;
    }
    uint32_t cp = 0;
    size_t len = utf8_decode(p + i, n - i, &cp);
    if (len == 0) { o += "\\ufffd"; ++i; continue; }
    if (cp == 0x2028 || cp == 0x2029) { o += cp == 0x2028 ? "\\u2028" : "\\u2029"; i += len; continue; }
    o.append(s, i, len);
    i += len;
  }
  o.push_back('"');
}

std::string Marshal(const Message& m) {
  char buf[160];
  std::string o = "{\"Type\":" + std::to_string((int)m.Type) + ",\"Data\":";
  json_string(o, m.Data);
  snprintf(buf, sizeof buf, ",\"Lower\":%" PRIu64 ",\"Upper\":%" PRIu64 ",\"Hash\":%" PRIu64 ",\"Nonce\":%" PRIu64 "}",
           m.Lower, m.Upper, m.Hash, m.Nonce);
  return o + buf;
}

// ----------------------------------------------------------------- JSON in
namespace {
struct Parser {
  const char* p;
  const char* e;
  void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p; }
  bool lit(const char* s) {
    size_t n = strlen(s);
    if ((size_t)(e - p) < n || strncmp(p, s, n) != 0) return false;
    p += n;
    return true;
  }
  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o.push_back((char)cp);
    else if (cp < 0x800) { o.push_back((char)(0xC0 | (cp >> 6))); o.push_back((char)(0x80 | (cp & 0x3F))); }
    else if (cp < 0x10000) {
      o.push_back((char)(0xE0 | (cp >> 12))); o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      o.push_back((char)(0xF0 | (cp >> 18))); o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); o.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  bool hex4(uint32_t* v) {
    if (e - p < 4) return false;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
      char c = p[i];
      r <<= 4;
      if (c >= '0' && c <= '9') r |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') r |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') r |= (uint32_t)(c - 'A' + 10);
      else return false;
    }
    p += 4;
    *v = r;
    return true;
  }
  bool str(std::string* out) {
    if (p >= e || *p != '"') return false;
    ++p;
    std::string o;
    while (p < e && *p != '"') {
      if ((unsigned char)*p < 0x20) return false;
      if (*p != '\\') { o.push_back(*p++); continue; }
      if (++p >= e) return false;
      char c = *p++;
      switch (c) {
        case '"': o.push_back('"'); break;
        case '\\': o.push_back('\\'); break;
        case '/': o.push_back('/'); break;
        case 'b': o.push_back('\b'); break;
        case 'f': o.push_back('\f'); break;
        case 'n': o.push_back('\n'); break;
        case 'r': o.push_back('\r'); break;
        case 't': o.push_back('\t'); break;
        case 'u': {
          uint32_t cp;
          if (!hex4(&cp)) return false;
          if (cp >= 0xD800 && cp < 0xDC00) {  // surrogate pair
            uint32_t lo;
            const char* save = p;
            if (lit("\\u") && hex4(&lo) && lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            else { p = save; cp = 0xFFFD; }
          } else if (cp >= 0xDC00 && cp < 0xE000) {
            cp = 0xFFFD;
          }
          put_utf8(o, cp);
          break;
        }
        default: return false;
      }
    }
    if (p >= e) return false;
    ++p;
    if (out) *out = o;
    return true;
  }
  // JSON number that must be an unsigned 64-bit integer (Go rejects others).
  bool u64(uint64_t* v, bool allow_neg_int) {
    bool neg = false;
    if (p < e && *p == '-') { neg = true; ++p; }
    if (p >= e || !isdigit((unsigned char)*p)) return false;
    uint64_t r = 0;
    while (p < e && isdigit((unsigned char)*p)) {
      uint64_t d = (uint64_t)(*p - '0');
      if (r > (UINT64_MAX - d) / 10) return false;  // overflow
      r = r * 10 + d;
      ++p;
    }
    if (p < e && (*p == '.' || *p == 'e' || *p == 'E')) return false;
    if (neg) {
      if (!allow_neg_int) return false;
      r = (uint64_t)(-(int64_t)r);
    }
    *v = r;
    return true;
  }
  bool skip() {  // any JSON value
    ws();
    if (p >= e) return false;
    if (*p == '"') return str(nullptr);
    if (*p == '{' || *p == '[') {
      char close = *p == '{' ? '}' : ']';
      bool obj = *p == '{';
      ++p;
      ws();
      if (p < e && *p == close) { ++p; return true; }
      for (;;) {
        ws();
        if (obj) {
          if (!str(nullptr)) return false;
          ws();
          if (p >= e || *p++ != ':') return false;
        }
        if (!skip()) return false;
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == close) { ++p; return true; }
        return false;
      }
    }
    if (lit("true") || lit("false") || lit("null")) return true;
    uint64_t v;
    if (*p == '-' || isdigit((unsigned char)*p)) {
      const char* s = p;
      if (*p == '-') ++p;
      while (p < e && (isdigit((unsigned char)*p) || *p == '.' || *p == 'e' || *p == 'E' || *p == '+' || *p == '-')) ++p;
      return p > s;
    }
    (void)v;
    return false;
  }
};

bool ieq(const std::string& a, const char* b) {
  if (a.size() != strlen(b)) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (tolower((unsigned char)a[i]) != tolower((unsigned char)b[i])) return false;
  return true;
}
}  // namespace

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

namespace miner {

void ScanChunked(const std::string& msg, uint64_t lower, uint64_t upper, uint64_t chunk, uint64_t* hash,
                 uint64_t* nonce) {
  uint64_t best = UINT64_MAX, bi = 0;
  bool found = false;
  if (chunk == 0) chunk = kDefaultChunk;
  if (lower <= upper) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(msg.data());
    for (uint64_t lo = lower;;) {
      const uint64_t hi = (upper - lo >= chunk) ? lo + (chunk - 1) : upper;
      uint64_t h = 0, n = 0;
      int rc = p1hip_scan(p, msg.size(), lo, hi, &h, &n);
      if (rc != P1HIP_OK) throw bitcoin::HipError(rc, std::string("p1hip_scan: ") + p1hip_last_error());
      // chunks are visited in increasing nonce order: strict '<' keeps the
      // first minimum (miner.go:59); an all-MaxUint64 chunk reads (Max, 0)
      if (h < best) { best = h; bi = n; found = true; }
      if (hi == upper) break;
      lo = hi + 1;
    }
  }
  *hash = best;
  *nonce = found ? bi : 0;
}

bitcoin::Message HandleRequest(const bitcoin::Message& req, uint64_t chunk) {
  uint64_t h = 0, n = 0;
  ScanChunked(req.Data, req.Lower, req.Upper, chunk, &h, &n);
  return bitcoin::NewResult(h, n);
}

}  // namespace miner
