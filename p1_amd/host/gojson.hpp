// gojson.hpp -- the pieces of Go 1.4 encoding/json that the host mirror's
// wire formats need (bitcoin.Message, lsp.Message): string escaping as Go's
// encoder writes it, and a strict recursive-descent reader with Go's
// Unmarshal rules (case-insensitive keys, unknown keys skipped, null leaves a
// field unchanged, integers only where Go's target type is an integer).
#pragma once
#include <ctype.h>
#include <stdint.h>
#include <string.h>

#include <string>

namespace gojson {

// ---------------------------------------------------------------- JSON out
// Go 1.4 encoding/json string escaping (escapeHTML on): ", \, \n, \r, \t
// short forms; other control bytes and < > & as \u00XX; U+2028/2029 escaped;
// invalid UTF-8 bytes become �.
inline size_t utf8_decode(const unsigned char* s, size_t n, uint32_t* cp) {
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

inline void json_string(std::string& o, const std::string& s) {
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

// ----------------------------------------------------------------- JSON in
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
  // JSON number into a Go int (int64): integers only, range-checked.
  bool i64(int64_t* v) {
    bool neg = false;
    if (p < e && *p == '-') { neg = true; ++p; }
    if (p >= e || !isdigit((unsigned char)*p)) return false;
    uint64_t r = 0;
    const uint64_t lim = neg ? (uint64_t)INT64_MAX + 1u : (uint64_t)INT64_MAX;
    while (p < e && isdigit((unsigned char)*p)) {
      uint64_t d = (uint64_t)(*p - '0');
      if (r > (lim - d) / 10) return false;
      r = r * 10 + d;
      ++p;
    }
    if (p < e && (*p == '.' || *p == 'e' || *p == 'E')) return false;
    *v = neg ? (int64_t)(0u - r) : (int64_t)r;
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

inline bool ieq(const std::string& a, const char* b) {
  if (a.size() != strlen(b)) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (tolower((unsigned char)a[i]) != tolower((unsigned char)b[i])) return false;
  return true;
}

}  // namespace gojson
