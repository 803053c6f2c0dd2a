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
// Go 1.4 encoding/json.Unmarshal into a struct of known fields, in Go's two
// stages (decode.go Unmarshal):
//   1. checkValid: the scanner's grammar over the WHOLE input.  A syntax
//      error (trailing bytes, "01", "1.", a bad escape, a raw control byte in
//      a string, ...) returns an error and leaves the target untouched.
//   2. decode: an object's members in order; a member whose key folds to a
//      field name (fold.go: ASCII case, plus U+017F for s and U+212A for k)
//      is assigned by literalStore's rules, later duplicates win, unknown
//      keys are skipped.  A value of the wrong type for its field (a negative
//      or fractional number for a uint64, a string for an int, a number that
//      overflows, bad base64 for []byte, ...) leaves that field unchanged,
//      the rest of the object is still decoded, and Unmarshal returns an
//      error: callers that ignore it (miner.go:55, client.go:53) use the
//      partial result.  Strings are unquoted with invalid UTF-8 bytes and lone
//      surrogates replaced by U+FFFD.  null leaves a field unchanged, except
//      a slice, which becomes nil.  A top-level null decodes nothing and is no
//      error; any other non-object top level is a type error.
// Both stages run without recursion (a datagram of 64 Ki '[' is a syntax
// error or a skip, not a stack overflow).
enum Status { kOk = 0, kTypeError = 1, kSyntaxError = 2 };

inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

// stage 1: the scanner's grammar (scanner.go), with an explicit stack
inline bool valid(const char* p, const char* e) {
  std::string stack;  // '{' / '[' per open container
  auto ws = [&] { while (p < e && is_ws(*p)) ++p; };
  auto string_ok = [&]() -> bool {  // at '"'
    ++p;
    while (p < e) {
      const unsigned char c = (unsigned char)*p++;
      if (c == '"') return true;
      if (c < 0x20) return false;
      if (c != '\\') continue;
      if (p >= e) return false;
      const char x = *p++;
      if (x == 'u') {
        for (int i = 0; i < 4; ++i, ++p)
          if (p >= e || !isxdigit((unsigned char)*p)) return false;
      } else if (!strchr("\"\\/bfnrt", x) || x == 0) {
        return false;
      }
    }
    return false;
  };
  auto number_ok = [&]() -> bool {
    if (p < e && *p == '-') ++p;
    if (p >= e) return false;
    if (*p == '0') ++p;
    else if (*p >= '1' && *p <= '9') while (p < e && isdigit((unsigned char)*p)) ++p;
    else return false;
    if (p < e && *p == '.') {
      ++p;
      if (p >= e || !isdigit((unsigned char)*p)) return false;
      while (p < e && isdigit((unsigned char)*p)) ++p;
    }
    if (p < e && (*p == 'e' || *p == 'E')) {
      ++p;
      if (p < e && (*p == '+' || *p == '-')) ++p;
      if (p >= e || !isdigit((unsigned char)*p)) return false;
      while (p < e && isdigit((unsigned char)*p)) ++p;
    }
    return true;
  };
  auto lit = [&](const char* w) -> bool {
    const size_t n = strlen(w);
    if ((size_t)(e - p) < n || strncmp(p, w, n) != 0) return false;
    p += n;
    return true;
  };
  for (;;) {
    // expecting a value
    ws();
    if (p >= e) return false;
    if (*p == '{' || *p == '[') {
      const char open = *p++;
      ws();
      if (p < e && *p == (open == '{' ? '}' : ']')) {
        ++p;  // empty container: a complete value
      } else {
        stack.push_back(open);
        if (open == '{') {
          if (p >= e || *p != '"' || !string_ok()) return false;
          ws();
          if (p >= e || *p++ != ':') return false;
        }
        continue;
      }
    } else if (*p == '"') {
      if (!string_ok()) return false;
    } else if (*p == '-' || isdigit((unsigned char)*p)) {
      if (!number_ok()) return false;
    } else if (!lit("true") && !lit("false") && !lit("null")) {
      return false;
    }
    // a value is complete: close containers / take the next member
    for (;;) {
      ws();
      if (stack.empty()) return p == e;
      if (p >= e) return false;
      const char open = stack.back();
      if (*p == (open == '{' ? '}' : ']')) {
        ++p;
        stack.pop_back();
        continue;
      }
      if (*p++ != ',') return false;
      if (open == '{') {
        ws();
        if (p >= e || *p != '"' || !string_ok()) return false;
        ws();
        if (p >= e || *p++ != ':') return false;
      }
      break;
    }
  }
}

enum Kind { kNull, kFalse, kTrue, kNumber, kString, kArray, kObject };
struct Value {
  Kind kind;
  const char* b;  // [b, e): the value's bytes (a string's include its quotes)
  const char* e;
};

inline void put_utf8(std::string& o, uint32_t cp) {
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

// unquoteBytes of a string literal from a valid input
inline std::string unquote(const Value& v) {
  auto hex4 = [](const char* q, const char* e, uint32_t* out) -> bool {
    if (e - q < 6 || q[0] != '\\' || q[1] != 'u') return false;
    uint32_t r = 0;
    for (int i = 2; i < 6; ++i) {
      const char c = q[i];
      r <<= 4;
      if (c >= '0' && c <= '9') r |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') r |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') r |= (uint32_t)(c - 'A' + 10);
      else return false;
    }
    *out = r;
    return true;
  };
  std::string o;
  const char* p = v.b + 1;
  const char* e = v.e - 1;  // the closing quote
  while (p < e) {
    const unsigned char c = (unsigned char)*p;
    if (c == '\\') {
      const char x = p[1];
      if (x == 'u') {
        uint32_t cp = 0xFFFD, lo = 0;
        hex4(p, e, &cp);
        p += 6;
        if (cp >= 0xD800 && cp < 0xE000) {  // utf16.IsSurrogate
          if (cp < 0xDC00 && hex4(p, e, &lo) && lo >= 0xDC00 && lo < 0xE000) {
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            p += 6;
          } else {
            cp = 0xFFFD;  // invalid surrogate: only the first escape is consumed
          }
        }
        put_utf8(o, cp);
        continue;
      }
      switch (x) {
        case 'b': o.push_back('\b'); break;
        case 'f': o.push_back('\f'); break;
        case 'n': o.push_back('\n'); break;
        case 'r': o.push_back('\r'); break;
        case 't': o.push_back('\t'); break;
        default: o.push_back(x); break;  // " \ /
      }
      p += 2;
    } else if (c < 0x80) {
      o.push_back((char)c);
      ++p;
    } else {
      uint32_t cp = 0;
      const size_t n = utf8_decode((const unsigned char*)p, (size_t)(e - p), &cp);
      if (n == 0) {  // utf8.DecodeRune: (RuneError, 1)
        o += "\xEF\xBF\xBD";
        ++p;
      } else {
        o.append(p, n);
        p += n;
      }
    }
  }
  return o;
}

// one value of a valid input, skipped without recursion
struct Reader {
  const char* p;
  const char* e;
  void ws() { while (p < e && is_ws(*p)) ++p; }
  void skip_string() {  // at '"'
    ++p;
    while (p < e && *p != '"') p += (*p == '\\') ? 2 : 1;
    ++p;
  }
  Value value() {
    ws();
    Value v{kNull, p, p};
    const char c = *p;
    if (c == '"') {
      v.kind = kString;
      skip_string();
    } else if (c == '{' || c == '[') {
      v.kind = c == '{' ? kObject : kArray;
      int depth = 0;
      do {
        if (*p == '"') { skip_string(); continue; }
        if (*p == '{' || *p == '[') ++depth;
        else if (*p == '}' || *p == ']') --depth;
        ++p;
      } while (depth > 0);
    } else if (c == 't') { v.kind = kTrue; p += 4; }
    else if (c == 'f') { v.kind = kFalse; p += 5; }
    else if (c == 'n') { v.kind = kNull; p += 4; }
    else {
      v.kind = kNumber;
      while (p < e && (isdigit((unsigned char)*p) || *p == '-' || *p == '+' || *p == '.' || *p == 'e' || *p == 'E')) ++p;
    }
    v.e = p;
    return v;
  }
};

// strconv.ParseInt(s, 10, 64) / ParseUint(s, 10, 64) of a JSON number's text
inline bool parse_int(const Value& v, int64_t* out) {
  const char* p = v.b;
  const bool neg = p < v.e && *p == '-';
  if (neg) ++p;
  if (p >= v.e) return false;
  const uint64_t lim = neg ? (uint64_t)INT64_MAX + 1u : (uint64_t)INT64_MAX;
  uint64_t r = 0;
  for (; p < v.e; ++p) {
    if (!isdigit((unsigned char)*p)) return false;
    const uint64_t d = (uint64_t)(*p - '0');
    if (r > (lim - d) / 10) return false;
    r = r * 10 + d;
  }
  *out = neg ? (int64_t)(0u - r) : (int64_t)r;
  return true;
}
inline bool parse_uint(const Value& v, uint64_t* out) {
  if (v.b >= v.e) return false;
  uint64_t r = 0;
  for (const char* p = v.b; p < v.e; ++p) {
    if (!isdigit((unsigned char)*p)) return false;  // a sign is a syntax error for ParseUint
    const uint64_t d = (uint64_t)(*p - '0');
    if (r > (UINT64_MAX - d) / 10) return false;
    r = r * 10 + d;
  }
  *out = r;
  return true;
}

// literalStore's outcome for one field
enum Assign { kSet, kSkip /* d.saveError: field unchanged, decoding goes on */,
              kAbort /* d.error: decoding stops here */ };

// Go int field (int / int64 / MsgType on amd64)
inline Assign assign_int(const Value& v, int64_t* f) {
  if (v.kind == kNull) return kSet;  // no effect
  if (v.kind != kNumber) return kSkip;
  int64_t x;
  if (!parse_int(v, &x)) return kSkip;
  *f = x;
  return kSet;
}
// Go uint64 field
inline Assign assign_uint(const Value& v, uint64_t* f) {
  if (v.kind == kNull) return kSet;
  if (v.kind != kNumber) return kSkip;
  uint64_t x;
  if (!parse_uint(v, &x)) return kSkip;
  *f = x;
  return kSet;
}
// Go string field: a number is d.error (the decode stops), other kinds a
// saved type error
inline Assign assign_string(const Value& v, std::string* f) {
  if (v.kind == kNull) return kSet;
  if (v.kind == kNumber) return kAbort;
  if (v.kind != kString) return kSkip;
  *f = unquote(v);
  return kSet;
}

// fold.go: does `key` (unquoted bytes) match the ASCII field name?
inline bool key_matches(const std::string& key, const char* name) {
  const unsigned char* t = (const unsigned char*)key.data();
  size_t n = key.size();
  for (const char* s = name; *s; ++s) {
    if (n == 0) return false;
    const unsigned char sb = (unsigned char)*s;
    if (t[0] < 0x80) {
      if (sb != t[0] && ((sb & 0xDF) < 'A' || (sb & 0xDF) > 'Z' || (sb & 0xDF) != (t[0] & 0xDF))) return false;
      ++t;
      --n;
      continue;
    }
    uint32_t cp = 0;
    size_t len = utf8_decode(t, n, &cp);
    if (len == 0) return false;
    if ((sb & 0xDF) == 'S' && cp == 0x017F) { t += len; n -= len; continue; }  // long s
    if ((sb & 0xDF) == 'K' && cp == 0x212A) { t += len; n -= len; continue; }  // Kelvin sign
    return false;
  }
  return n == 0;
}

// Stage 2 driver.  field(key, value, reader) -> Assign; returns the Status
// Unmarshal's error would have.
template <class Field>
Status decode_struct(const std::string& json, Field field) {
  const char* b = json.data();
  const char* e = b + json.size();
  if (!valid(b, e)) return kSyntaxError;
  Reader R{b, e};
  R.ws();
  if (*R.p == 'n') return kOk;       // null: no effect, no error
  if (*R.p != '{') return kTypeError;  // string / number / bool / array into a struct
  ++R.p;
  Status st = kOk;
  for (;;) {
    R.ws();
    if (*R.p == '}') break;
    const Value k = R.value();
    R.ws();
    ++R.p;  // ':'
    const Value v = R.value();
    const Assign a = field(unquote(k), v);
    if (a == kAbort) return kTypeError;
    if (a == kSkip) st = kTypeError;
    R.ws();
    if (*R.p == ',') ++R.p;
  }
  return st;
}

}  // namespace gojson
