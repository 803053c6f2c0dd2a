// libFuzzer harness for the host-side wire codecs: the JSON a miner, server
// or client parses from the network (LSP datagrams, lsp/message.go; the
// bitcoin messages inside their payloads, bitcoin/message.go) and the
// base64 payload codec.  Built with ASan + UBSan (`make fuzz`); run by
// tests/test_fuzz.py and tools/fuzz.sh.
//
// Properties checked on every input, beyond "no sanitizer report":
//   - a syntax error leaves the (fresh) message untouched;
//   - otherwise (no error, or Go's partial decode after a type error) the
//     message re-encodes to a canonical form that decodes error-free to the
//     same fields and re-encodes to the same bytes;
//   - base64: Decode(Encode(Decode(s))) == Decode(s).
// The first input byte picks the codec, so one corpus covers all three.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../p1_amd/host/bitcoin.hpp"
#include "../../p1_amd/host/gojson.hpp"
#include "../../p1_amd/host/lsp_message.hpp"

[[noreturn]] static void property_failed(const char* what, int line) {
  fprintf(stderr, "property failed: %s (line %d)\n", what, line);
  abort();
}
#define REQUIRE(c) \
  do {             \
    if (!(c)) property_failed(#c, __LINE__); \
  } while (0)

static bool same(const lsp::Message& a, const lsp::Message& b) {
  return a.Type == b.Type && a.ConnID == b.ConnID && a.SeqNum == b.SeqNum && a.Size == b.Size &&
         a.Payload == b.Payload && a.PayloadNil == b.PayloadNil;
}

static bool same(const bitcoin::Message& a, const bitcoin::Message& b) {
  return a.Type == b.Type && a.Data == b.Data && a.Lower == b.Lower && a.Upper == b.Upper && a.Hash == b.Hash &&
         a.Nonce == b.Nonce;
}

// decode from a fresh message; a syntax error must leave it untouched,
// anything else must re-encode to a canonical, error-free fixed point
template <class M, class Same>
static void check_codec(const std::string& s, int (*unmarshal)(const std::string&, M*),
                        std::string (*marshal)(const M&), Same same) {
  M m;
  const int st = unmarshal(s, &m);
  if (st == gojson::kSyntaxError) {
    REQUIRE(same(m, M()));
    return;
  }
  (void)m.String();
  const std::string e1 = marshal(m);
  M m2;
  REQUIRE(unmarshal(e1, &m2) == gojson::kOk);
  REQUIRE(same(m, m2));
  REQUIRE(marshal(m2) == e1);
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size == 0) return 0;
  const std::string s((const char*)data + 1, size - 1);
  switch (data[0] % 3) {
    case 0:
      check_codec<lsp::Message>(s, lsp::UnmarshalStatus, lsp::Marshal,
                                [](const lsp::Message& a, const lsp::Message& b) { return same(a, b); });
      break;
    case 1:
      check_codec<bitcoin::Message>(s, bitcoin::UnmarshalStatus, bitcoin::Marshal,
                                    [](const bitcoin::Message& a, const bitcoin::Message& b) { return same(a, b); });
      break;
    default: {
      std::vector<uint8_t> b;
      if (!lsp::Base64Decode(s, &b)) return 0;
      std::vector<uint8_t> b2;
      REQUIRE(lsp::Base64Decode(lsp::Base64Encode(b), &b2));
      REQUIRE(b2 == b);
      break;
    }
  }
  return 0;
}
