// bitcoin.hpp -- C++ host mirror of the reference's `bitcoin` package and of
// the miner's Request -> Result step, on top of libp1hip.so's C ABI.
//
// The reference is Go (no Go toolchain in this image), so the host side above
// the C ABI is C++ with the same names, argument meaning and error behaviour:
//   MsgType / Message / NewRequest / NewResult / NewJoin / String
//       /root/reference/src/github.com/cmu440/bitcoin/message.go:7-62
//   Hash(msg, nonce)
//       /root/reference/src/github.com/cmu440/bitcoin/hash.go:13-17
//       (computed on the GPU: the one-nonce scan [nonce, nonce])
//   Marshal / Unmarshal  -- encoding/json wire form of Message, as used at
//       miner.go:21,55,66 and client.go:35,52
//   miner::HandleRequest -- miner.go:55-66: decode a Request, scan
//       [Lower, Upper] (miner.go:56-63, on the GPU), build the Result.
// The LSP transport (SRC/lsp) is out of scope; tools read/write the same JSON
// messages over stdio instead.
#pragma once
#include <stdint.h>

#include <stdexcept>
#include <string>

namespace bitcoin {

enum MsgType { Join = 0, Request = 1, Result = 2 };  // message.go:7-13

struct Message {  // message.go:18-23
  int64_t Type = Join;  // Go: type MsgType int (64-bit), any value decodes
  std::string Data;
  uint64_t Lower = 0, Upper = 0;
  uint64_t Hash = 0, Nonce = 0;
  std::string String() const;  // message.go:51-62
};

Message NewRequest(const std::string& data, uint64_t lower, uint64_t upper);  // message.go:27-34
Message NewResult(uint64_t hash, uint64_t nonce);                             // message.go:38-44
Message NewJoin();                                                            // message.go:47-49

// bitcoin.Hash on the GPU.  Throws HipError if the library/device fails.
uint64_t Hash(const std::string& msg, uint64_t nonce);

// encoding/json.Marshal of a Message (field order, escaping and number
// format of Go's encoder).
std::string Marshal(const Message& m);
// encoding/json.Unmarshal into a Message (gojson.hpp: Go 1.4's rules).
// Returns true when Go's error would be nil.  On a type error (e.g. a
// negative Lower) *out holds Go's partial decode and false is returned; on
// a syntax error *out is untouched.  miner.go:55 and client.go:53 ignore the
// error and use whatever was decoded.
bool Unmarshal(const std::string& json, Message* out);
// The same, returning gojson::Status (0 ok, 1 type error, 2 syntax error).
int UnmarshalStatus(const std::string& json, Message* out);

struct HipError : std::runtime_error {
  int rc;
  HipError(int code, const std::string& what) : std::runtime_error(what), rc(code) {}
};

}  // namespace bitcoin

namespace miner {

// Nonces handed to the GPU per p1hip_scan call when a request is split
// ("miner-side chunking": one LSP job may cover far more than one GPU pass;
// between chunks the host thread is free, e.g. for LSP epochs).
constexpr uint64_t kDefaultChunk = 1ull << 36;

// Scan [lower, upper] in chunks of `chunk` nonces; same result as one call.
void ScanChunked(const std::string& msg, uint64_t lower, uint64_t upper, uint64_t chunk, uint64_t* hash,
                 uint64_t* nonce);

// miner.go:55-66 for one decoded Request: returns NewResult(min, minIndex).
bitcoin::Message HandleRequest(const bitcoin::Message& req, uint64_t chunk = kDefaultChunk);

}  // namespace miner
