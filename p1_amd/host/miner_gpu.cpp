// miner_gpu.cpp -- the parts of bitcoin.hpp that run on the GPU through
// libp1hip.so's C ABI: bitcoin::Hash (hash.go:13-17) and the miner's scan
// step with miner-side chunking (miner.go:55-66).  Every hash is computed by
// the library; there is no CPU path.
#include <string>

#include "../../include/p1hip.h"
#include "bitcoin.hpp"

namespace bitcoin {

static void check(int rc) {
  if (rc != P1HIP_OK) throw HipError(rc, std::string("p1hip: ") + p1hip_last_error());
}

uint64_t Hash(const std::string& msg, uint64_t nonce) {
  uint64_t h = 0;
  check(p1hip_hash(reinterpret_cast<const uint8_t*>(msg.data()), msg.size(), nonce, &h));
  return h;
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
