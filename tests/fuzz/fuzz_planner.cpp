// libFuzzer harness for the host-side planner (p1_amd/csrc/planner.hpp):
// make_plan (decades -> fast / generic pieces -> launches) and plan_shards
// (cost-balanced contiguous shards) on fuzzer-chosen message lengths, ranges
// (biased to decade edges and the top of the u64 range), shard counts and
// planner switches.  Built with ASan + UBSan on the host (`make fuzz`).
// Properties: make_plan succeeds, its launches hash exactly upper-lower+1
// nonces with no empty launch; the shards are in order, contiguous and cover
// [lower, upper] exactly (first > last marks an empty shard).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../p1_amd/csrc/planner.hpp"

[[noreturn]] static void property_failed(const char* what, int line) {
  fprintf(stderr, "property failed: %s (line %d)\n", what, line);
  abort();
}
#define REQUIRE(c) \
  do {             \
    if (!(c)) property_failed(#c, __LINE__); \
  } while (0)

static uint64_t take(const uint8_t*& p, const uint8_t* e) {
  uint64_t v = 0;
  for (int i = 0; i < 8 && p < e; ++i) v = v << 8 | *p++;
  return v;
}

// a nonce near something interesting: 0, a decade edge, the u64 top, raw
static uint64_t pick(uint64_t sel, uint64_t raw) {
  const int d = (int)(sel % 21);
  const int64_t off = (int64_t)(raw % 4001) - 2000;
  switch ((sel >> 8) % 4) {
    case 0: return (uint64_t)(off < 0 ? -off : off);
    case 1: {
      const uint64_t edge = d == 0 ? 1 : (d >= 20 ? ~0ull : p1::pow10u(d));
      return edge + (uint64_t)off;  // wraps near 0 / the top: fine, still a nonce
    }
    case 2: return ~0ull - (raw % 100000);
    default: return raw;
  }
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size < 20) return 0;
  const uint8_t* p = data;
  const uint8_t* e = data + size;
  const uint64_t c0 = take(p, e), c1 = take(p, e);
  const uint32_t flags = (uint32_t)take(p, e);
  const size_t L = (size_t)(c0 % 300);
  std::vector<uint8_t> msg(L, 'x');
  uint64_t lo = pick(c0 >> 9, c1), hi = pick(c1 >> 7, c0 ^ c1);
  if (flags & 1) { const uint64_t t = lo; lo = hi; hi = t; }
  if (lo > hi) { const uint64_t t = lo; lo = hi; hi = t; }
  // the library plans at most one share of this size at a time
  if (hi - lo > (1ull << 40)) hi = lo + (flags >> 8) % (1ull << 40);
  const uint64_t min_threads = (flags & 2) ? 1 : ((flags & 4) ? 200 : p1::kMinFastThreads);
  p1::Plan plan;
  const std::string err = p1::make_plan(msg.data(), L, lo, hi, plan, (flags & 8) == 0, min_threads,
                                        (flags & 16) == 0, (flags & 32) == 0);
  REQUIRE(err.empty());
  uint64_t total = 0;
  for (const p1::Launch& l : plan.launches) {
    REQUIRE(l.nonces > 0);
    total += l.nonces;
  }
  REQUIRE(total == hi - lo + 1);
  REQUIRE(plan.total_nonces == total);

  const int n = 1 + (int)((flags >> 6) % 64);
  std::vector<uint64_t> f(n), t(n);
  p1::plan_shards(msg.data(), L, lo, hi, n, f.data(), t.data());
  uint64_t next = lo;
  bool done = false;
  for (int i = 0; i < n; ++i) {
    if (f[i] > t[i]) continue;
    REQUIRE(!done && f[i] == next);
    if (t[i] == hi) done = true;
    else next = t[i] + 1;
  }
  REQUIRE(done);
  return 0;
}
