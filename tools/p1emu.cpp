// p1emu -- TEST TOOL: replays the scan plan and the kernels' per-thread code
// (fast_thread / generic_thread from p1_amd/csrc/scan_core.hpp) on the host,
// one simulated GPU thread at a time, and prints the (hash, nonce) result.
//
// It exists so the layout logic (decade split, digit placement, lo-digit
// deltas, PRE/TRAIL blocks) can be parity-tested against the oracle in the
// CPU-only test suite.  It is never part of libp1hip.so and never used to
// produce a product result.
//
// usage: p1emu <msg-hex> <lower> <upper> [generic | minthreads=N] [nosplit] [notable]
//   minthreads=N sets the planner's occupancy floor (1 keeps k = 3 on small
//   ranges, so every k = 3 variant is replayed); nosplit uses mode 2 for
//   straddling lo digits (p1emu is built with -DP1_NV2_PLAIN); notable keeps
//   layouts whose tail block 1 holds only lo digits off MODE 5
//   prints "<hash> <nonce> <fast_launches> <generic_launches> <variants>"
//   where <variants> lists the fast variants run as FV:MODE:TRAIL,... ("-"
//   when none)
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../p1_amd/csrc/planner.hpp"

using namespace p1;

template <int FV, int MODE, bool TR>
static Key run_fast(const FastArgs& A, uint64_t threads) {
  Key best = {~0ull, ~0ull};
  for (uint64_t t = 0; t < threads; ++t) {
    Key k = fast_thread<FV, MODE, TR>(A, (uint32_t)t);
    if (key_lt(k, best)) best = k;
  }
  return best;
}

static Key dispatch_fast(const Launch& L0) {
  Launch L = L0;
  std::vector<uint32_t> tab;  // MODE 5: the K+W table, here in host memory
  if (L.mode == 5 || L.mode == 7) {
    tab = build_kwtable(L);
    L.fa.kwtab = (uint64_t)(uintptr_t)tab.data();
  }
#define P1_CASE(FV, MODE, TR) \
  if (L.fv == FV && L.mode == MODE && L.trail == TR) return run_fast<FV, MODE, TR>(L.fa, L.threads);
#include "../p1_amd/csrc/fast_variants.inc"
#undef P1_CASE
  fprintf(stderr, "no fast variant fv=%d mode=%d trail=%d\n", L.fv, L.mode, (int)L.trail);
  exit(3);
}

static std::vector<uint8_t> unhex(const char* s) {
  std::vector<uint8_t> v;
  size_t n = strlen(s);
  for (size_t i = 0; i + 1 < n; i += 2) {
    unsigned b;
    sscanf(s + i, "%2x", &b);
    v.push_back((uint8_t)b);
  }
  return v;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s <msg-hex|-> <lower> <upper> [generic|minthreads=N]\n", argv[0]);
    return 2;
  }
  std::vector<uint8_t> msg = strcmp(argv[1], "-") == 0 ? std::vector<uint8_t>() : unhex(argv[1]);
  const uint64_t lower = strtoull(argv[2], nullptr, 10);
  const uint64_t upper = strtoull(argv[3], nullptr, 10);
  const bool generic_only = argc > 4 && strcmp(argv[4], "generic") == 0;
  uint64_t min_threads = kMinFastThreads;
  bool split = true, tabulate = true;
  for (int i = 4; i < argc; ++i) {
    if (strncmp(argv[i], "minthreads=", 11) == 0) min_threads = strtoull(argv[i] + 11, nullptr, 10);
    if (strcmp(argv[i], "nosplit") == 0) split = false;
    if (strcmp(argv[i], "notable") == 0) tabulate = false;
  }
  Key best = {~0ull, ~0ull};
  int nf = 0, ng = 0;
  std::string vars;
  if (lower <= upper) {
    Plan plan;
    std::string err = make_plan(msg.data(), msg.size(), lower, upper, plan, !generic_only, min_threads, split, tabulate);
    if (!err.empty()) {
      fprintf(stderr, "plan error: %s\n", err.c_str());
      return 1;
    }
    for (const Launch& L : plan.launches) {
      Key k;
      if (L.fast) {
        ++nf;
        k = dispatch_fast(L);
        char v[32];
        snprintf(v, sizeof v, "%s%d:%d:%d", vars.empty() ? "" : ",", L.fv, L.mode, (int)L.trail);
        vars += v;
      } else {
        ++ng;
        k = {~0ull, ~0ull};
        for (uint64_t g = 0; g < L.threads; ++g) {
          Key t = generic_thread(L.ga, g);
          if (key_lt(t, k)) k = t;
        }
      }
      if (key_lt(k, best)) best = k;
    }
  }
  if (best.h == ~0ull) best.n = 0;  // identity of miner.go:56
  printf("%" PRIu64 " %" PRIu64 " %d %d %s\n", best.h, best.n, nf, ng, vars.empty() ? "-" : vars.c_str());
  return 0;
}
