// planner.hpp -- host side of the scan: midstate, tail templates and the
// split of [lower, upper] into kernel launches.
//
// Reference: the loop being planned is miner.go:56-63 and the bytes being
// hashed are hash.go:15 (fmt.Sprintf("%s %d", msg, nonce)); paths relative
// to /root/reference/src/github.com/cmu440/bitcoin.
//
// Split, per call:
//   1. decades: every nonce in a segment has the same digit count d, so the
//      tail layout (which bytes hold which digit, B_tail, the bit length) is
//      uniform per launch;
//   2. inside a decade, nonce = hi * 10^k + lo.  Whole 10^k-aligned blocks go
//      to a fast piece (one thread per hi value, at most kMaxFastThreads per
//      piece); the ragged edges and decades with d <= k go to generic pieces
//      (one thread per nonce).
//   3. the pieces become the segments of one multi-segment k_scan launch
//      (p1hip.hip), longest-running workgroups first.
// k is 3 except where the last 3 digits would straddle the two tail blocks;
// then k = 1 or 2 so that all lo digits sit in the last block.
#pragma once
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "scan_core.hpp"

namespace p1 {

constexpr uint64_t kMaxFastThreads = 1ull << 26;   // hi values per fast piece
constexpr uint64_t kMaxGenericThreads = 1ull << 26; // nonces per generic piece
constexpr uint64_t kAlgOpsPerCompression = 1384;
// A fast launch wants >= 4 waves on each of the 1024 SIMDs; decades too small
// for that at k = 3 drop to k = 2 or 1 (shorter per-thread loops, more threads)
// instead of running a few long waves on a mostly idle chip.
constexpr uint64_t kMinFastThreads = 1ull << 18;

inline uint64_t pow10u(int e) {
  uint64_t v = 1;
  for (int i = 0; i < e; ++i) v *= 10u;
  return v;
}

// Midstate of the constant prefix msg || ' ' and its leftover bytes.
struct Prefix {
  uint32_t mid[8];
  uint8_t rem[64];
  uint32_t r;    // (L+1) mod 64
  uint64_t len;  // L+1
};

inline void make_prefix(const uint8_t* msg, size_t L, Prefix& P) {
  for (int i = 0; i < 8; ++i) P.mid[i] = iv256(i);
  P.len = (uint64_t)L + 1;
  const uint64_t nfull = P.len / 64;
  uint8_t blk[64];
  for (uint64_t b = 0; b < nfull; ++b) {
    for (int j = 0; j < 64; ++j) {
      const uint64_t pos = b * 64 + j;
      blk[j] = pos < L ? msg[pos] : (uint8_t)' ';
    }
    uint32_t w[64];
    for (int t = 0; t < 16; ++t)
      w[t] = ((uint32_t)blk[4 * t] << 24) | ((uint32_t)blk[4 * t + 1] << 16) |
             ((uint32_t)blk[4 * t + 2] << 8) | (uint32_t)blk[4 * t + 3];
    compress_full(P.mid, w);
  }
  P.r = (uint32_t)(P.len % 64);
  memset(P.rem, 0, sizeof P.rem);
  for (uint32_t j = 0; j < P.r; ++j) {
    const uint64_t pos = nfull * 64 + j;
    P.rem[j] = pos < L ? msg[pos] : (uint8_t)' ';
  }
}

// Where the digits of a d-digit nonce fall in the tail.
struct Layout {
  int d;      // digits
  int q;      // tail byte index of the last digit (r + d - 1)
  int nb;     // tail blocks (B_tail)
  int vb;     // fast path: tail block holding the lo digits
  int k;      // fast path: lo digits per thread loop
  bool trail; // fast path: a constant block follows block vb
};

inline Layout make_layout(uint32_t r, int d) {
  Layout Y;
  Y.d = d;
  Y.q = (int)r + d - 1;
  Y.nb = ((int)r + d + 9 <= 64) ? 1 : 2;
  if (Y.nb == 1) { Y.vb = 0; Y.k = 3; Y.trail = false; }
  else if (Y.q <= 63) { Y.vb = 0; Y.k = 3; Y.trail = true; }     // lo digits in block 0
  else if (Y.q - 64 >= 2) { Y.vb = 1; Y.k = 3; Y.trail = false; } // lo digits in block 1
  else { Y.vb = 1; Y.k = Y.q - 63; Y.trail = false; }             // q in {64,65}: k = 1, 2
  return Y;
}

// Tail words: prefix leftovers, digit bytes ('0' at the last `zero_digits`
// positions, 0 elsewhere), 0x80, zeros, 64-bit bit length.
inline void make_tmpl(const Prefix& P, int d, int zero_digits, uint32_t tmpl[32], int* nb_out) {
  uint8_t b[128];
  memset(b, 0, sizeof b);
  memcpy(b, P.rem, P.r);
  for (int i = 0; i < d; ++i) b[P.r + i] = (i >= d - zero_digits) ? (uint8_t)'0' : 0;
  b[P.r + d] = 0x80;
  const int nb = ((int)P.r + d + 9 <= 64) ? 1 : 2;
  const uint64_t bits = (P.len + (uint64_t)d) * 8u;
  for (int i = 0; i < 8; ++i) b[64 * nb - 1 - i] = (uint8_t)(bits >> (8 * i));
  for (int t = 0; t < 32; ++t)
    tmpl[t] = ((uint32_t)b[4 * t] << 24) | ((uint32_t)b[4 * t + 1] << 16) |
              ((uint32_t)b[4 * t + 2] << 8) | (uint32_t)b[4 * t + 3];
  *nb_out = nb;
}

struct Launch {
  bool fast;
  int fv, nv, mode;  // mode: scan_core.hpp fast_thread
  bool trail;
  FastArgs fa;
  GenArgs ga;
  uint64_t threads;  // threads launched (valid ones)
  uint32_t blocks;
  uint64_t nonces;
  int btail;
};

struct Plan {
  std::vector<Launch> launches;
  uint32_t total_blocks = 0;
  uint64_t total_nonces = 0;
};

inline void add_generic(const Prefix& P, const Layout& Y, uint64_t s, uint64_t e, Plan& plan) {
  // [s, e] inclusive, e >= s
  uint64_t cur = s;
  for (;;) {
    const uint64_t left = e - cur;  // count - 1
    const uint64_t cnt = left >= kMaxGenericThreads ? kMaxGenericThreads : left + 1;
    Launch Ln;
    memset(&Ln, 0, sizeof Ln);
    Ln.fast = false;
    int nb = 0;
    memcpy(Ln.ga.mid, P.mid, sizeof P.mid);
    make_tmpl(P, Y.d, 0, Ln.ga.tmpl, &nb);
    Ln.ga.lo = cur;
    Ln.ga.count = cnt;
    Ln.ga.d = (uint32_t)Y.d;
    Ln.ga.p_last = (uint32_t)Y.q;
    Ln.ga.nb = (uint32_t)nb;
    Ln.threads = cnt;
    Ln.blocks = (uint32_t)((cnt + kBlock - 1) / kBlock);
    Ln.nonces = cnt;
    Ln.btail = nb;
    Ln.ga.part_off = plan.total_blocks;
    plan.total_blocks += Ln.blocks;
    plan.total_nonces += cnt;
    plan.launches.push_back(Ln);
    if (cnt == left + 1) break;
    cur += cnt;
  }
}

// Returns an empty string on success, else a description of the problem.
// `split`: lo digits that straddle two words use the split variants (modes
// 3/4: the first word's work hoisted per 100 or per 10 nonces) rather than
// updating both words per nonce (mode 2).
inline std::string add_fast(const Prefix& P, const Layout& Y, uint64_t hs, uint64_t he, Plan& plan,
                            bool split = true) {
  const int k = Y.k;  // may be below make_layout's choice (see make_plan)
  const int qv = Y.q - 64 * Y.vb;          // last digit inside the variable block
  const int fv = (qv - k + 1) >> 2;
  const int jl = qv >> 2;
  const int nv = jl - fv + 1;
  uint32_t tmpl[32];
  int nb = 0;
  make_tmpl(P, Y.d, k, tmpl, &nb);
  if (nb != Y.nb) return "internal: tail block count mismatch";
  // check the compile-time assumptions of fast_tail_hash
  const uint32_t* vw = tmpl + 16 * Y.vb;
  for (int i = fv + nv + 1; i < 16; ++i) {
    const bool is_len = (!Y.trail && i == 15);
    if (!is_len && vw[i] != 0u) return "internal: unexpected non-zero tail word";
  }
  uint32_t dlt[3][2] = {{0, 0}, {0, 0}, {0, 0}};  // per lo digit (units, tens, hundreds)
  for (int t = 0; t < k; ++t) {
    const int p = qv - t;
    const int slot = (p >> 2) - fv;
    dlt[t][slot] = 1u << (24 - 8 * (p & 3));
  }
  // units are always in the last word; mode 3 = only the hundreds digit in
  // word FV, mode 4 = tens (and hundreds) in word FV
  int mode = 1;
  if (nv == 2) mode = !split ? 2 : (k >= 2 && dlt[1][0] != 0) ? 4 : 3;
  if (mode >= 3 && dlt[0][0] != 0) return "internal: split variant with the units digit in the outer word";
  if (mode == 3 && dlt[1][0] != 0) return "internal: mode 3 with the tens digit in the outer word";
  FastArgs fa;
  memset(&fa, 0, sizeof fa);
  memcpy(fa.mid, P.mid, sizeof P.mid);
  memcpy(fa.tmpl, tmpl, sizeof tmpl);
  if (Y.trail) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i) w[i] = tmpl[16 + i];
    for (int t = 16; t < 64; ++t) w[t] = sched(w, t);
    for (int t = 0; t < 64; ++t) fa.kw2[t] = k256(t) + w[t];
  }
  fa.dh = (uint32_t)(Y.d - k);
  fa.p_last = (uint32_t)(Y.q - k);
  fa.pre = (uint32_t)Y.vb;
  fa.kpow = (uint32_t)pow10u(k);
  fa.n1 = k >= 2 ? 10u : 1u;
  fa.n2 = k >= 3 ? 10u : 1u;
  for (int s = 0; s < 2; ++s) {
    fa.du[s] = dlt[0][s];
    fa.dt[s] = dlt[1][s] - 10u * dlt[0][s];
    fa.dhd[s] = dlt[2][s] - 10u * dlt[1][s];
  }
  uint64_t cur = hs;
  for (;;) {
    const uint64_t left = he - cur;
    const uint64_t cnt = left >= kMaxFastThreads ? kMaxFastThreads : left + 1;
    Launch Ln;
    memset(&Ln, 0, sizeof Ln);
    Ln.fast = true;
    Ln.fv = fv;
    Ln.nv = nv;
    Ln.mode = mode;
    Ln.trail = Y.trail;
    Ln.fa = fa;
    Ln.fa.hi_first = cur;
    Ln.fa.nthreads = (uint32_t)cnt;
    Ln.threads = cnt;
    Ln.blocks = (uint32_t)((cnt + kBlock - 1) / kBlock);
    Ln.nonces = cnt * fa.kpow;
    Ln.btail = Y.nb;
    Ln.fa.part_off = plan.total_blocks;
    plan.total_blocks += Ln.blocks;
    plan.total_nonces += Ln.nonces;
    plan.launches.push_back(Ln);
    if (cnt == left + 1) break;
    cur += cnt;
  }
  return std::string();
}

// Build the launch list for [lower, upper] (inclusive); lower <= upper.
// `fast_ok` = false routes everything through the generic kernel (tests).
// `min_fast_threads` is the occupancy floor that lowers k for small decades;
// tests pass 1 so that k = 3 (and the NV = 2, PRE and TRAIL variants it
// selects) is exercised on ranges the oracle finishes in seconds.
inline std::string make_plan(const uint8_t* msg, size_t L, uint64_t lower, uint64_t upper, Plan& plan,
                             bool fast_ok = true, uint64_t min_fast_threads = kMinFastThreads, bool split = true) {
  Prefix P;
  make_prefix(msg, L, P);
  plan = Plan();
  for (int d = 1; d <= 20; ++d) {
    const uint64_t dlo = (d == 1) ? 0u : pow10u(d - 1);
    const uint64_t dhi = (d == 20) ? ~0ull : pow10u(d) - 1u;
    const uint64_t s = lower > dlo ? lower : dlo;
    const uint64_t e = upper < dhi ? upper : dhi;
    if (s > e) continue;
    Layout Y = make_layout(P.r, d);
    // smaller k keeps the lo digits inside the same block (they are a suffix
    // of make_layout's k digits), so any k <= Y.k is a valid layout
    while (Y.k > 1 && (e - s) / pow10u(Y.k) + 1 < min_fast_threads) --Y.k;
    if (!fast_ok || d <= Y.k) {
      add_generic(P, Y, s, e, plan);
      continue;
    }
    const uint64_t B = pow10u(Y.k);
    const uint64_t hs = s / B + (s % B != 0 ? 1u : 0u);
    bool have = true;
    uint64_t he = 0;
    if (e % B == B - 1) he = e / B;
    else if (e / B == 0) have = false;
    else he = e / B - 1;
    if (have && hs > he) have = false;
    if (!have) {
      add_generic(P, Y, s, e, plan);
      continue;
    }
    if (hs * B > s) add_generic(P, Y, s, hs * B - 1, plan);
    std::string err = add_fast(P, Y, hs, he, plan, split);
    if (!err.empty()) return err;
    if (e % B != B - 1) add_generic(P, Y, (he + 1) * B, e, plan);
  }
  return std::string();
}

}  // namespace p1
