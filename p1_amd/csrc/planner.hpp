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
// k is 3, except when the digits reach 1..7 bytes into the second tail block:
// then k = that count, so that the block holds only lo digits (MODE 5, its
// message schedule tabulated per lo value) and never a digit of block 0.
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
// MODE 5 tabulates tail block 1's schedule for every lo value: at most 7
// digits there (10^7 rows x 256 B = 2.56 GB per layout, built on the device
// and cached there; measured 46.5 GH/s at 7 digits, 48.0 at 6, 48.9 at 5,
// against 34 for the same layouts without a table).
#ifndef P1_MAX_TAB_DIGITS
#define P1_MAX_TAB_DIGITS 7  // A/B builds: make variant NAME=x HOSTEXTRA=-DP1_MAX_TAB_DIGITS=5
#endif
constexpr int kMaxTabDigits = P1_MAX_TAB_DIGITS;

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
  bool tab;   // MODE 5 allowed (tabulated block-1 schedule)
  bool two;   // MODE 7: one digit in block 1 (table), tens/hundreds in block 0's W15; k = 3
};

// `tabulate` = false keeps layouts whose block 1 holds only lo digits on
// the digit-update variants (k = 3 or q - 63, MODE 1) instead of MODE 5:
// the A/B and cross-check path of P1HIP_NO_TABLE.
// `two_level` = false keeps a one-digit block 1 on plain MODE 5 (k = 1)
// instead of MODE 7 (ranges too small for 1000 nonces per thread).
inline Layout make_layout(uint32_t r, int d, bool tabulate = true, bool two_level = true) {
  Layout Y;
  Y.d = d;
  Y.tab = tabulate;
  Y.two = false;
  Y.q = (int)r + d - 1;
  Y.nb = ((int)r + d + 9 <= 64) ? 1 : 2;
  if (Y.nb == 1) { Y.vb = 0; Y.k = 3; Y.trail = false; }
  else if (Y.q <= 63) { Y.vb = 0; Y.k = 3; Y.trail = true; }     // lo digits in block 0
  else if (tabulate && two_level && Y.q == 64 && d > 3) { Y.vb = 1; Y.k = 3; Y.trail = false; Y.two = true; }  // MODE 7
  else if (tabulate && Y.q - 63 <= kMaxTabDigits) { Y.vb = 1; Y.k = Y.q - 63; Y.trail = false; }  // MODE 5
  else if (Y.q - 64 >= 2) { Y.vb = 1; Y.k = 3; Y.trail = false; }                // lo digits in block 1
  else { Y.vb = 1; Y.k = Y.q - 63; Y.trail = false; }                            // q in {64,65}: k = 1, 2
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
  Layout Y;           // fast: the layout it was planned with (Y.k = its k)
  // MODE 5: what its K+W table is built from (build_kwtable); fa.kwtab is
  // filled in by whoever runs the plan (a device copy in p1hip.hip, a host
  // copy in tools/p1emu)
  uint32_t tabw[16];  // tail block 1 words, '0' at the lo digit bytes
  int tabk;           // MODE 5 / 7: digits the table covers (10^tabk rows; MODE 7: 1)
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

// The fast variant <FV, MODE, TRAIL> that runs layout Y at Y.k lo digits:
// FV = first tail word of the variable block holding a lo digit, NV = words
// holding lo digits (1 or 2).  Units are always in the last word; with two
// words, mode 3 = only the hundreds digit in word FV, mode 4 = the tens (and
// hundreds) there, mode 2 = both words updated per nonce (split = false).
struct Variant {
  int fv, nv, mode;
};

inline Variant fast_variant(const Layout& Y, bool split = true) {
  const int qv = Y.q - 64 * Y.vb;
  Variant v;
  if (Y.two) {  // MODE 7: the per-nonce word of block 0 is W15
    v.fv = 15;
    v.nv = 1;
    v.mode = 7;
    return v;
  }
  if (Y.tab && Y.vb == 1 && Y.q - 63 == Y.k) {  // tail block 1 holds only lo digits (W[0], W[1]) and constants
    v.fv = 0;
    v.nv = 1;
    v.mode = 5;
    return v;
  }
  v.fv = (qv - Y.k + 1) >> 2;
  v.nv = (qv >> 2) - v.fv + 1;
  v.mode = 1;
  if (v.nv == 2) v.mode = !split ? 2 : (Y.k >= 2 && ((qv - 1) >> 2) == v.fv) ? 4 : 3;
  // lo digits from byte 0: no hi digit in word FV (TRAIL stays on mode 1:
  // its 64 trailing-block constants already fill the SGPRs)
  else if (!Y.trail && ((qv - Y.k + 1) & 3) == 0) v.mode = 6;
  return v;
}

// Returns an empty string on success, else a description of the problem.
// `split`: lo digits that straddle two words use the split variants (modes
// 3/4: the first word's work hoisted per 100 or per 10 nonces) rather than
// updating both words per nonce (mode 2).
inline std::string add_fast(const Prefix& P, const Layout& Y, uint64_t hs, uint64_t he, Plan& plan,
                            bool split = true) {
  const int k = Y.k;  // may be below make_layout's choice (see make_plan)
  const int qv = Y.q - 64 * Y.vb;          // last digit inside the variable block
  const Variant var = fast_variant(Y, split);
  const int fv = var.fv, nv = var.nv;
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
  // the digit-update modes handle k <= 3; only MODE 5 (tabulated) takes k = 4..7
  if (k > 3 && var.mode != 5) return "internal: more than 3 lo digits outside MODE 5";
  uint32_t dlt[3][2] = {{0, 0}, {0, 0}, {0, 0}};  // per lo digit (units, tens, hundreds)
  if (var.mode == 7) {
    // units: tail byte 64 (block 1, from the table); tens, hundreds: bytes 63,
    // 62 = the low bytes of block 0's W15; block 1 = units, 0x80, zeros, length
    if (Y.q != 64 || k != 3) return "internal: MODE 7 layout";
    if (tmpl[16] != 0x30800000u) return "internal: MODE 7 block 1 word 0";
    for (int i = 17; i < 30; ++i)
      if (tmpl[i] != 0u) return "internal: MODE 7 block 1 not empty";
    if ((tmpl[15] & 0xffffu) != 0x3030u) return "internal: MODE 7 tens/hundreds not in W15";
    dlt[1][0] = 1u;
    dlt[2][0] = 1u << 8;
  } else {
    for (int t = 0; t < k && t < 3; ++t) {
      const int p = qv - t;
      const int slot = (p >> 2) - fv;
      dlt[t][slot] = 1u << (24 - 8 * (p & 3));
    }
  }
  // units are always in the last word; mode 3 = only the hundreds digit in
  // word FV, mode 4 = tens (and hundreds) in word FV
  int mode = var.mode;
  if ((mode == 3 || mode == 4) && dlt[0][0] != 0)
    return "internal: split variant with the units digit in the outer word";
  if (mode == 3 && dlt[1][0] != 0) return "internal: mode 3 with the tens digit in the outer word";
  if (mode == 4 && dlt[1][0] == 0) return "internal: mode 4 without the tens digit in the outer word";
  // the kernel reads the per-nonce word of modes 6 (word FV) and 3/4 (word
  // FV+1) from lane 0 only: no hi digit may sit in it (last hi byte: qv - k).
  // fast_variant only picks mode 6 when that holds; should a later layout
  // change break it, the scan falls back to mode 1 (the same word per lane,
  // slower, still exact) rather than failing.  Modes 3/4 have no shipped
  // per-lane twin (mode 2 is an A/B build), so there it stays an error; the
  // CPU replay runs every (L+1)%64 x digit count x k through this function
  // (tests/test_host_logic.py test_emu_every_tail_layout*), so it cannot fire
  // unnoticed.
  if (mode == 6 && qv - k >= 4 * fv) mode = 1;
  if ((mode == 3 || mode == 4) && qv - k >= 4 * (fv + 1))
    return "internal: hi digit in the wave-uniform per-nonce word";
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
  fa.pre = mode == 7 ? 0u : (uint32_t)Y.vb;  // MODE 7 steps block 0 (W15); its block 1 is the table
  fa.kpow = (uint32_t)pow10u(k);
  fa.nsub = (mode == 5 && k > 3) ? (uint32_t)pow10u(k - 3) : 1u;
  fa.n1 = k >= 2 ? 10u : 1u;
  fa.n2 = k >= 3 ? 10u : 1u;
  for (int s = 0; s < 2; ++s) {
    fa.du[s] = dlt[0][s];
    fa.dt[s] = dlt[1][s] - 10u * dlt[0][s];
    fa.dhd[s] = dlt[2][s] - 10u * dlt[1][s];
  }
  // MODE 5 runs nsub threads per hi: cap the hi values so a piece stays
  // within kMaxFastThreads threads (32-bit thread ids)
  const uint64_t max_hi = kMaxFastThreads / fa.nsub;
  uint64_t cur = hs;
  for (;;) {
    const uint64_t left = he - cur;
    const uint64_t cnt = left >= max_hi ? max_hi : left + 1;
    Launch Ln;
    memset(&Ln, 0, sizeof Ln);
    Ln.fast = true;
    Ln.fv = fv;
    Ln.nv = nv;
    Ln.mode = mode;
    Ln.trail = Y.trail;
    Ln.fa = fa;
    Ln.fa.hi_first = cur;
    Ln.fa.nthreads = (uint32_t)cnt;  // hi values
    // MODE 5 with nsub runs per hi: whole waves of 64 hi values per run
    Ln.threads = fa.nsub > 1 ? (cnt + 63) / 64 * 64 * fa.nsub : cnt;
    Ln.blocks = (uint32_t)((Ln.threads + kBlock - 1) / kBlock);
    Ln.nonces = cnt * fa.kpow;
    Ln.btail = Y.nb;
    Ln.Y = Y;
    if (mode == 5 || mode == 7) memcpy(Ln.tabw, tmpl + 16, sizeof Ln.tabw);
    Ln.tabk = mode == 5 ? k : mode == 7 ? 1 : 0;
    Ln.fa.part_off = plan.total_blocks;
    plan.total_blocks += Ln.blocks;
    plan.total_nonces += Ln.nonces;
    plan.launches.push_back(Ln);
    if (cnt == left + 1) break;
    cur += cnt;
  }
  return std::string();
}

// MODE 5 table of a launch on the host (tools/p1emu; the library builds it on
// the device with k_kwtable): 10^k rows of 64 words, row c for lo value c:
// row[0] = W[0] (round 0's per-thread half already holds K[0]), row[t] =
// K[t] + W[t] for t >= 1, W = tail block 1 with c's k digits in place.
inline std::vector<uint32_t> build_kwtable(const Launch& L) {
  const int k = L.tabk;
  const int qv = L.Y.q - 64;
  const uint32_t rows = (uint32_t)pow10u(k);
  std::vector<uint32_t> tab((size_t)rows * 64u);
  for (uint32_t c = 0; c < rows; ++c) kwtable_row(L.tabw, k, qv, c, tab.data() + (size_t)c * 64u);
  return tab;
}

// [s, e] inside one decade at layout Y: whole 10^k blocks as fast pieces,
// the ragged edges generic -- except for MODE 5 at k > 3, whose edges (up to
// 10^k - 1 nonces each) are planned again at the k = 3 digit layout, so only
// < 10^3 nonces per edge end up one per thread.
inline std::string add_pieces(const Prefix& P, const Layout& Y, uint64_t s, uint64_t e, Plan& plan, bool split) {
  auto edge = [&](uint64_t a, uint64_t b) -> std::string {
    if (Y.k <= 3) {
      add_generic(P, Y, a, b, plan);
      return std::string();
    }
    return add_pieces(P, make_layout(P.r, Y.d, false), a, b, plan, split);
  };
  const uint64_t B = pow10u(Y.k);
  const uint64_t hs = s / B + (s % B != 0 ? 1u : 0u);
  bool have = true;
  uint64_t he = 0;
  if (e % B == B - 1) he = e / B;
  else if (e / B == 0) have = false;
  else he = e / B - 1;
  if (have && hs > he) have = false;
  if (!have) return edge(s, e);
  std::string err;
  if (hs * B > s && !(err = edge(s, hs * B - 1)).empty()) return err;
  if (!(err = add_fast(P, Y, hs, he, plan, split)).empty()) return err;
  if (e % B != B - 1) return edge((he + 1) * B, e);
  return std::string();
}

// Build the launch list for [lower, upper] (inclusive); lower <= upper.
// `fast_ok` = false routes everything through the generic kernel (tests).
// `min_fast_threads` is the occupancy floor that lowers k for small decades;
// tests pass 1 so that k = 3 (and the NV = 2, PRE and TRAIL variants it
// selects) is exercised on ranges the oracle finishes in seconds.
inline std::string make_plan(const uint8_t* msg, size_t L, uint64_t lower, uint64_t upper, Plan& plan,
                             bool fast_ok = true, uint64_t min_fast_threads = kMinFastThreads, bool split = true,
                             bool tabulate = true) {
  Prefix P;
  make_prefix(msg, L, P);
  plan = Plan();
  for (int d = 1; d <= 20; ++d) {
    const uint64_t dlo = (d == 1) ? 0u : pow10u(d - 1);
    const uint64_t dhi = (d == 20) ? ~0ull : pow10u(d) - 1u;
    const uint64_t s = lower > dlo ? lower : dlo;
    const uint64_t e = upper < dhi ? upper : dhi;
    if (s > e) continue;
    Layout Y = make_layout(P.r, d, tabulate);
    // smaller k keeps the lo digits inside the same block (they are a suffix
    // of make_layout's k digits), so any k <= Y.k is a valid layout; a thread
    // runs at most 10^3 nonces (MODE 5 splits k > 3 into runs of 1000), so a
    // MODE 5 layout that is too small goes straight to the k = 3 digit layout
    if (Y.k > 3 && (e - s) / 1000u + 1 < min_fast_threads) Y = make_layout(P.r, d, false);
    // MODE 7 runs 1000 nonces per thread; too small a decade takes plain MODE 5 at k = 1
    if (Y.two && (e - s) / 1000u + 1 < min_fast_threads) Y = make_layout(P.r, d, tabulate, false);
    if (Y.k <= 3)
      while (Y.k > 1 && (e - s) / pow10u(Y.k) + 1 < min_fast_threads) --Y.k;
    if (!fast_ok || d <= Y.k) {
      add_generic(P, Y, s, e, plan);
      continue;
    }
    std::string err = add_pieces(P, Y, s, e, plan, split);
    if (!err.empty()) return err;
  }
  return std::string();
}

// ---------------------------------------------------------------------------
// Cost-balanced contiguous shards (multi-device scans, one shard per device
// or rank).  Every nonce of a decade runs the same kernel variant, and the
// variants differ by up to 2x in cost (TRAIL layouts hash two blocks; a
// variant's cost falls as FV grows).  Equal-count shards therefore finish at
// different times when they cover different decades (configs[3] on 8 GPUs:
// the d = 11 shards run `4,1`, 2% slower per nonce than d = 12's `4,4`), and
// a multi-GPU scan waits for its slowest shard.  plan_shards cuts [lower,
// upper] where the predicted cost, not the nonce count, reaches i/n of the
// total.  The cut points are still contiguous, so the lexicographic min of
// the shard results is the serial first-minimum (miner.go:56-63).
// ---------------------------------------------------------------------------

// SIMD cycles per wave-instruction of the two issue classes at 4 waves/SIMD
// with 8-byte instructions at 4 mod 8 (tools/valu_runs).
constexpr double kCyclesA = 4.37, kCyclesB = 2.66;
// A nonce with nothing hoisted (generic kernel; also the per-thread prologue
// of a fast thread): ~1384 ops per block plus the digit formatting.
constexpr double kUnhoistedCyclesPerBlock = 1600.0 * 3.6;

// Predicted SIMD cycles per wave of 64 nonces of variant <fv, mode, trail>'s
// loop (variant_cost.inc: VALU counts of each variant's per-nonce loop, read
// from the shipped code object by tools/variant_report.py); 0 if not listed.
inline double variant_cycles(int fv, int mode, bool trail) {
#define P1_COST(FV, MODE, TR, A, B) \
  if (fv == FV && mode == MODE && trail == TR) return (A) * kCyclesA + (B) * kCyclesB;
#include "variant_cost.inc"
#undef P1_COST
  return 0.0;
}

// Predicted cost of one nonce of decade d (d digits) for a message whose
// prefix is P: the fast variant's loop plus its per-thread prologue spread
// over the 10^k nonces of a thread, or the generic kernel for d <= k.
inline double nonce_cycles(const Prefix& P, int d) {
  const Layout Y = make_layout(P.r, d);
  const double unhoisted = kUnhoistedCyclesPerBlock * Y.nb;
  if (d <= Y.k) return unhoisted;
  const Variant v = fast_variant(Y);
  double c = variant_cycles(v.fv, v.mode, Y.trail);
  if (c <= 0.0) c = 1384.0 * 3.6 * Y.nb;
  return c + unhoisted / (double)pow10u(Y.k > 3 ? 3 : Y.k);  // a thread runs <= 10^3 nonces
}

// Split [lower, upper] (inclusive, lower <= upper) into n >= 1 contiguous
// shards of near-equal predicted cost: shard i = [first[i], last[i]], in
// order; first[i] > last[i] marks an empty shard (fewer nonces than shards).
// `cost[i]`, if not null, receives each shard's predicted cost (SIMD cycles
// per 64 nonces, summed).
inline void plan_shards(const uint8_t* msg, size_t L, uint64_t lower, uint64_t upper, int n, uint64_t* first,
                        uint64_t* last, double* cost = nullptr) {
  typedef unsigned __int128 u128;
  Prefix P;
  make_prefix(msg, L, P);
  struct Piece { uint64_t s, e; double c; };
  std::vector<Piece> pcs;
  double total = 0.0;
  for (int d = 1; d <= 20; ++d) {
    const uint64_t dlo = (d == 1) ? 0u : pow10u(d - 1);
    const uint64_t dhi = (d == 20) ? ~0ull : pow10u(d) - 1u;
    const uint64_t s = lower > dlo ? lower : dlo;
    const uint64_t e = upper < dhi ? upper : dhi;
    if (s > e) continue;
    const Piece pc = {s, e, nonce_cycles(P, d)};
    pcs.push_back(pc);
    total += ((double)(e - s) + 1.0) * pc.c;
  }
  std::vector<u128> cut((size_t)n + 1);
  cut[0] = lower;
  cut[n] = (u128)upper + 1u;
  size_t j = 0;
  double before = 0.0;  // cost of pieces [0, j)
  for (int i = 1; i < n; ++i) {
    const double t = total * (double)i / (double)n;
    while (j < pcs.size() && before + ((double)(pcs[j].e - pcs[j].s) + 1.0) * pcs[j].c <= t) {
      before += ((double)(pcs[j].e - pcs[j].s) + 1.0) * pcs[j].c;
      ++j;
    }
    u128 x = cut[n];
    if (j < pcs.size()) {
      const double off = (t - before) / pcs[j].c;
      const uint64_t span = pcs[j].e - pcs[j].s;
      const uint64_t o = off <= 0.0 ? 0u : off >= (double)span ? span : (uint64_t)off;
      x = (u128)pcs[j].s + o;
    }
    if (x < cut[i - 1]) x = cut[i - 1];
    if (x > cut[n]) x = cut[n];
    cut[i] = x;
  }
  for (int i = 0; i < n; ++i) {
    if (cut[i] < cut[i + 1]) {
      first[i] = (uint64_t)cut[i];
      last[i] = (uint64_t)(cut[i + 1] - 1u);
    } else {
      first[i] = 1;
      last[i] = 0;
    }
    if (cost) {
      cost[i] = 0.0;
      if (first[i] > last[i]) continue;
      for (const Piece& pc : pcs) {
        const uint64_t s = pc.s > first[i] ? pc.s : first[i];
        const uint64_t e = pc.e < last[i] ? pc.e : last[i];
        if (s <= e) cost[i] += ((double)(e - s) + 1.0) * pc.c;
      }
    }
  }
}

}  // namespace p1
