// scan_core.hpp -- per-thread work of the nonce-scan kernels.
//
// Reference loop: /root/reference/src/github.com/cmu440/bitcoin/miner/miner.go:56-63
// (min over i in [Lower, Upper] of bitcoin.Hash(Data, i), strict '<').
// bitcoin.Hash:   /root/reference/src/github.com/cmu440/bitcoin/hash.go:13-17
// (SHA-256 of  msg ' ' decimal(nonce), first 8 digest bytes big-endian).
//
// Data layout (all in registers / kernel arguments; no HBM traffic besides
// one 16-byte partial per workgroup):
//   * "prefix" = msg || ' ' (L+1 bytes).  Its floor((L+1)/64) full blocks are
//     compressed once on the host into `mid` (the midstate).
//   * "tail" = the remaining r = (L+1) mod 64 prefix bytes, the d decimal
//     digits of the nonce, 0x80, zeros and the 64-bit bit length: one or two
//     64-byte blocks (B_tail), kept as 32 big-endian words `tmpl[32]`.
//   * A decade segment (every nonce with the same digit count d) is split as
//     nonce = hi * 10^k + lo.  One GPU thread owns one `hi` and loops over the
//     10^k values of `lo` (k = 3 normally).  Its hi digits are formatted once
//     per thread; the lo digits are ASCII-incremented in one or two message
//     words (`FV`, `FV+1`) inside the loop, so per nonce only the rounds from
//     word FV on and the schedule words that depend on them are recomputed.
//   * Tail blocks before the "variable" block are thread-constant and are
//     compressed once per thread (PRE); a tail block after it (TRAIL) has a
//     constant message, so its K[t]+W[t] are host-precomputed (kw2).
//
// These functions are __host__ __device__ only so tools/p1emu can replay the
// identical per-thread logic on the host in layout tests.
#pragma once
#include "sha256_dev.hpp"

namespace p1 {

constexpr int kBlock = 256;  // threads per workgroup (4 waves of 64)

struct Key {
  uint64_t h;  // bitcoin.Hash value
  uint64_t n;  // nonce
};

P1_HD bool key_lt(const Key& a, const Key& b) {
  return a.h < b.h || (a.h == b.h && a.n < b.n);
}

// Arguments of the fast kernel (one decade segment, aligned 10^k blocks).
struct FastArgs {
  uint32_t mid[8];    // chaining value entering the tail
  uint32_t tmpl[32];  // tail words; '0' at lo-digit bytes, 0 at hi-digit bytes
  uint32_t kw2[64];   // TRAIL: K[t] + W[t] of the constant last block
  uint64_t hi_first;  // hi of thread 0
  uint32_t nthreads;  // number of hi values in this launch
  uint32_t dh;        // hi digit count (= d - k)
  uint32_t p_last;    // tail byte index of the last hi digit
  uint32_t pre;       // 1: variable block is tail block 1, block 0 per-thread
  uint32_t kpow;      // 10^k
  uint32_t n1, n2;    // trip counts of the tens / hundreds digit loops (1 or 10)
  uint32_t du[2];     // units-digit increment of words FV, FV+1
  uint32_t dt[2];     // tens carry:     (tens delta) - 10 * du
  uint32_t dhd[2];    // hundreds carry: (hundreds delta) - 10 * (tens delta)
  uint32_t part_off;  // first partial slot of this launch
  uint64_t kwtab;     // MODE 5: 10^k rows of 64 words (row[0] = W[0], row[t] = K[t] + W[t])
  uint32_t nsub;      // MODE 5: runs of 1000 rows per hi value (10^(k-3) for k > 3, else 1)
  uint32_t pad_;
};

// Arguments of the generic kernel (one nonce per thread, any layout).
struct GenArgs {
  uint32_t mid[8];
  uint32_t tmpl[32];  // 0 at every digit byte
  uint64_t lo;        // first nonce
  uint64_t count;     // nonces in this launch
  uint32_t d;         // digit count
  uint32_t p_last;    // tail byte index of the last digit
  uint32_t nb;        // tail blocks (1 or 2)
  uint32_t part_off;
};

// Write the `ndig` low decimal digits of x (leading zeros kept) as ASCII so
// that the last digit lands on tail byte p_last, OR-ing into tmpl words.
// The digits are built right-aligned in a 24-byte window at compile-time
// positions, funnel-shifted to the uniform byte phase and merged at a
// uniform word offset, so no register array is ever indexed at run time.
P1_HD void place_digits(const uint32_t* tmpl, uint64_t x, uint32_t ndig, uint32_t p_last,
                        uint32_t T[32]) {
  uint32_t G[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 20; ++j) {
    const uint64_t q = x / 10u;
    const uint32_t dig = (uint32_t)(x - q * 10u);
    x = q;
    const uint32_t c = ((uint32_t)j < ndig) ? (dig + 0x30u) : 0u;
    G[5 - j / 4] |= c << (8 * (j % 4));
  }
  // window byte 23 <-> tail byte p_last; window byte 0 <-> tail byte p_last-23
  const uint32_t start = p_last + 9u;  // (p_last - 23) + 32, never negative
  const uint32_t sb = start & 3u;
  const int wb = (int)(start >> 2) - 8;  // tail word of H[0]
  uint32_t H[7];
#pragma unroll
  for (int m = 0; m < 7; ++m) {
    const uint32_t hi = (m == 0) ? 0u : G[m - 1];
    const uint32_t lo = (m == 6) ? 0u : G[m];
    H[m] = funnel(hi, lo, 8u * sb);
  }
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int idx = i - wb;
    uint32_t v = 0;
#pragma unroll
    for (int m = 0; m < 7; ++m) v = (idx == m) ? H[m] : v;
    T[i] = tmpl[i] | v;
  }
}

// ---------------------------------------------------------------------------
// Fast path: thread `tid` scans nonces hi*10^k + [0, 10^k).
// FV = first message word of the variable block holding lo digits,
// NV = number of such words (1 or 2), TRAIL = a constant block follows.
// Words of the variable block:  i <  FV       thread-constant
//                               FV..FV+NV-1   per nonce
//                               FV+NV         uniform (pad byte or 0)
//                               > FV+NV       0, except W15 = bit length
//                                             when !TRAIL (host-checked)
// Everything that does not depend on the per-nonce words is computed once
// per thread before the loop (explicitly: the bitop3 asm is convergent, so
// the compiler would not hoist it): rounds 0..FV-1, the invariant half of
// round FV, every invariant schedule word (as K[t]+W[t]) and the invariant
// part of every variant schedule word.
// ---------------------------------------------------------------------------

// Bit t set <=> schedule word t depends on the per-nonce words.
P1_HD constexpr uint64_t var_mask(int fv, int nv) {
  uint64_t m = 0;
  for (int t = 0; t < 64; ++t) {
    bool v = false;
    if (t < 16) v = (t >= fv && t < fv + nv);
    else v = ((m >> (t - 2)) & 1) || ((m >> (t - 7)) & 1) || ((m >> (t - 15)) & 1) || ((m >> (t - 16)) & 1);
    if (v) m |= 1ull << t;
  }
  return m;
}

template <int FV, int NV, bool TRAIL>
struct FastPre {
  static constexpr uint64_t kVar = var_mask(FV, NV);
  P1_HD static constexpr bool var(int t) { return (kVar >> t) & 1; }
  uint32_t cv[8];   // chaining value entering the variable block
  uint32_t kw[64];  // !var(t): K[t] + W[t];   var(t), t >= 16: invariant partial sum of W[t]
  uint32_t wI[16];  // invariant message words (valid where !var)
  State s1;         // state after round FV, minus the per-nonce word:
                    //   a = s1.v[0] + W[FV], e = s1.v[4] + W[FV], rest as is
};

// The invariant half of round T: everything but the "+ W[T]" that the
// per-nonce word contributes (a = t1 + t2 + W[T], e = d + t1 + W[T]).
template <int T>
P1_HD void round_half(const State& s, State& out) {
  const uint32_t a = s.v[0], b = s.v[1], c = s.v[2], d = s.v[3];
  const uint32_t e = s.v[4], f = s.v[5], g = s.v[6], h = s.v[7];
  const uint32_t t1 = h + bsig1(e) + ch(e, f, g) + k256(T);  // + W[T] per nonce
  const uint32_t t2 = bsig0(a) + maj(a, b, c);
  out.v[0] = t1 + t2; out.v[1] = a; out.v[2] = b; out.v[3] = c;
  out.v[4] = d + t1;  out.v[5] = e; out.v[6] = f; out.v[7] = g;
}

// UNI: the per-nonce word W[FV] (NV = 1) holds no hi digit, so it is the
// same in every lane (an SGPR); the schedule sigmas of that word alone then
// run on the SALU (sha256_dev.hpp ssig0_s/ssig1_s) instead of the VALU.
// The variable block's rounds FV..63 for one nonce: its working state after
// round 63 (not yet added to the chaining value P.cv).
template <int FV, int NV, bool TRAIL, bool UNI = false>
P1_HD State fast_rounds(const FastPre<FV, NV, TRAIL>& P, uint32_t wv0, uint32_t wv1) {
  using FP = FastPre<FV, NV, TRAIL>;
  static_assert(!UNI || NV == 1, "a uniform per-nonce word is the only one");
  uint32_t w[64];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = (i == FV) ? wv0 : (NV == 2 && i == FV + 1) ? wv1 : P.wI[i];
  // P1_SCHED_JIT (A/B builds only): form each variant schedule word right
  // before its round instead of all of them first.  It keeps the live set to
  // the 16-word window -- the c2 loop then fits 64 VGPRs without spills, for
  // an 8-wave build -- but costs FV <= 1 loops ~14% more instructions and
  // gains nothing at 8 waves ("Occupancy budget").
  constexpr bool kJit =
#ifdef P1_SCHED_JIT
      true;
#else
      false;
#endif
  auto sched_var = [&](int t) {
    uint32_t v = P.kw[t];
    if (FP::var(t - 2)) v = add2(v, (UNI && t - 2 == FV) ? ssig1_s(w[t - 2]) : ssig1(w[t - 2]));
    if (FP::var(t - 7)) v = add2(v, w[t - 7]);
    if (FP::var(t - 15)) v = add2(v, (UNI && t - 15 == FV) ? ssig0_s(w[t - 15]) : ssig0(w[t - 15]));
    if (FP::var(t - 16)) v = add2(v, w[t - 16]);
    w[t] = v;
  };
  if constexpr (!kJit) {
#pragma unroll
    for (int t = 16; t < 64; ++t)
      if (FP::var(t)) sched_var(t);
  }
  State s = P.s1;
  s.v[0] = add2(s.v[0], wv0);  // round FV, per-nonce half
  s.v[4] = add2(s.v[4], wv0);
#pragma unroll
  for (int t = FV + 1; t < 64; ++t) {
    if (kJit && t >= 16 && FP::var(t)) sched_var(t);
    sha_round(s, FP::var(t) ? k256(t) + w[t] : P.kw[t]);
  }
  return s;
}

template <int FV, int NV, bool TRAIL, bool UNI = false>
P1_HD uint64_t fast_hash(const FastPre<FV, NV, TRAIL>& P, uint32_t wv0, uint32_t wv1, const uint32_t* kw2) {
  const State s = fast_rounds<FV, NV, TRAIL, UNI>(P, wv0, wv1);
  if constexpr (!TRAIL) {
    return ((uint64_t)(P.cv[0] + s.v[0]) << 32) | (uint64_t)(P.cv[1] + s.v[1]);
  } else {
    uint32_t cv2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) cv2[i] = P.cv[i] + s.v[i];
    State s2;
#pragma unroll
    for (int i = 0; i < 8; ++i) s2.v[i] = cv2[i];
#pragma unroll
    for (int t = 0; t < 64; ++t) sha_round(s2, kw2[t]);
    return ((uint64_t)(cv2[0] + s2.v[0]) << 32) | (uint64_t)(cv2[1] + s2.v[1]);
  }
}

// Per-thread invariants of variant <FV, NV, TRAIL>: P.cv must hold the
// chaining value entering the variable block; Wt are its 16 message words
// (hi digits placed, lo digits '0'), wu the uniform word after the per-nonce
// ones, wlen the bit-length word.
template <int FV, int NV, bool TRAIL>
P1_HD void make_pre(FastPre<FV, NV, TRAIL>& P, const uint32_t Wt[16], uint32_t wu, uint32_t wlen) {
  using FP = FastPre<FV, NV, TRAIL>;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i < FV) P.wI[i] = Wt[i];
    else if (i < FV + NV) P.wI[i] = 0u;  // per-nonce word (never read as invariant)
    else if (i == FV + NV) P.wI[i] = wu;
    else if (!TRAIL && i == 15) P.wI[i] = wlen;
    else P.wI[i] = 0u;
  }
  // invariant schedule: full words where !var, partial sums where var
  {
    uint32_t wi[64];
#pragma unroll
    for (int i = 0; i < 16; ++i) wi[i] = P.wI[i];
#pragma unroll
    for (int t = 16; t < 64; ++t) {
      if (!FP::var(t)) {
        wi[t] = sched(wi, t);
      } else {
        uint32_t v = 0;
        if (!FP::var(t - 2)) v += ssig1(wi[t - 2]);
        if (!FP::var(t - 7)) v += wi[t - 7];
        if (!FP::var(t - 15)) v += ssig0(wi[t - 15]);
        if (!FP::var(t - 16)) v += wi[t - 16];
        wi[t] = 0u;
        P.kw[t] = v;
      }
    }
#pragma unroll
    for (int t = 0; t < 64; ++t)
      if (!FP::var(t)) P.kw[t] = k256(t) + wi[t];
  }
  // rounds 0..FV-1 and the invariant half of round FV
  State s;
#pragma unroll
  for (int i = 0; i < 8; ++i) s.v[i] = P.cv[i];
#pragma unroll
  for (int t = 0; t < FV; ++t) sha_round(s, P.kw[t]);
  round_half<FV>(s, P.s1);
}

// Split variants (modes 3, 4): the lo digits straddle words O and O+1, but
// word O changes only every 100 (mode 3: hundreds digit alone in O) or every
// 10 nonces (mode 4: hundreds and tens in O).  Per thread: the invariants of
// <O, 2> (nothing depends on W[O] or W[O+1]).  Per change of W[O]: this
// update to the invariants of <O+1, 1> -- round O, the invariant half of
// round O+1, and only the schedule terms that come from words depending on
// W[O] but not on W[O+1].  Per nonce: the <O+1, 1> loop, which hoists one
// more round and more schedule words than <O, 2>.
template <int O, bool TRAIL>
P1_HD void outer_update(const FastPre<O, 2, TRAIL>& B, uint32_t wO, FastPre<O + 1, 1, TRAIL>& P) {
  using FB = FastPre<O, 2, TRAIL>;
  using FI = FastPre<O + 1, 1, TRAIL>;
#pragma unroll
  for (int i = 0; i < 8; ++i) P.cv[i] = B.cv[i];
#pragma unroll
  for (int i = 0; i < 16; ++i) P.wI[i] = (i == O) ? wO : B.wI[i];
  uint32_t wx[64];  // full values of the words in var(O,2) \ var(O+1,1)
#pragma unroll
  for (int t = 0; t < 16; ++t) wx[t] = (t == O) ? wO : 0u;
#pragma unroll
  for (int t = 0; t < 16; ++t) P.kw[t] = B.kw[t];
#pragma unroll
  for (int t = 16; t < 64; ++t) {
    if (!FB::var(t)) {
      P.kw[t] = B.kw[t];  // K + W, untouched by either word
      wx[t] = 0u;
      continue;
    }
    uint32_t v = B.kw[t];  // terms from words independent of W[O], W[O+1]
    if (FB::var(t - 2) && !FI::var(t - 2)) v = add2(v, ssig1(wx[t - 2]));
    if (FB::var(t - 7) && !FI::var(t - 7)) v = add2(v, wx[t - 7]);
    if (FB::var(t - 15) && !FI::var(t - 15)) v = add2(v, ssig0(wx[t - 15]));
    if (FB::var(t - 16) && !FI::var(t - 16)) v = add2(v, wx[t - 16]);
    if (FI::var(t)) {
      P.kw[t] = v;  // still a partial sum: it also depends on W[O+1]
      wx[t] = 0u;
    } else {
      wx[t] = v;  // complete now
      P.kw[t] = k256(t) + v;
    }
  }
  // round O with its word, then the invariant half of round O+1
  State s = B.s1;
  s.v[0] = add2(s.v[0], wO);
  s.v[4] = add2(s.v[4], wO);
  round_half<O + 1>(s, P.s1);
}

// Thread setup shared by all fast variants: hi digits placed into the tail,
// PRE block compressed, the variable block's words.
struct FastSetup {
  uint64_t hi;
  bool valid;
  uint32_t cv[8];
  uint32_t Wt[16];
  uint32_t wlen;
};

P1_HD void fast_setup(const FastArgs& A, uint32_t tid, FastSetup& S) {
  S.valid = tid < A.nthreads;
  S.hi = A.hi_first + (S.valid ? tid : 0u);
  uint32_t T[32];
  place_digits(A.tmpl, S.hi, A.dh, A.p_last, T);
#pragma unroll
  for (int i = 0; i < 8; ++i) S.cv[i] = A.mid[i];
  const bool pre = A.pre != 0;
  if (pre) {  // tail block 0 holds only prefix bytes and hi digits
    uint32_t w[64];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = T[i];
    compress_full(S.cv, w);
  }
  // variable block = tail block `pre`; a mask blend (not a select) keeps the
  // compiler from lowering this to a runtime-indexed scratch array
  const uint32_t pm = 0u - (uint32_t)pre;
#pragma unroll
  for (int i = 0; i < 16; ++i) S.Wt[i] = (T[i] & ~pm) | (T[16 + i] & pm);
  S.wlen = pre ? A.tmpl[31] : A.tmpl[15];
}

P1_HD uint32_t uniform_word(const FastArgs& A, int i) {  // the tail word after the per-nonce ones
  return i < 16 ? (A.pre ? A.tmpl[16 + i] : A.tmpl[i]) : 0u;
}

// MODE of a fast variant (how the lo digits sit in the variable block):
//   1  all in word FV (NV = 1)
//   2  in words FV and FV+1, both updated per nonce (NV = 2)
//   3  hundreds in FV, tens and units in FV+1: split, W[FV] work per 100 nonces
//   4  hundreds and tens in FV, units in FV+1: split, W[FV] work per 10 nonces
//   5  uniform block: PRE layout whose variable block (tail block 1) holds
//      only the k lo digits and constants (tail bytes 64..q, k = q - 63 <= 7)
//   6  as 1, with the lo digits from byte 0 of word FV: the word holds no hi
//      digit, so it is wave-uniform (SGPR, SALU updates and sigmas)
//   7  two-level MODE 5: the last digit alone is in tail block 1 (byte 64),
//      the tens and hundreds at bytes 62, 63 of block 0 (W15): per 10 nonces
//      block 0's rounds 15..63 (the `15,1` update), per nonce block 1 from a
//      10-row table (FV = 15: the variable word of block 0)
// In modes 3/4 the per-nonce word FV+1 starts with the lo digits too, so it
// is always wave-uniform and their inner loop always runs as in mode 6.
P1_HD constexpr int mode_nv(int mode) { return mode == 2 || mode == 3 || mode == 4 ? 2 : 1; }

// Row c of a MODE 5 table: tail block 1 (`tabw`, '0' at the lo digit bytes)
// with c's k digits in place -- the 10^j digit at byte qv - j, always in
// words 0..3 for the k <= 7 digits a table covers -- then row[0] = W[0] and
// row[t] = K[t] + W[t].  The device builds tables with it (k_kwtable), the
// host replay (tools/p1emu, planner.hpp build_kwtable) too.
P1_HD void kwtable_row(const uint32_t tabw[16], int k, int qv, uint32_t c, uint32_t* row) {
  uint32_t w[64];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = tabw[i];
  uint32_t x = c;
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    if (j < k) {
      const int p = qv - j;
      const uint32_t v = (x % 10u) << (24 - 8 * (p & 3));
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] += ((p >> 2) == i) ? v : 0u;  // no runtime-indexed array
      x /= 10u;
    }
  }
#pragma unroll
  for (int t = 16; t < 64; ++t) w[t] = sched(w, t);
  row[0] = w[0];
#pragma unroll
  for (int t = 1; t < 64; ++t) row[t] = k256(t) + w[t];
}

// A word of a wave-uniform table row: a scalar load on the device (constant
// address space: the table is read-only for the whole launch).
P1_HD uint32_t ld_uniform(const uint32_t* p, uint32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
  return ((const __attribute__((address_space(4))) uint32_t*)p)[i];
#else
  return p[i];
#endif
}

// MODE 5.  Every word of the variable block is a lo digit or a launch
// constant, so its whole message schedule depends on the lo value alone --
// the same for every thread of the launch at a given loop step.  The host
// tabulates it once per launch (FastArgs::kwtab: row c = lo value c), and the
// per-nonce loop is the 64 rounds with K[t] + W[t] read from the row by
// scalar loads into SGPRs: no schedule work at all.  Round 0's per-thread
// half is hoisted (row[0] is W[0] alone).  The chaining value entering the
// block is the thread's PRE block (hi digits), computed once per 10^k nonces.
// A value the caller knows to be the same in every lane of the wave, made
// visibly uniform (an SGPR) for the compiler.
P1_HD uint32_t wave_uniform(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
#else
  return x;
#endif
}

// One nonce of a MODE 5 / MODE 7 block: s1 = the block's state after the
// per-thread half of round 0, cv = its chaining value, row = the lo value's
// table row (scalar loads).  Returns bitcoin.Hash's 64-bit value.
P1_HD uint64_t table_block(const State& s1, const uint32_t* cv, const uint32_t* row) {
  State s = s1;
  const uint32_t w0 = ld_uniform(row, 0);
  s.v[0] = add2(s.v[0], w0);
  s.v[4] = add2(s.v[4], w0);
#pragma unroll
  for (int t = 1; t < 64; ++t) sha_round(s, ld_uniform(row, (uint32_t)t));
  return ((uint64_t)(cv[0] + s.v[0]) << 32) | (uint64_t)(cv[1] + s.v[1]);
}

// MODE 7 (two-level MODE 5, one digit in tail block 1).  A thread owns
// hi = nonce / 1000: its digits fill block 0 up to byte 61, the hundreds and
// tens digits are bytes 62, 63 (W15 of block 0, '0' in the template and
// ASCII-stepped like mode 1's per-nonce word), the units digit is byte 64 =
// tail block 1, whose schedule is the 10-row MODE 5 table.  Per thread:
// block 0's rounds 0..14 and its W15-invariant schedule (make_pre<15,1>).
// Per tens value: rounds 15..63 of block 0 -> block 1's chaining value and
// the per-thread half of its round 0.  Per nonce: block 1's rounds 1..63.
// Plain MODE 5 at k = 1 recompresses the whole of block 0 every 10 nonces.
P1_HD Key fast_thread_two(const FastArgs& A, uint32_t tid) {
  FastSetup S;
  fast_setup(A, tid, S);  // pre = 0: S.Wt = block 0 with the hi digits, S.cv = midstate
  FastPre<15, 1, false> P;
#pragma unroll
  for (int i = 0; i < 8; ++i) P.cv[i] = S.cv[i];
  make_pre<15, 1, false>(P, S.Wt, 0u, 0u);
  const uint32_t* tab = (const uint32_t*)(uintptr_t)A.kwtab;
  uint32_t w15 = S.Wt[15];
  uint64_t best = ~0ull;
  uint32_t bestc = 0;
  uint32_t c = 0;
  for (uint32_t c2 = 0; c2 < 10u; ++c2) {
    for (uint32_t c1 = 0; c1 < 10u; ++c1) {
      const State s0 = fast_rounds<15, 1, false>(P, w15, 0u);
      uint32_t cv1[8];
      State b0, b1;
#pragma unroll
      for (int i = 0; i < 8; ++i) b0.v[i] = cv1[i] = P.cv[i] + s0.v[i];
      round_half<0>(b0, b1);
#pragma nounroll
      for (uint32_t u = 0; u < 10u; ++u) {
        const uint64_t h = table_block(b1, cv1, tab + (size_t)u * 64u);
        const bool lt = h < best;  // strict '<': first minimum wins (miner.go:59)
        best = lt ? h : best;
        bestc = lt ? c : bestc;
        ++c;
      }
      w15 += A.dt[0];
    }
    w15 += A.dhd[0];
  }
  Key k;
  k.h = S.valid ? best : ~0ull;
  k.n = S.valid ? S.hi * (uint64_t)A.kpow + bestc : ~0ull;
  return k;
}

// With k = 4..7 the 10^k lo values of a hi are split into nsub = 10^(k-3)
// runs of 1000 rows (the same thread length as k = 3, so a 2^32-nonce scan
// still has thousands of workgroups).  The run index must be uniform per wave
// for the row loads to stay scalar: wave w takes run w % nsub for 64 hi values
// (planner: threads = ceil(his / 64) * 64 * nsub).  Each thread compresses
// its hi's PRE block itself.
P1_HD Key fast_thread_uniform(const FastArgs& A, uint32_t tid) {
  const uint32_t wv = tid >> 6, lane = tid & 63u;
  const uint32_t sub = wave_uniform(wv % A.nsub);
  const uint32_t hid = (wv / A.nsub) * 64u + lane;
  const uint32_t per = A.kpow / A.nsub;  // rows of this thread
  const uint32_t c0 = sub * per;
  FastSetup S;
  fast_setup(A, hid, S);
  State s0, s1;
#pragma unroll
  for (int i = 0; i < 8; ++i) s0.v[i] = S.cv[i];
  round_half<0>(s0, s1);
  const uint32_t* tab = (const uint32_t*)(uintptr_t)A.kwtab;
  uint64_t best = ~0ull;
  uint32_t bestc = 0;
  for (uint32_t c = c0; c < c0 + per; ++c) {
    const uint64_t h = table_block(s1, S.cv, tab + (size_t)c * 64u);
    const bool lt = h < best;  // strict '<': first minimum wins (miner.go:59)
    best = lt ? h : best;
    bestc = lt ? c : bestc;
  }
  Key k;
  k.h = S.valid ? best : ~0ull;
  k.n = S.valid ? S.hi * (uint64_t)A.kpow + bestc : ~0ull;
  return k;
}

template <int FV, int MODE, bool TRAIL>
P1_HD Key fast_thread_digits(const FastArgs& A, uint32_t tid) {
  constexpr int NV = mode_nv(MODE);
  FastSetup S;
  fast_setup(A, tid, S);
  FastPre<FV, NV, TRAIL> P;
#pragma unroll
  for (int i = 0; i < 8; ++i) P.cv[i] = S.cv[i];
  make_pre<FV, NV, TRAIL>(P, S.Wt, uniform_word(A, FV + NV), S.wlen);

  // mode 6: word FV has no hi digit (host-checked), so every lane holds the
  // same value; readfirstlane makes that visible and the word an SGPR
  uint32_t wv0 = (MODE == 6) ? wave_uniform(S.Wt[FV]) : S.Wt[FV];
  uint32_t wv1 = (NV == 2) ? S.Wt[FV + 1] : 0u;
  uint64_t best = ~0ull;
  uint32_t bestc = 0;
  uint32_t c = 0;
  if constexpr (MODE <= 2 || MODE == 6) {
    for (uint32_t c2 = 0; c2 < A.n2; ++c2) {
      for (uint32_t c1 = 0; c1 < A.n1; ++c1) {
        for (uint32_t c0 = 0; c0 < 10u; ++c0) {
          const uint64_t h = fast_hash<FV, NV, TRAIL, MODE == 6>(P, wv0, wv1, A.kw2);
          const bool lt = h < best;  // strict '<': first minimum wins (miner.go:59)
          best = lt ? h : best;
          bestc = lt ? c : bestc;
          ++c;
          wv0 += A.du[0];
          if (NV == 2) wv1 += A.du[1];
        }
        wv0 += A.dt[0];
        if (NV == 2) wv1 += A.dt[1];
      }
      wv0 += A.dhd[0];
      if (NV == 2) wv1 += A.dhd[1];
    }
  } else {
    // split: W[FV] changes only in the hundreds (MODE 3) or tens (MODE 4)
    // step (host-checked: du[0] == 0, and dt[0] == 0 for MODE 3).  W[FV+1]
    // begins with the lo digits (no hi digit), so it is wave-uniform, as in
    // mode 6 (not used with TRAIL: its 64 K+W constants already fill the
    // SGPRs, and a uniform word there spills them).  It is re-read from lane
    // 0 per 10 nonces: the compiler packs wv0/wv1 into one (divergent) vector
    // for their shared carry updates.
    constexpr bool kUni = !TRAIL;
    FastPre<FV + 1, 1, TRAIL> Q;
    for (uint32_t c2 = 0; c2 < A.n2; ++c2) {
      if (MODE == 3) outer_update<FV, TRAIL>(P, wv0, Q);
      for (uint32_t c1 = 0; c1 < A.n1; ++c1) {
        if (MODE == 4) outer_update<FV, TRAIL>(P, wv0, Q);
        uint32_t u = kUni ? wave_uniform(wv1) : wv1;
        for (uint32_t c0 = 0; c0 < 10u; ++c0) {
          const uint64_t h = fast_hash<FV + 1, 1, TRAIL, kUni>(Q, u, 0u, A.kw2);
          const bool lt = h < best;  // strict '<': first minimum wins (miner.go:59)
          best = lt ? h : best;
          bestc = lt ? c : bestc;
          ++c;
          u += A.du[1];
        }
        wv1 = u;
        if (MODE == 4) wv0 += A.dt[0];
        wv1 += A.dt[1];
      }
      wv0 += A.dhd[0];
      wv1 += A.dhd[1];
    }
  }
  Key k;
  k.h = S.valid ? best : ~0ull;
  k.n = S.valid ? S.hi * (uint64_t)A.kpow + bestc : ~0ull;
  return k;
}

template <int FV, int MODE, bool TRAIL>
P1_HD Key fast_thread(const FastArgs& A, uint32_t tid) {
  if constexpr (MODE == 5) {
    static_assert(FV == 0 && !TRAIL, "MODE 5 is the whole tail block 1");
    return fast_thread_uniform(A, tid);
  } else if constexpr (MODE == 7) {
    static_assert(FV == 15 && !TRAIL, "MODE 7 steps W15 of block 0");
    return fast_thread_two(A, tid);
  } else {
    return fast_thread_digits<FV, MODE, TRAIL>(A, tid);
  }
}

// ---------------------------------------------------------------------------
// Generic path: one nonce per thread, any tail layout (edges of a range,
// decades with d <= k, and layouts where the lo digits straddle blocks).
// ---------------------------------------------------------------------------
P1_HD Key generic_thread(const GenArgs& A, uint64_t gid) {
  const bool valid = gid < A.count;
  const uint64_t n = A.lo + (valid ? gid : 0u);
  uint32_t T[32];
  place_digits(A.tmpl, n, A.d, A.p_last, T);
  uint32_t cv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) cv[i] = A.mid[i];
  uint32_t w[64];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = T[i];
  compress_full(cv, w);
  if (A.nb == 2) {
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = T[16 + i];
    compress_full(cv, w);
  }
  Key k;
  k.h = valid ? (((uint64_t)cv[0] << 32) | cv[1]) : ~0ull;
  k.n = valid ? n : ~0ull;
  return k;
}

}  // namespace p1
