// sha256_dev.hpp -- gfx950 SHA-256 building blocks for the nonce scan.
//
// FIPS 180-4 section 6.2.2 compression, written for CDNA4's 32-bit VALU:
//   rotr      -> v_alignbit_b32 (funnel shift of x:x)
//   Ch / Maj  -> one v_bitop3_b32 each (truth tables 0xCA / 0xE8)
//   xor3      -> one v_bitop3_b32 (0x96) for the three rotations of S0/S1/s0/s1
//   T1, a'    -> v_add3_u32 (selected by the compiler from the '+' chains)
// LLVM does not reliably form bitop3 from C inside the round's sums, so the
// three are the gfx950 builtin __builtin_amdgcn_bitop3_b32 (r01-r03e: one-line
// inline asm; the compiler then had to pad hazard s_nops after the opaque asm
// -- 57 per nonce in the MODE 7 loop -- and never hoisted it, which is why
// fast_thread hoists invariants by hand).  Every helper folds to a constant
// when its inputs are compile-time constants (`__builtin_constant_p`,
// resolved after unrolling/inlining), so zero words of the schedule cost nothing.
//
// The helpers are __host__ __device__ only so that tools/p1emu can run the
// exact per-thread scan logic on the host for layout tests; the host branch
// is plain C and is never linked into libp1hip.so's scan path.
//
// Reference semantics: bitcoin.Hash = SHA-256 of "msg nonce"
// (/root/reference/src/github.com/cmu440/bitcoin/hash.go:13-17); SHA-256
// itself is Go stdlib crypto/sha256 (not in the reference tree).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define P1_HD __host__ __device__ __forceinline__

namespace p1 {

P1_HD constexpr uint32_t k256(int t) {
  constexpr uint32_t k[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
  return k[t];
}

P1_HD constexpr uint32_t iv256(int i) {
  constexpr uint32_t v[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                             0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  return v[i];
}

#define P1_CONST3(a, b, c) (__builtin_constant_p(a) && __builtin_constant_p(b) && __builtin_constant_p(c))

P1_HD uint32_t rotr(uint32_t x, uint32_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (!__builtin_constant_p(x)) return __builtin_amdgcn_alignbit(x, x, n);
#endif
  return (x >> n) | (x << ((32u - n) & 31u));
}

// Funnel shift: low 32 bits of (hi:lo) >> s, s in [0, 31].
P1_HD uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(hi, lo, s);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> s);
#endif
}

P1_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (!P1_CONST3(a, b, c)) return (uint32_t)__builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#endif
  return a ^ b ^ c;
}

// Ch(e,f,g) = (e & f) ^ (~e & g).  (Plain C also becomes one bitop3 in
// isolation, but inside the T1 sum LLVM rewrites the disjoint terms into
// and + add and the loop grows by ~100 instructions per nonce -- measured.)
P1_HD uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (!P1_CONST3(e, f, g)) return (uint32_t)__builtin_amdgcn_bitop3_b32(e, f, g, 0xca);
#endif
  return (e & f) ^ (~e & g);
}

// Maj(a,b,c) = (a & b) ^ (a & c) ^ (b & c)
P1_HD uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (!P1_CONST3(a, b, c)) return (uint32_t)__builtin_amdgcn_bitop3_b32(a, b, c, 0xe8);
#endif
  return (a & b) ^ (a & c) ^ (b & c);
}

// Two-input add.  Kept as a named helper: on gfx950 v_add3_u32 is a half-rate
// op (tools/valu_peak), as is every other 3-operand VOP3 integer op except
// v_bitop3_b32, but forcing plain v_add_u32 pairs costs the same issue cycles
// and makes the compiler pad with s_nop (measured), so the
// compiler's add3 fusion is left on.
P1_HD uint32_t add2(uint32_t a, uint32_t b) { return a + b; }

P1_HD uint32_t bsig0(uint32_t a) { return xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)); }
P1_HD uint32_t bsig1(uint32_t e) { return xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)); }
P1_HD uint32_t ssig0(uint32_t x) { return xor3(rotr(x, 7), rotr(x, 18), x >> 3); }
P1_HD uint32_t ssig1(uint32_t x) { return xor3(rotr(x, 17), rotr(x, 19), x >> 10); }

// Scalar (wave-uniform) forms of the message-schedule sigmas: SALU shifts,
// so a word that is the same in every lane never occupies the VALU.
P1_HD uint32_t ssig_s(uint32_t x, int r1, int r2, int sh) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t a, b, c;
  asm("s_lshr_b32 %0, %3, %4\n\t"
      "s_lshl_b32 %1, %3, %5\n\t"
      "s_or_b32 %0, %0, %1\n\t"
      "s_lshr_b32 %1, %3, %6\n\t"
      "s_lshl_b32 %2, %3, %7\n\t"
      "s_or_b32 %1, %1, %2\n\t"
      "s_xor_b32 %0, %0, %1\n\t"
      "s_lshr_b32 %1, %3, %8\n\t"
      "s_xor_b32 %0, %0, %1"
      : "=&s"(a), "=&s"(b), "=&s"(c)
      : "s"(x), "i"(r1), "i"(32 - r1), "i"(r2), "i"(32 - r2), "i"(sh)
      : "scc");
  return a;
#else
  return ((x >> r1) | (x << (32 - r1))) ^ ((x >> r2) | (x << (32 - r2))) ^ (x >> sh);
#endif
}
P1_HD uint32_t ssig0_s(uint32_t x) { return ssig_s(x, 7, 18, 3); }
P1_HD uint32_t ssig1_s(uint32_t x) { return ssig_s(x, 17, 19, 10); }

// Working variables a..h of one compression.
struct State {
  uint32_t v[8];
};

// One round with kw = K[t] + W[t] (either may be a compile-time constant).
P1_HD void sha_round(State& s, uint32_t kw) {
  const uint32_t a = s.v[0], b = s.v[1], c = s.v[2], d = s.v[3];
  const uint32_t e = s.v[4], f = s.v[5], g = s.v[6], h = s.v[7];
  const uint32_t t1 = add2(add2(add2(h, kw), bsig1(e)), ch(e, f, g));
  const uint32_t t2 = add2(bsig0(a), maj(a, b, c));
  s.v[7] = g; s.v[6] = f; s.v[5] = e; s.v[4] = add2(d, t1);
  s.v[3] = c; s.v[2] = b; s.v[1] = a; s.v[0] = add2(t1, t2);
}

// Message-schedule word t >= 16 of a 64-entry array (unrolled callers only).
P1_HD uint32_t sched(const uint32_t* w, int t) {
  return add2(add2(add2(ssig1(w[t - 2]), w[t - 7]), ssig0(w[t - 15])), w[t - 16]);
}

// Full compression of the block in w[0..15] chained into cv[8];
// w[16..63] is scratch for the schedule.
P1_HD void compress_full(uint32_t cv[8], uint32_t w[64]) {
#pragma unroll
  for (int t = 16; t < 64; ++t) w[t] = sched(w, t);
  State s;
#pragma unroll
  for (int i = 0; i < 8; ++i) s.v[i] = cv[i];
#pragma unroll
  for (int t = 0; t < 64; ++t) sha_round(s, k256(t) + w[t]);
#pragma unroll
  for (int i = 0; i < 8; ++i) cv[i] += s.v[i];
}

}  // namespace p1
