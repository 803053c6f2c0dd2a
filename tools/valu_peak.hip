// valu_peak -- micro-benchmark of the gfx950 integer VALU rate for the
// instructions the SHA-256 rounds are made of (v_alignbit_b32, v_bitop3_b32,
// v_add3_u32, v_add_u32).  Measures lane-ops/s at several occupancies so the
// roofline peak used by bench.py is a measurement, not an assumption.
//
// usage: valu_peak            -> one JSON line per (instruction, waves/SIMD)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int kIters = 4096;
constexpr int kChains = 8;   // independent dependency chains per lane
constexpr int kPerIter = 4;  // instructions per chain per iteration

#define P1_BODY4(I) asm volatile(I "\n\t" I "\n\t" I "\n\t" I : "+v"(r[c]) : "v"(s1), "v"(s2))

template <int OP>
__global__ __launch_bounds__(256) void k_valu(uint32_t* out, uint32_t seed) {
  uint32_t r[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) r[c] = seed * (threadIdx.x + 1) + c;
  const uint32_t s1 = seed ^ 0x9e3779b9u, s2 = (seed + 7u) & 31u;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      if (OP == 0) P1_BODY4("v_alignbit_b32 %0, %0, %0, 7");
      else if (OP == 1) P1_BODY4("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96");
      else if (OP == 2) P1_BODY4("v_add3_u32 %0, %0, %1, %2");
      else if (OP == 3) P1_BODY4("v_add_u32_e32 %0, %0, %1");
      else if (OP == 4) P1_BODY4("v_xor_b32_e32 %0, %0, %1");
      else if (OP == 5) P1_BODY4("v_lshrrev_b32_e32 %0, 7, %0");
      else if (OP == 6) P1_BODY4("v_lshl_or_b32 %0, %0, 7, %1");
      else if (OP == 7) P1_BODY4("v_alignbyte_b32 %0, %0, %1, 1");
      else if (OP == 8) P1_BODY4("v_perm_b32 %0, %0, %1, %2");
      else if (OP == 9) P1_BODY4("v_xad_u32 %0, %0, %1, %2");
      else if (OP == 10) P1_BODY4("v_or3_b32 %0, %0, %1, %2");
      else if (OP == 11) P1_BODY4("v_lshl_add_u32 %0, %0, 3, %1");
      else if (OP == 12) P1_BODY4("v_add_lshl_u32 %0, %0, %1, 3");
      else if (OP == 13) P1_BODY4("v_and_or_b32 %0, %0, %1, %2");
      else if (OP == 14) P1_BODY4("v_bfi_b32 %0, %0, %1, %2");
      else if (OP == 15) P1_BODY4("v_add_u32_e64 %0, %0, %1");
      else if (OP == 16) P1_BODY4("v_lshrrev_b32_e64 %0, %2, %0");
      else if (OP == 17) P1_BODY4("v_alignbit_b32 %0, %0, %1, %2");
      else if (OP == 18) P1_BODY4("v_pk_add_u16 %0, %0, %1");
      else if (OP == 19) P1_BODY4("v_bfe_u32 %0, %0, 3, 20");
      else if (OP == 20) P1_BODY4("v_mad_u32_u24 %0, %0, %1, %2");
      else if (OP == 21) P1_BODY4("v_cndmask_b32_e64 %0, %0, %1, s[0:1]");
      else if (OP == 22) P1_BODY4("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca");
      else if (OP == 23) P1_BODY4("v_bitop3_b16 %0, %0, %1, %2 bitop3:0x96");
      else if (OP == 24) P1_BODY4("v_mov_b32_e32 %0, %1");
      else if (OP == 26) {  // 64-bit shift of a register pair (r, r): low word = rotr
        uint64_t v = ((uint64_t)r[c] << 32) | r[c];
        asm volatile("v_lshrrev_b64 %0, 7, %0\n\tv_lshrrev_b64 %0, 9, %0\n\tv_lshrrev_b64 %0, 3, %0\n\tv_lshrrev_b64 %0, 5, %0"
                     : "+v"(v));
        r[c] = (uint32_t)v ^ (uint32_t)(v >> 32);
      }
      else if (OP == 27) P1_BODY4("v_add_u32_e32 %0, 0x428a2f98, %0");
      else if (OP == 25) {  // half alignbit, half bitop3 interleaved
        asm volatile("v_alignbit_b32 %0, %0, %0, 7\n\tv_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n\t"
                     "v_alignbit_b32 %0, %0, %0, 9\n\tv_bitop3_b32 %0, %0, %1, %2 bitop3:0xca"
                     : "+v"(r[c]) : "v"(s1), "v"(s2));
      }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) acc ^= r[c];
  if (acc == 0x12345678u) out[0] = acc;  // keep the chains live
}

template <int OP>
static int run(const char* name, int cus) {
  uint32_t* d;
  CHK(hipMalloc(&d, 4));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  for (int wps : {2, 8}) {
    // blocks of 256 threads = 4 waves = one wave per SIMD; wps blocks per CU
    const int blocks = cus * wps;  // one round: wps waves on every SIMD
    hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a));
    const int reps = 3;
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(256), 0, 0, d, 3u);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    const double ops = (double)reps * blocks * 256.0 * kIters * kChains * kPerIter;
    printf("{\"instr\": \"%s\", \"blocks_per_cu_wave_slots\": %d, \"lane_ops_per_s\": %.4e, \"per_cu_per_clk_at_2.4GHz\": %.2f}\n",
           name, wps, ops / (ms * 1e-3), ops / (ms * 1e-3) / cus / 2.4e9);
  }
  CHK(hipFree(d));
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  int cus = p.multiProcessorCount;
#define RUN(I, N) if (run<I>(N, cus)) return 1
  RUN(0, "v_alignbit_b32 (x,x,imm)"); RUN(17, "v_alignbit_b32 (x,y,vgpr)"); RUN(7, "v_alignbyte_b32");
  RUN(1, "v_bitop3_b32 0x96"); RUN(22, "v_bitop3_b32 0xca"); RUN(23, "v_bitop3_b16");
  RUN(2, "v_add3_u32"); RUN(3, "v_add_u32_e32"); RUN(15, "v_add_u32_e64"); RUN(4, "v_xor_b32_e32");
  RUN(5, "v_lshrrev_b32_e32"); RUN(16, "v_lshrrev_b32_e64"); RUN(6, "v_lshl_or_b32"); RUN(8, "v_perm_b32");
  RUN(9, "v_xad_u32"); RUN(10, "v_or3_b32"); RUN(11, "v_lshl_add_u32"); RUN(12, "v_add_lshl_u32");
  RUN(13, "v_and_or_b32"); RUN(14, "v_bfi_b32"); RUN(18, "v_pk_add_u16"); RUN(19, "v_bfe_u32");
  RUN(20, "v_mad_u32_u24"); RUN(21, "v_cndmask_b32_e64"); RUN(24, "v_mov_b32"); RUN(25, "alignbit/bitop3 mix");
  RUN(26, "v_lshrrev_b64 (+2 VALU per 4)"); RUN(27, "v_add_u32_e32 literal");
#undef RUN
  return 0;
}
