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

template <int OP>
__global__ __launch_bounds__(256) void k_valu(uint32_t* out, uint32_t seed) {
  uint32_t r[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) r[c] = seed * (threadIdx.x + 1) + c;
  const uint32_t s1 = seed ^ 0x9e3779b9u, s2 = seed + 7u;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      if (OP == 0) {
        asm volatile(
            "v_alignbit_b32 %0, %0, %0, 7\n\t"
            "v_alignbit_b32 %0, %0, %0, 13\n\t"
            "v_alignbit_b32 %0, %0, %0, 5\n\t"
            "v_alignbit_b32 %0, %0, %0, 11"
            : "+v"(r[c]));
      } else if (OP == 1) {
        asm volatile(
            "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n\t"
            "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca\n\t"
            "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8\n\t"
            "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96"
            : "+v"(r[c]) : "v"(s1), "v"(s2));
      } else if (OP == 2) {
        asm volatile(
            "v_add3_u32 %0, %0, %1, %2\n\t"
            "v_add3_u32 %0, %0, %1, %2\n\t"
            "v_add3_u32 %0, %0, %1, %2\n\t"
            "v_add3_u32 %0, %0, %1, %2"
            : "+v"(r[c]) : "v"(s1), "v"(s2));
      } else {
        asm volatile(
            "v_add_u32_e32 %0, %0, %1\n\t"
            "v_xor_b32_e32 %0, %0, %2\n\t"
            "v_add_u32_e32 %0, %0, %1\n\t"
            "v_xor_b32_e32 %0, %0, %2"
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
  for (int wps : {1, 2, 4, 8}) {
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
  if (run<0>("v_alignbit_b32", cus)) return 1;
  if (run<1>("v_bitop3_b32", cus)) return 1;
  if (run<2>("v_add3_u32", cus)) return 1;
  if (run<3>("v_add_u32+v_xor_b32", cus)) return 1;
  return 0;
}
