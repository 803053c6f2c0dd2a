// XCD balance probe (measurement program, not product).
//
// Question (round 6): the clock probe around bench.py's timed steps reads a
// different average shader clock on each XCD (r06a: 2.27-2.34 GHz).  k_scan
// gives every workgroup the same work and the hardware hands workgroups to
// the XCDs in a fixed order, so if the XCDs really run at different clocks
// under load, the slowest one decides when a launch ends.  This program
// measures, under a dense integer-VALU load of the kernel's own mix
// (alignbit / add3 / bitop3 chains, 4 waves per SIMD):
//   * which XCD runs workgroup i (is it i mod 8?),
//   * each XCD's shader clock while its workgroups are running
//     (delta s_memtime / delta s_memrealtime inside every workgroup),
//   * when each XCD's last workgroup ends, relative to the first start.
// Stamps go to a buffer of their own through vector stores.
//
// usage: xcd_probe [workgroups] [iterations]   -> one JSON line per run
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define HWREG_XCC_ID (20 | (0 << 6) | ((4 - 1) << 11))
#define CHK(x)                                                                     \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                     \
    }                                                                              \
  } while (0)

__device__ __forceinline__ unsigned rotr(unsigned x, unsigned s) { return __builtin_amdgcn_alignbit(x, x, s); }

// 128 VGPRs-worth of live state is not needed to load the SIMD; what matters
// is a dense VALU stream of both issue classes and 4 waves per SIMD, which
// __launch_bounds__(256, 1) plus the LDS request below enforce.
__global__ void __launch_bounds__(256) k_busy(unsigned long long* out, int iters, unsigned seed) {
  extern __shared__ unsigned lds[];
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned a = threadIdx.x * 0x9e3779b9u ^ seed, b = a * 3u + 1u, c = a ^ 0x6a09e667u, d = b + 0xbb67ae85u;
  unsigned e = a + 7u, f = b ^ 5u, g = c * 9u, h = d - 11u;
  for (int i = 0; i < iters; ++i) {
    unsigned s1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
    unsigned ch = (e & f) ^ (~e & g);
    unsigned t1 = h + s1 + ch + (unsigned)i;
    unsigned s0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
    unsigned mj = (a & b) ^ (a & c) ^ (b & c);
    h = g; g = f; f = e; e = d + t1;
    d = c; c = b; b = a; a = t1 + s0 + mj;
  }
  unsigned long long t1s = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  unsigned xcc = __builtin_amdgcn_s_getreg(HWREG_XCC_ID);
  if (threadIdx.x == 0) {
    unsigned long long* o = out + 6ull * blockIdx.x;
    o[0] = t0;
    o[1] = r0;
    o[2] = t1s;
    o[3] = r1;
    o[4] = xcc;
    o[5] = a ^ e;
  }
  if (a == 0x12345678u && e == 0x9abcdef0u) lds[threadIdx.x] = a;  // keep the chain live
}

int main(int argc, char** argv) {
  int nwg = argc > 1 ? atoi(argv[1]) : 65536;
  int iters = argc > 2 ? atoi(argv[2]) : 4000;
  int runs = argc > 3 ? atoi(argv[3]) : 3;
  if (nwg < 8 || nwg > (1 << 22) || iters < 1) return 1;
  unsigned long long* d = nullptr;
  size_t bytes = sizeof(unsigned long long) * 6 * (size_t)nwg;
  CHK(hipMalloc((void**)&d, bytes));
  std::vector<unsigned long long> h(6 * (size_t)nwg);
  // 40 KB of LDS per 256-thread workgroup: at most 4 workgroups per CU
  // (160 KB LDS), i.e. 4 waves per SIMD as k_scan runs
  const size_t lds = 40 * 1024;
  CHK(hipFuncSetAttribute((const void*)k_busy, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  for (int run = 0; run < runs; ++run) {
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_busy, dim3(nwg), dim3(256), lds, 0, d, iters, 0x1234u + run);
    CHK(hipGetLastError());
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    CHK(hipMemcpy(h.data(), d, bytes, hipMemcpyDeviceToHost));
    unsigned long long rmin = ~0ull;
    for (int i = 0; i < nwg; ++i) rmin = std::min(rmin, h[6 * i + 1]);
    double cyc[8] = {0}, wall[8] = {0}, last[8] = {0}, first[8];
    long cnt[8] = {0}, rr = 0, bad = 0;
    for (int x = 0; x < 8; ++x) first[x] = 1e30;
    for (int i = 0; i < nwg; ++i) {
      unsigned long long* o = &h[6 * i];
      int x = (int)o[4];
      if (x < 0 || x > 7) {
        bad++;
        continue;
      }
      cnt[x]++;
      rr += (x == i % 8);
      cyc[x] += (double)(o[2] - o[0]);
      wall[x] += (double)(o[3] - o[1]);
      last[x] = std::max(last[x], (double)(o[3] - rmin) / 1e5);  // ms (100 MHz counter)
      first[x] = std::min(first[x], (double)(o[1] - rmin) / 1e5);
    }
    printf("{\"run\": %d, \"workgroups\": %d, \"iters\": %d, \"kernel_ms\": %.3f, \"xcc_is_wg_mod_8\": %.4f, \"bad_xcc\": %ld, "
           "\"per_xcc\": [",
           run, nwg, iters, ms, (double)rr / nwg, bad);
    for (int x = 0; x < 8; ++x)
      printf("%s{\"xcc\": %d, \"workgroups\": %ld, \"busy_clock_GHz\": %.4f, \"first_start_ms\": %.3f, \"last_end_ms\": %.3f}",
             x ? ", " : "", x, cnt[x], wall[x] > 0 ? cyc[x] / wall[x] * 0.1 : 0.0, first[x], last[x]);
    printf("]}\n");
    fflush(stdout);
    CHK(hipEventDestroy(e0));
    CHK(hipEventDestroy(e1));
  }
  CHK(hipFree(d));
  return 0;
}
