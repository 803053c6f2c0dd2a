// wcal -- calibration of rocprofv3's WRITE_SIZE / FETCH_SIZE for the access
// pattern of k_scan's partials (MI355X_MICROARCH.md, HBM section: "Other
// access widths are uncalibrated: calibrate on a known byte count in your
// own access pattern before trusting an absolute").
//
// k_scan writes ONE 16-byte (hash, nonce) partial per workgroup of 256
// threads, from one lane, after the LDS reduction; k_reduce reads them back.
// Kernels here, each over G workgroups of 256 threads:
//   k_part16   lane 0 of each workgroup stores 16 B at out[blockIdx.x]
//              (k_scan's pattern; G x 16 B written)
//   k_stream16 every lane stores 16 B, coalesced (the guide's calibrated
//              pattern: WRITE_SIZE reads exactly; G x 256 x 16 B)
//   k_read16   lane 0 of each workgroup loads 16 B at in[blockIdx.x]
//              (k_reduce's reads, spread over workgroups; G x 16 B)
// usage: wcal [G]   (default 1,080,784 = configs[3]'s k_scan grid on one GPU)
// Profile each launch with rocprofv3 --pmc WRITE_SIZE (resp. FETCH_SIZE)
// --kernel-trace; the program prints the byte counts each kernel moves.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct Key { uint64_t h, n; };

__global__ __launch_bounds__(256) void k_part16(Key* out, uint64_t seed) {
  if (threadIdx.x == 0) out[blockIdx.x] = Key{seed ^ blockIdx.x, blockIdx.x};
}

__global__ __launch_bounds__(256) void k_stream16(Key* out, uint64_t seed) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  out[i] = Key{seed ^ i, i};
}

__global__ __launch_bounds__(256) void k_read16(const Key* in, Key* sink) {
  if (threadIdx.x == 0) {
    const Key k = in[blockIdx.x];
    if (k.h == 0x0123456789abcdefull) sink[0] = k;  // keep the load live
  }
}

int main(int argc, char** argv) {
  const uint32_t G = argc > 1 ? (uint32_t)strtoul(argv[1], nullptr, 10) : 1080784u;
  Key *part = nullptr, *stream = nullptr, *sink = nullptr;
  CHK(hipMalloc(&part, sizeof(Key) * (size_t)G));
  CHK(hipMalloc(&stream, sizeof(Key) * (size_t)G * 256));
  CHK(hipMalloc(&sink, sizeof(Key)));
  hipLaunchKernelGGL(k_part16, dim3(G), dim3(256), 0, 0, part, 1ull);
  hipLaunchKernelGGL(k_stream16, dim3(G), dim3(256), 0, 0, stream, 2ull);
  hipLaunchKernelGGL(k_read16, dim3(G), dim3(256), 0, 0, part, sink);
  CHK(hipDeviceSynchronize());
  printf("{\"workgroups\": %u, \"k_part16_bytes_written\": %zu, \"k_stream16_bytes_written\": %zu, "
         "\"k_read16_bytes_read\": %zu}\n",
         G, (size_t)G * 16, (size_t)G * 256 * 16, (size_t)G * 16);
  CHK(hipFree(part));
  CHK(hipFree(stream));
  CHK(hipFree(sink));
  return 0;
}
