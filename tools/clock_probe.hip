// Shader-clock probe for bench.py (measurement only, not part of the scan).
//
// One stamp = every workgroup of a tiny launch reads s_memtime (ticks at the
// shader clock, MI355X_MICROARCH.md "s_memtime tick vs SQ PMC units"), then
// s_memrealtime (the constant-rate wall counter), then s_memtime again, and
// the XCC it runs on.  Two stamps around bench.py's timed steps give the
// average shader clock of every XCD over them: delta memtime / delta
// memrealtime x the wall-counter rate (MI355X_MICROARCH.md "DVFS give-back"
// item 6).  The scan's code object is untouched; this kernel runs only
// before and after the timed region, on its own stream.
//
// C ABI (bench.py loads tools/libp1clock.so with ctypes):
//   int p1clk_stamp(int device, int nblocks, unsigned long long* out);
//     out[4*b + 0..3] = memtime before, memrealtime, memtime after, XCC id
//     of workgroup b; returns 0 or a hipError_t.
//   int p1clk_wall_rate_khz(int device);   hipDeviceAttributeWallClockRate
#include <hip/hip_runtime.h>

// hwreg(HW_REG_XCC_ID, offset 0, 4 bits): which of the 8 XCDs the wave is on
#define P1CLK_HWREG_XCC_ID (20 | (0 << 6) | ((4 - 1) << 11))

__global__ void __launch_bounds__(64) k_clock_stamp(unsigned long long* out) {
  if (threadIdx.x != 0) return;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r = __builtin_amdgcn_s_memrealtime();
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned xcc = __builtin_amdgcn_s_getreg(P1CLK_HWREG_XCC_ID);
  unsigned long long* o = out + 4ull * blockIdx.x;
  o[0] = t0;
  o[1] = r;
  o[2] = t1;
  o[3] = xcc;
}

extern "C" int p1clk_wall_rate_khz(int device) {
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess) return -1;
  return khz;
}

extern "C" int p1clk_stamp(int device, int nblocks, unsigned long long* out) {
  if (nblocks < 1 || nblocks > 4096 || !out) return (int)hipErrorInvalidValue;
  int prev = 0;
  hipError_t e = hipGetDevice(&prev);
  if (e != hipSuccess) return (int)e;
  if ((e = hipSetDevice(device)) != hipSuccess) return (int)e;
  unsigned long long* d = nullptr;
  hipStream_t s = nullptr;
  size_t bytes = sizeof(unsigned long long) * 4 * (size_t)nblocks;
  if ((e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) == hipSuccess &&
      (e = hipMalloc((void**)&d, bytes)) == hipSuccess) {
    hipLaunchKernelGGL(k_clock_stamp, dim3(nblocks), dim3(64), 0, s, d);
    if ((e = hipGetLastError()) == hipSuccess && (e = hipMemcpyAsync(out, d, bytes, hipMemcpyDeviceToHost, s)) == hipSuccess)
      e = hipStreamSynchronize(s);
  }
  if (d) (void)hipFree(d);
  if (s) (void)hipStreamDestroy(s);
  (void)hipSetDevice(prev);
  return (int)e;
}
