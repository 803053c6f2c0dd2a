// asan_teardown -- MEASUREMENT PROGRAM (not product): does a host program
// built with ROCm's AddressSanitizer abort at exit with the device-allocator
// CHECK "!dev_runtime_unloaded_" (sanitizer_allocator_device.h) when
// libp1hip.so is NOT involved at all?  (whose free
// trips it.)  Plain HIP runtime + RCCL calls only, each allocation freed
// before main returns, then a normal exit through the static destructors.
//
//   asan_teardown <mode>
//     none     hipGetDeviceCount only
//     malloc   hipSetDevice + hipMalloc/hipFree + hipHostMalloc/hipHostFree
//              + a stream, all released
//     rccl     malloc + ncclCommInitAll on one device + ncclCommDestroy
// Built with `make tools/asan_teardown` (host-side ASan, no device code).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <string.h>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const char* mode = argc > 1 ? argv[1] : "malloc";
  int n = 0;
  CK(hipGetDeviceCount(&n));
  printf("devices %d mode %s\n", n, mode);
  if (strcmp(mode, "none") != 0) {
    CK(hipSetDevice(0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    void *d = nullptr, *h = nullptr;
    CK(hipMalloc(&d, 1 << 20));
    CK(hipHostMalloc(&h, 1 << 16, hipHostMallocDefault));
    CK(hipMemsetAsync(d, 0, 1 << 20, s));
    CK(hipStreamSynchronize(s));
    if (strcmp(mode, "rccl") == 0) {
      ncclComm_t c;
      int dev = 0;
      if (ncclCommInitAll(&c, 1, &dev) != ncclSuccess) return 1;
      ncclCommDestroy(c);
    }
    CK(hipFree(d));
    CK(hipHostFree(h));
    CK(hipStreamDestroy(s));
  }
  printf("released, returning from main\n");
  return 0;
}
