// queue_ctl.cpp -- TEST PROGRAM (tests/test_gpu_paths.py::test_one_hardware_queue_per_process).
//
// Counts what the r02i configs[4] hang was blamed on: hardware queues per
// process.  `queue_ctl` scans through libp1hip.so only (the production
// shape: every device operation on the library's one stream).
// `queue_ctl nullstream` additionally makes ONE synchronous null-stream call
// (hipMemset), the pattern the library used to have at init -- the control
// that shows such a call costs the process a second hardware queue.  The test
// counts distinct HWq in the HIP runtime's own log (AMD_LOG_LEVEL=3).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include "../include/p1hip.h"

int main(int argc, char** argv) {
  const bool nullstream = argc > 1 && !strcmp(argv[1], "nullstream");
  int got = 0;
  if (p1hip_init(1, &got) != 0) {
    fprintf(stderr, "p1hip_init: %s\n", p1hip_last_error());
    return 2;
  }
  uint64_t h = 0, n = 0;
  if (p1hip_scan((const uint8_t*)"bradfitz", 8, 0, 99999999, &h, &n) != 0) return 3;
  if (nullstream) {
    void* p = nullptr;
    if (hipMalloc(&p, 4) != hipSuccess || hipMemset(p, 0, 4) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
      return 4;
    (void)hipFree(p);
  }
  if (p1hip_scan((const uint8_t*)"bradfitz", 8, 0, 99999999, &h, &n) != 0) return 5;
  printf("%llu %llu\n", (unsigned long long)h, (unsigned long long)n);
  p1hip_shutdown();
  return 0;
}
