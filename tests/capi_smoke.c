/* Plain-C client of include/p1hip.h: proves the header is C99 and that a C
 * (or cgo) caller links against libp1hip.so.  Prints "nodevice" on a host
 * without a GPU (rc -1, no CPU fallback), else checks the handout KAT and
 * the configs[0] answer.  Built and run by tests/test_capi_c.py. */
#include <inttypes.h>
#include <stdio.h>
#include <string.h>

#include "p1hip.h"

int main(void) {
  uint64_t h = 0, n = 0;
  const char *msg = "bradfitz";
  int rc = p1hip_scan((const uint8_t *)msg, strlen(msg), 0, 9999, &h, &n);
  if (rc == P1HIP_ERR_NO_DEVICE) {
    printf("nodevice %s\n", p1hip_last_error());
    return 0;
  }
  if (rc != P1HIP_OK) {
    printf("error %d %s\n", rc, p1hip_last_error());
    return 1;
  }
  printf("Result %" PRIu64 " %" PRIu64 "\n", h, n);
  if (h != 1419516646206828ull || n != 9898) return 2;
  if (p1hip_hash((const uint8_t *)"msg", 3, 1, &h) != 0 || h != 4754799531757243342ull) return 3;
  rc = p1hip_scan((const uint8_t *)msg, strlen(msg), 9, 3, &h, &n); /* lower > upper */
  if (rc != 0 || h != UINT64_MAX || n != 0) return 4;
  p1hip_shutdown();
  return 0;
}
