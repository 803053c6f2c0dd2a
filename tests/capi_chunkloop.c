/* The miner change of INTEGRATION.md section 2, replayed in C through the C
 * ABI the cgo bridge binds: a server job [lower, upper] goes to the GPU in
 * chunks (one p1hip_scan per chunk, strict '<' across chunks); a chunk whose
 * call fails (rc != 0) is scanned by the CPU loop of miner.go:56-63.  Here
 * that CPU loop is the oracle restatement (test code may link the checker);
 * the product library has no CPU path.
 *
 *   capi_chunkloop <msg> <lower> <upper> <chunk> [fail-every-k]
 * prints "Result <hash> <nonce> gpu_chunks=<g> cpu_chunks=<c>".  With
 * fail-every-k > 0 every k-th chunk is issued with an invalid argument
 * (msg == NULL with msg_len > 0 -> P1HIP_ERR_ARGS) to take the rc != 0 branch.
 * Built and run by tests/test_capi_c.py. */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "p1hip.h"

/* oracle/libp1oracle.so: bitcoin.Hash (hash.go:13-17) on the CPU */
uint64_t p1o_hash(const uint8_t *msg, size_t len, uint64_t nonce);

int main(int argc, char **argv) {
  if (argc < 5) return 2;
  const char *msg = argv[1];
  const size_t len = strlen(msg);
  const uint64_t lower = strtoull(argv[2], NULL, 10), upper = strtoull(argv[3], NULL, 10);
  const uint64_t chunk = strtoull(argv[4], NULL, 10);
  const int fail_every = argc > 5 ? atoi(argv[5]) : 0;
  if (chunk == 0) return 2;
  uint64_t min = UINT64_MAX, min_index = 0; /* miner.go:56 */
  int gpu_chunks = 0, cpu_chunks = 0, k = 0;
  for (uint64_t lo = lower; lo <= upper;) {
    uint64_t hi = upper;
    if (hi - lo >= chunk) hi = lo + chunk - 1;
    uint64_t h = 0, n = 0;
    const int inject = fail_every > 0 && (++k % fail_every) == 0;
    const int rc = inject ? p1hip_scan(NULL, 1, lo, hi, &h, &n)
                          : p1hip_scan((const uint8_t *)msg, len, lo, hi, &h, &n);
    if (rc == P1HIP_ERR_NO_DEVICE) {
      printf("nodevice %s\n", p1hip_last_error());
      return 0;
    }
    if (rc != P1HIP_OK) {
      if (!inject || rc != P1HIP_ERR_ARGS) {
        printf("unexpected rc %d: %s\n", rc, p1hip_last_error());
        return 1;
      }
      /* the reference's own loop for this chunk (err != nil) */
      for (uint64_t i = lo;; ++i) {
        const uint64_t r = p1o_hash((const uint8_t *)msg, len, i);
        if (r < min) {
          min = r;
          min_index = i;
        }
        if (i == hi) break;
      }
      ++cpu_chunks;
    } else {
      if (h < min) { /* strict '<' across chunks: the first minimum wins */
        min = h;
        min_index = n;
      }
      ++gpu_chunks;
    }
    if (hi == upper) break;
    lo = hi + 1;
  }
  printf("Result %" PRIu64 " %" PRIu64 " gpu_chunks=%d cpu_chunks=%d\n", min, min_index, gpu_chunks, cpu_chunks);
  p1hip_shutdown();
  return 0;
}
