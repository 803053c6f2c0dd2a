/* INTEGRATION.md's Go binding gpu.PlanShards, replayed in C through the C
 * ABI it binds: n <= 0 hands the library NULL outputs
 * and returns the library's own rejection; n >= 1 passes two caller-owned
 * arrays of n entries.  Host only: p1hip_plan_shards needs no device, so
 * this runs in the CPU suite (tests/test_capi_c.py).
 *
 *   capi_plan_shards <msg> <lower> <upper> <n>
 * prints "rc <rc> <message>" for a rejection, otherwise "ok" and one line
 * "<first> <last> <ok>" per shard (ok = 0 for an empty shard, as the
 * binding's ok[i] = f[i] <= l[i]); exit 0 unless the call broke a rule
 * checked here (shards in order, contiguous, covering [lower, upper]). */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "p1hip.h"

int main(int argc, char **argv) {
  if (argc != 5) return 2;
  const char *msg = argv[1];
  const size_t len = strlen(msg);
  const uint64_t lower = strtoull(argv[2], NULL, 10), upper = strtoull(argv[3], NULL, 10);
  const int n = atoi(argv[4]);
  if (p1hip_abi_version() != P1HIP_ABI_VERSION) {
    printf("abi mismatch\n");
    return 1;
  }
  const uint8_t *p = len ? (const uint8_t *)msg : NULL; /* the binding's &b[0] or nil */
  if (n <= 0) {
    /* the binding: no &f[0] to take, the library rejects the call */
    const int rc = p1hip_plan_shards(p, len, lower, upper, n, NULL, NULL);
    printf("rc %d %s\n", rc, p1hip_last_error());
    return rc == P1HIP_ERR_ARGS ? 0 : 1;
  }
  uint64_t *f = calloc((size_t)n, sizeof *f), *l = calloc((size_t)n, sizeof *l);
  if (!f || !l) return 1;
  const int rc = p1hip_plan_shards(p, len, lower, upper, n, f, l);
  if (rc != P1HIP_OK) {
    printf("rc %d %s\n", rc, p1hip_last_error());
    return 1;
  }
  printf("ok\n");
  int bad = 0;
  uint64_t next = lower; /* the first nonce the next non-empty shard must start at */
  int seen = 0;
  for (int i = 0; i < n; ++i) {
    const int ok = f[i] <= l[i];
    printf("%" PRIu64 " %" PRIu64 " %d\n", f[i], l[i], ok);
    if (!ok) continue;
    if (f[i] != next || l[i] > upper) bad = 1;
    next = l[i] + 1;
    seen = 1;
    if (l[i] == upper) next = 0; /* done: any later non-empty shard is an error */
  }
  if (lower <= upper && (!seen || next != 0)) bad = 1;
  free(f);
  free(l);
  return bad;
}
