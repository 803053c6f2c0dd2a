/*
 * p1hip.h -- C ABI of libp1hip.so, the MI355X (gfx950) drop-in for the
 * bitcoin miner's nonce scan.
 *
 * Reference seam (paths relative to /root/reference, SRC = src/github.com/cmu440):
 *   SRC/bitcoin/miner/miner.go:56-63   the loop this library replaces:
 *       var min, minIndex uint64 = math.MaxUint64, 0
 *       for i := req.Lower; i <= req.Upper; i++ {
 *           res := bitcoin.Hash(req.Data, i)
 *           if res < min { min = res; minIndex = i }
 *       }
 *   SRC/bitcoin/hash.go:13-17          bitcoin.Hash(msg, nonce) =
 *       BigEndian.Uint64(SHA-256(fmt.Sprintf("%s %d", msg, nonce))[0:8])
 *   SRC/bitcoin/message.go:18-44       Request{Data, Lower, Upper} in,
 *                                      Result{Hash, Nonce} out.
 * The reference has no FFI of its own; these are the entry points a cgo
 * bridge in the miner binds (INTEGRATION.md shows the binding).
 *
 * Plain C: no HIP/torch types, caller-owned buffers, no allocation crosses
 * the boundary.  `msg` is only borrowed for the duration of a call (cgo's
 * pointer-passing rule).  All calls are synchronous and serialised
 * internally; every call may be made from any host thread.
 *
 * Return codes: 0 ok; negative values are errors (details in
 * p1hip_last_error(), a per-thread string).
 */
#ifndef P1HIP_H
#define P1HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define P1HIP_OK 0
#define P1HIP_ERR_NO_DEVICE (-1) /* no gfx950 device visible / bad ordinal      */
#define P1HIP_ERR_HIP (-2)       /* HIP runtime error, or a host-side failure
                                    (allocation, thread creation): no C++
                                    exception ever crosses this ABI            */
#define P1HIP_ERR_RCCL (-3)      /* RCCL error (multi-device all-gather)        */
#define P1HIP_ERR_ARGS (-4)      /* msg==NULL with msg_len>0, msg_len too large */

/* Longest message accepted (bytes).  Keeps the SHA-256 bit length in one
 * 32-bit word; the reference's LSP frames cap Data at ~1.3 KB anyway
 * (SRC/lsp/common.go:7, 2000-byte receive buffers). */
#define P1HIP_MAX_MSG_LEN ((size_t)1 << 28)

/* Open `want_devices` devices (<= 0: every visible device), create one HIP
 * stream per device and, when more than one device is used, one RCCL
 * communicator per device (ncclCommInitAll).  Idempotent: a second call with
 * the same count is a no-op; a different count re-initialises. */
int p1hip_init(int want_devices, int *got_devices);

/* Same, but with an explicit list of device ordinals (e.g. {LOCAL_RANK} for
 * a one-process-per-GPU miner). */
int p1hip_init_devices(const int *ordinals, int n);

/* The drop-in for miner.go:56-63.  Scans [lower, upper] INCLUSIVE and
 * returns the minimum bitcoin.Hash(msg, i) and its nonce; ties go to the
 * lowest nonce (strict '<' at miner.go:59).  lower > upper returns
 * (UINT64_MAX, 0) with rc 0, exactly like the reference loop.  If every hash
 * in the range equals UINT64_MAX the nonce is 0 (identity of miner.go:56).
 * Documented divergence: upper == UINT64_MAX is scanned inclusively and the
 * call returns; the Go loop wraps (i++) and never terminates.
 * With several devices the range is split contiguously across them
 * (p1hip_plan_shards) and the 16-byte per-device partials are combined by an
 * RCCL all-gather + host min.
 * Lazily calls p1hip_init(0, NULL) if nothing is initialised. */
int p1hip_scan(const uint8_t *msg, size_t msg_len, uint64_t lower, uint64_t upper,
               uint64_t *out_hash, uint64_t *out_nonce);

/* The contiguous split p1hip_scan uses across devices, for callers that
 * shard themselves (one process per GPU, or a server handing miners pieces
 * of one request, server.go:119-140): [lower, upper] (inclusive) into n >= 1
 * shards of near-equal predicted GPU time, in order; shard i is
 * [first[i], last[i]], and first[i] > last[i] marks an empty shard.  Host
 * only (no device needed).  Kernel variants differ in cost per nonce by
 * decade (digit count), so equal-count shards over different decades would
 * finish at different times.  Contiguous shards keep the lexicographic min
 * of the shard results equal to the serial first-minimum of miner.go:56-63.
 * lower > upper gives n empty shards. */
int p1hip_plan_shards(const uint8_t *msg, size_t msg_len, uint64_t lower, uint64_t upper, int n,
                      uint64_t *first, uint64_t *last);

/* bitcoin.Hash(msg, nonce) (hash.go:13-17), computed on the GPU as the
 * one-nonce scan [nonce, nonce]. */
int p1hip_hash(const uint8_t *msg, size_t msg_len, uint64_t nonce, uint64_t *out_hash);

/* Test hook for the device-side argmin: reduces n crafted (hash, nonce)
 * pairs with the scan's own wave/LDS/grid reduction kernels and applies the
 * same result rules as p1hip_scan (lexicographic (hash, nonce) minimum,
 * nonce 0 when the minimum hash is UINT64_MAX, (UINT64_MAX, 0) when n == 0). */
int p1hip_reduce_pairs(const uint64_t *hashes, const uint64_t *nonces, size_t n,
                       uint64_t *out_hash, uint64_t *out_nonce);

/* Kernel-level accounting.  One p1hip_scan = one (rarely several) launch of
 * the scan kernel k_scan per device, covering every decade of the range; a
 * share of at most 2^16 nonces is one launch of k_scan_small instead (plan in
 * the kernel arguments, reduce fused into the last workgroup, result written
 * to pinned host memory). */
typedef struct {
  uint64_t scans;            /* p1hip_scan calls since reset                      */
  uint64_t fast_launches;    /* fast segments (one thread per 10^k nonces)        */
  uint64_t fast_nonces;      /* nonces hashed by fast segments                    */
  uint64_t fast_alg_ops;     /* algorithmic int32 ops: 1384 * B_tail per nonce    */
  uint64_t generic_launches; /* generic segments (one thread per nonce)           */
  uint64_t generic_nonces;   /* nonces hashed by generic segments                 */
  double scan_wall_ms;       /* host wall time inside p1hip_scan                  */
  uint64_t scan_launches;    /* launches of k_scan                                */
  uint64_t scan_nonces;      /* nonces hashed by those launches                   */
  uint64_t scan_alg_ops;     /* their algorithmic int32 ops (1384 * B_tail each)  */
  double scan_kernel_ms;     /* sum of HIP-event durations of those launches
                                (recorded only while profiling is on)            */
  uint64_t small_scans;      /* device scans that took the one-launch small path
                                (<= 2^16 nonces: k_scan_small, fused reduce)     */
  uint64_t table_replans;    /* device shares re-planned without MODE 5 because a
                                K+W table could not be had (before any launch)   */
} p1hip_stats_t;

/* Per-device accounting since p1hip_reset_stats (device `index` in the order
 * p1hip_init / p1hip_init_devices opened them), so a multi-device scan can
 * explain its own scaling: which shard each device took, how long its
 * kernels ran, how long its host thread spent in the scan phase and in the
 * all-gather phase. */
typedef struct {
  int32_t ordinal;           /* HIP device ordinal                                */
  int32_t active;            /* its shard of the last scan was non-empty          */
  uint64_t shard_first;      /* last scan's shard [first, last] (first > last:    */
  uint64_t shard_last;       /*   empty)                                          */
  uint64_t scans;            /* p1hip_scan calls this device took part in         */
  uint64_t scan_launches;    /* k_scan / k_scan_small launches                    */
  uint64_t scan_nonces;      /* nonces they hashed                                */
  uint64_t scan_alg_ops;     /* their algorithmic int32 ops (1384 * B_tail each)  */
  double scan_kernel_ms;     /* HIP-event kernel time (while profiling is on)     */
  double phase1_ms;          /* host wall ms: plan + launches + stream sync       */
  double gather_ms;          /* host wall ms in the RCCL all-gather phase (0 for  */
                             /*   one device / host combine)                      */
} p1hip_device_stats_t;

int p1hip_get_device_stats(int index, p1hip_device_stats_t *out);

/* Record HIP events (on the library's own stream) around every fast-kernel
 * launch.  Off by default: the events cost a little host time per launch. */
int p1hip_set_profiling(int on);
int p1hip_get_stats(p1hip_stats_t *out);
void p1hip_reset_stats(void);

/* Number of devices currently in use (0 before init). */
int p1hip_device_count(void);

/* Identity of device `index` (as for p1hip_get_device_stats), so a record of
 * an N-GPU run can show that N distinct GPUs took part. */
typedef struct {
  int32_t ordinal;           /* HIP device ordinal                                */
  int32_t cu_count;          /* compute units                                     */
  int32_t clock_khz;         /* peak engine clock                                 */
  int32_t reserved;
  uint64_t hbm_bytes;        /* device memory                                     */
  char pci_bus_id[32];       /* "dddd:bb:dd.f" (hipDeviceGetPCIBusId)             */
  char arch[32];             /* gcnArchName, e.g. "gfx950:sramecc+:xnack-"        */
  unsigned char uuid[16];    /* hipDeviceProp_t.uuid                              */
} p1hip_device_info_t;

int p1hip_device_info(int index, p1hip_device_info_t *out);

/* The RCCL communicator of device `index` (as for p1hip_get_device_stats),
 * as RCCL itself reports it: *nranks = ncclCommCount, *rank =
 * ncclCommUserRank.  A device without a communicator (one device, or the
 * P1HIP_NO_RCCL host combine) gives *nranks = 0, *rank = -1 with rc 0.  With
 * N devices opened by p1hip_init(N) every device reports N ranks and the
 * ranks are 0..N-1 once each: the all-gather inside p1hip_scan spans them
 * all (bench.py refuses to time an N-GPU run for which this does not hold). */
int p1hip_comm_info(int index, int *nranks, int *rank);

/* Layout version of the structs above.  A consumer compiled against this
 * header checks p1hip_abi_version() == P1HIP_ABI_VERSION before reading any
 * p1hip_*_t the library fills in.  History: 4 = p1hip 0.4 (fast_kernel_ms
 * removed from p1hip_stats_t, so the fields after fast_alg_ops moved); 5 =
 * p1hip 0.5 (p1hip_comm_info and this query added; the structs are as in 4). */
#define P1HIP_ABI_VERSION 5
int p1hip_abi_version(void);

const char *p1hip_last_error(void);
const char *p1hip_version(void);

/* Test-only knobs in force for this process.  The library honours its
 * P1HIP_* test knobs (occupancy floor, injected failures, table and launch
 * caps, combine mode ...) only while the master switch P1HIP_TEST_KNOBS=1 is
 * set in the environment; otherwise they are ignored and this returns "".
 * With the switch set it returns "P1HIP_TEST_KNOBS=1" followed by
 * ";NAME=value" for every knob that is set; knobs read at init that the open
 * devices still run with are listed too ("NAME=(init: value)"), even if the
 * environment changed since.  bench.py refuses to time a run for which this
 * is not "".  The string is per thread and valid until the next call from
 * that thread. */
const char *p1hip_test_knobs(void);

/* Release streams, buffers and communicators.  Safe to call twice. */
void p1hip_shutdown(void);

#ifdef __cplusplus
}
#endif
#endif /* P1HIP_H */
