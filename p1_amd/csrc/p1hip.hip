// p1hip.hip -- libp1hip.so: host runtime (planning, launch orchestration,
// multi-device combine) and the C ABI declared in include/p1hip.h.
//
// Replaces the miner's scan loop /root/reference/src/github.com/cmu440/bitcoin/
// miner/miner.go:56-63 (see include/p1hip.h for the exact contract).
//
// Device pipeline of one p1hip_scan on one device (one HIP stream):
//   planner.hpp  -> list of pieces (fast: one thread per 10^k nonces;
//                   generic: one thread per nonce, for ragged edges)
//   k_scan       -> one launch, one segment per piece (p1hip_kernels.hip)
//   k_reduce     -> one workgroup folds all partials into the device result
// The kernels live in a gfx950 code object built from p1hip_kernels.hip via
// assembly + tools/isa_post.py (Makefile) and embedded in this library
// (p1hip_kernels_blob.S); each device loads it with hipModuleLoadData.
// Several devices: contiguous shards, one host thread per device, RCCL
// all-gather of the 16-byte results (ncclCommInitAll), host lexicographic min.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <exception>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/p1hip.h"
#include "planner.hpp"
#include "scan_abi.hpp"

// the embedded gfx950 code object (p1hip_kernels_blob.S)
extern "C" const unsigned char p1hip_kernels_co[];

using namespace p1;

static bool has_variant(int fv, int mode, bool trail) {
#define P1_CASE(FV, MODE, TR) \
  if (fv == FV && mode == MODE && trail == TR) return true;
#include "fast_variants.inc"
#undef P1_CASE
  return false;
}

// ----------------------------------------------------------------------------
// Runtime state
// ----------------------------------------------------------------------------
namespace {

thread_local std::string g_err;

int fail(int rc, const std::string& what) {
  g_err = what;
  return rc;
}

// Run an exported entry point's body; a host exception (std::bad_alloc from a
// caller-sized allocation, std::system_error from a thread) becomes rc -2
// with the message in p1hip_last_error() instead of crossing the C ABI.
template <typename Fn>
int guarded(Fn&& fn) {
  try {
    return fn();
  } catch (const std::exception& ex) {
    return fail(P1HIP_ERR_HIP, std::string("host: ") + ex.what());
  } catch (...) {
    return fail(P1HIP_ERR_HIP, "host: unknown exception");
  }
}

#define HIPCHK(expr)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return fail(P1HIP_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));       \
  } while (0)

#define NCCLCHK(expr)                                                                       \
  do {                                                                                      \
    ncclResult_t r_ = (expr);                                                               \
    if (r_ != ncclSuccess)                                                                  \
      return fail(P1HIP_ERR_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_));      \
  } while (0)

constexpr uint32_t kMaxSegs = 64;              // segments per launch
// Workgroups per launch: 2^22 x 256 threads stays below HIP's 2^32-thread
// grid limit and keeps configs[3] on one GPU (2^38 nonces, ~1.07M
// workgroups) in one launch, i.e. one grid drain per scan.
constexpr uint32_t kMaxLaunchBlocks = 1u << 22;

// P1HIP_SMALL_MAX_NONCES (tests only, read per scan): ranges of at most this
// many nonces take the one-launch small path (default kSmallMaxNonces; 0
// turns it off so small parity ranges exercise the fast kernel variants).
// Every P1HIP_* test knob is read through test_knob(): it is honoured only
// while the master switch P1HIP_TEST_KNOBS=1 is set (the test fixtures set
// it), so a stray knob in a production miner's environment changes nothing.
// p1hip_test_knobs() lists the knobs in force, for bench.py to refuse.
const char* const kTestKnobs[] = {
    "P1HIP_SMALL_MAX_NONCES", "P1HIP_MAX_LAUNCH_BLOCKS", "P1HIP_MAX_SCAN_SPAN", "P1HIP_KWTAB_MAX_BYTES",
    "P1HIP_NO_RCCL",          "P1HIP_FORCE_RCCL",        "P1HIP_MIN_FAST_THREADS", "P1HIP_TEST_FAIL_DEVICE",
    "P1HIP_NO_TABLE",         "P1HIP_NO_SPLIT",          "P1HIP_SCAN_GRID",
};

bool test_knobs_on() {
  const char* m = getenv("P1HIP_TEST_KNOBS");
  return m && m[0] == '1' && m[1] == 0;
}

const char* test_knob(const char* name) {
  if (!test_knobs_on()) return nullptr;
  const char* v = getenv(name);
  return v && *v ? v : nullptr;
}

uint64_t small_limit() {
  const char* v = test_knob("P1HIP_SMALL_MAX_NONCES");
  if (!v || !*v) return kSmallMaxNonces;
  const uint64_t n = strtoull(v, nullptr, 10);
  return n < kSmallMaxNonces ? n : kSmallMaxNonces;
}

// P1HIP_MAX_LAUNCH_BLOCKS (tests only, read per scan): a lower per-launch
// workgroup cap, so GPU tests run the multi-launch path on small ranges.  A
// piece larger than the cap gets a launch of its own (a piece is at most
// kMaxFastThreads / kBlock = 2^18 workgroups, far below HIP's grid limit).
uint64_t launch_block_limit() {
  const char* v = test_knob("P1HIP_MAX_LAUNCH_BLOCKS");
  const uint64_t n = v && *v ? strtoull(v, nullptr, 10) : 0;
  if (n == 0 || n >= kMaxLaunchBlocks) return kMaxLaunchBlocks;
  return n;
}

struct Dev {
  int ordinal = -1;
  hipStream_t stream = nullptr;
  Key* d_part = nullptr;
  size_t part_cap = 0;
  Key* d_res = nullptr;         // 1 Key
  Key* d_gather = nullptr;      // ndev Keys (multi-device)
  Key* h_res = nullptr;         // pinned, ndev Keys
  Segment* d_seg = nullptr;     // segment tables, kMaxSegs per launch slot
  Segment* h_seg = nullptr;     // pinned staging for the tables
  size_t seg_cap = 0;           // launch slots allocated
  ncclComm_t comm = nullptr;
  hipModule_t mod = nullptr;    // embedded code object, loaded on this device
  hipFunction_t f_scan = nullptr, f_reduce = nullptr, f_pairs = nullptr, f_small = nullptr, f_kwtable = nullptr;
  Key* d_small_part = nullptr;  // kSmallMaxBlocks partials of k_scan_small
  uint32_t* d_ticket = nullptr; // k_scan_small's last-workgroup counter (0 between scans)
  uint32_t* d_scan_ticket = nullptr;  // k_scan's work queue: [tiles handed out, workgroups done] (0 between launches)
  uint32_t scan_grid = 0;       // k_scan workgroups the device holds at once (occupancy x CUs)
  bool small_used = false;      // this scan ran k_scan_small (result already in h_res[0])
  std::vector<hipEvent_t> evs;  // profiling event pool (pairs)
  // MODE 5 K+W tables on this device, least recently used first (built by
  // k_kwtable; keyed by the block-1 template and k)
  struct KwTab {
    uint32_t w[16];
    int k;
    uint32_t* dptr;
    uint64_t used_in;  // run_range call that last used it (never evicted during it)
  };
  std::vector<KwTab> kwtabs;
  uint64_t range_id = 0;        // run_range calls on this device
  // per-scan accounting filled by run_range
  uint64_t fast_launches = 0, fast_nonces = 0, fast_ops = 0, gen_launches = 0, gen_nonces = 0;
  uint64_t scan_launches = 0, scan_nonces = 0, scan_ops = 0;
  double scan_ms = 0.0;
  uint64_t replans = 0;         // shares re-planned without MODE 5 (this scan)
  // since p1hip_reset_stats, for p1hip_get_device_stats
  p1hip_device_stats_t acc{};
};

struct Runtime {
  std::mutex mu;
  std::vector<Dev> devs;
  bool profiling = false;
  bool use_rccl = true;   // multi-device combine through ncclAllGather
  bool rccl_one = false;  // P1HIP_FORCE_RCCL=1: communicator even for one device
  // Test-only knobs, read from the environment at init (never set in
  // production; honoured only under P1HIP_TEST_KNOBS=1, see test_knob):
  //   P1HIP_MIN_FAST_THREADS  planner occupancy floor (1 keeps k = 3 on small
  //                           ranges so every k = 3 variant runs on the GPU)
  //   P1HIP_TEST_FAIL_DEVICE  device index whose scan phase reports a failure
  //                           (exercises the multi-device error path)
  //   P1HIP_MAX_LAUNCH_BLOCKS workgroups per k_scan launch (read per scan,
  //                           launch_block_limit)
  //   P1HIP_MAX_SCAN_SPAN     nonces per piece of a device's share (run_share)
  //   P1HIP_KWTAB_MAX_BYTES   MODE 5 table cap (read per scan; a larger table
  //                           re-plans the share without MODE 5)
  //   P1HIP_NO_TABLE          no MODE 5: layouts whose tail block 1 holds only
  //                           lo digits run the digit-update variants (A/B,
  //                           and a second kernel path to cross-check MODE 5)
  //   P1HIP_NO_SPLIT          straddling lo digits use mode 2 instead of the
  //                           split modes (A/B builds with -DP1_NV2_PLAIN)
  //   P1HIP_SCAN_GRID         k_scan's grid (read per scan, scan_grid_for;
  //                           large = one tile per workgroup, no queue)
  uint64_t min_fast_threads = kMinFastThreads;
  bool split = true;
  bool tabulate = true;
  int fail_device = -1;
  p1hip_stats_t stats{};
};

// Never destroyed: the runtime state outlives every static destructor, so a
// p1hip_* call made from a consumer's own atexit handler or static
// destructor still finds a valid mutex and device list, and the library
// issues no HIP call during process teardown (device memory is released
// only by p1hip_shutdown; what a process leaves open, the driver reclaims
// at exit).  The host containers it holds are reachable to the end.
Runtime& rt() {
  static Runtime* r = new Runtime();
  return *r;
}

int dev_release(Dev& d) {
  if (d.ordinal < 0) return 0;
  (void)hipSetDevice(d.ordinal);
  if (d.stream) (void)hipStreamSynchronize(d.stream);
  for (hipEvent_t e : d.evs) (void)hipEventDestroy(e);
  d.evs.clear();
  for (Dev::KwTab& t : d.kwtabs) (void)hipFree(t.dptr);
  d.kwtabs.clear();
  if (d.d_seg) (void)hipFree(d.d_seg);
  if (d.h_seg) (void)hipHostFree(d.h_seg);
  if (d.comm) ncclCommDestroy(d.comm);
  if (d.d_part) (void)hipFree(d.d_part);
  if (d.d_res) (void)hipFree(d.d_res);
  if (d.d_gather) (void)hipFree(d.d_gather);
  if (d.d_small_part) (void)hipFree(d.d_small_part);
  if (d.d_ticket) (void)hipFree(d.d_ticket);
  if (d.d_scan_ticket) (void)hipFree(d.d_scan_ticket);
  if (d.h_res) (void)hipHostFree(d.h_res);
  if (d.stream) (void)hipStreamDestroy(d.stream);
  if (d.mod) (void)hipModuleUnload(d.mod);
  d = Dev();
  return 0;
}

void shutdown_locked(Runtime& R) {
  for (Dev& d : R.devs) dev_release(d);
  R.devs.clear();
}

int init_devs(Runtime& R, const std::vector<int>& ords);

int init_locked(Runtime& R, const std::vector<int>& ords) {
  if (!R.devs.empty()) {
    bool same = R.devs.size() == ords.size();
    for (size_t i = 0; same && i < ords.size(); ++i) same = R.devs[i].ordinal == ords[i];
    if (same) return P1HIP_OK;
    shutdown_locked(R);
  }
  const int rc = init_devs(R, ords);
  if (rc != P1HIP_OK) {  // never leave a half-initialised device list behind
    const std::string keep = g_err;
    shutdown_locked(R);
    g_err = keep;
  }
  return rc;
}

int init_devs(Runtime& R, const std::vector<int>& ords) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
    return fail(P1HIP_ERR_NO_DEVICE, "no HIP device visible");
  for (int o : ords) {
    if (o < 0 || o >= count) return fail(P1HIP_ERR_NO_DEVICE, "device ordinal out of range: " + std::to_string(o));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, o));
    if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0)
      return fail(P1HIP_ERR_NO_DEVICE, std::string("device is not gfx950: ") + prop.gcnArchName);
  }
  R.devs.resize(ords.size());
  const int nd = (int)ords.size();
  for (int i = 0; i < nd; ++i) {
    Dev& d = R.devs[i];
    d.ordinal = ords[i];
    HIPCHK(hipSetDevice(d.ordinal));
    HIPCHK(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    HIPCHK(hipModuleLoadData(&d.mod, p1hip_kernels_co));
    HIPCHK(hipModuleGetFunction(&d.f_scan, d.mod, "k_scan"));
    HIPCHK(hipModuleGetFunction(&d.f_reduce, d.mod, "k_reduce"));
    HIPCHK(hipModuleGetFunction(&d.f_pairs, d.mod, "k_pairs"));
    HIPCHK(hipModuleGetFunction(&d.f_small, d.mod, "k_scan_small"));
    HIPCHK(hipModuleGetFunction(&d.f_kwtable, d.mod, "k_kwtable"));
    HIPCHK(hipMalloc(&d.d_small_part, sizeof(Key) * kSmallMaxBlocks));
    HIPCHK(hipMalloc(&d.d_ticket, sizeof(uint32_t)));
    HIPCHK(hipMalloc(&d.d_scan_ticket, 2 * sizeof(uint32_t)));
    // on the library's own stream: a null-stream call would give every
    // process a second hardware queue (8 miner processes share one GPU)
    HIPCHK(hipMemsetAsync(d.d_ticket, 0, sizeof(uint32_t), d.stream));
    HIPCHK(hipMemsetAsync(d.d_scan_ticket, 0, 2 * sizeof(uint32_t), d.stream));
    // k_scan's grid: every workgroup slot of the device once (the work queue
    // hands the tiles out; p1hip_kernels.hip k_scan)
    {
      hipDeviceProp_t prop;
      HIPCHK(hipGetDeviceProperties(&prop, d.ordinal));
      int per_cu = 0;
      HIPCHK(hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, d.f_scan, kBlock, 0));
      if (per_cu < 1 || prop.multiProcessorCount < 1)
        return fail(P1HIP_ERR_HIP, "k_scan occupancy: " + std::to_string(per_cu) + " blocks per CU");
      d.scan_grid = (uint32_t)per_cu * (uint32_t)prop.multiProcessorCount;
    }
    HIPCHK(hipStreamSynchronize(d.stream));
    HIPCHK(hipMalloc(&d.d_res, sizeof(Key)));
    HIPCHK(hipMalloc(&d.d_gather, sizeof(Key) * nd));
    HIPCHK(hipHostMalloc(&d.h_res, sizeof(Key) * nd, hipHostMallocDefault));
  }
  // P1HIP_NO_RCCL=1 (tests only): combine the per-device results through the
  // host instead of RCCL, so the multi-device code path (threads, sharding,
  // combine) can be exercised with the same GPU listed twice on a 1-GPU box.
  const char* norccl = test_knob("P1HIP_NO_RCCL");
  R.use_rccl = !(norccl && norccl[0] == '1');
  const char* force = test_knob("P1HIP_FORCE_RCCL");
  R.rccl_one = force && force[0] == '1' && R.use_rccl;
  const char* mft = test_knob("P1HIP_MIN_FAST_THREADS");
  R.min_fast_threads = mft ? strtoull(mft, nullptr, 10) : kMinFastThreads;
  const char* nsp = test_knob("P1HIP_NO_SPLIT");
  R.split = !(nsp && nsp[0] == '1');
  const char* ntb = test_knob("P1HIP_NO_TABLE");
  R.tabulate = !(ntb && ntb[0] == '1');
  const char* fdev = test_knob("P1HIP_TEST_FAIL_DEVICE");
  R.fail_device = fdev ? atoi(fdev) : -1;
  if ((nd > 1 || R.rccl_one) && R.use_rccl) {
    std::vector<ncclComm_t> comms(nd);
    NCCLCHK(ncclCommInitAll(comms.data(), nd, ords.data()));
    for (int i = 0; i < nd; ++i) R.devs[i].comm = comms[i];
  }
  return P1HIP_OK;
}

// hipModuleLaunchKernel with the arguments as a pointer array
template <typename... Args>
hipError_t launch(hipFunction_t f, uint32_t blocks, uint32_t threads, hipStream_t st, Args... args) {
  void* params[] = {(void*)&args...};
  return hipModuleLaunchKernel(f, blocks, 1, 1, threads, 1, 1, 0, st, params, nullptr);
}

int ensure_init(Runtime& R) {
  if (!R.devs.empty()) return P1HIP_OK;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
    return fail(P1HIP_ERR_NO_DEVICE, "no HIP device visible");
  std::vector<int> ords;
  for (int i = 0; i < count; ++i) ords.push_back(i);
  return init_locked(R, ords);
}

// Small share [lo, hi] (at most kSmallMaxNonces nonces): one k_scan_small
// launch; the Key lands in d.d_res and, when `to_host`, in d.h_res[0].
int run_small(Dev& d, const uint8_t* msg, size_t len, uint64_t lo, uint64_t hi, bool to_host, bool profiling) {
  HIPCHK(hipSetDevice(d.ordinal));
  d.fast_launches = d.fast_nonces = d.fast_ops = d.gen_launches = d.gen_nonces = 0;
  d.scan_launches = d.scan_nonces = d.scan_ops = 0;
  d.scan_ms = 0.0;
  Plan plan;
  std::string err = make_plan(msg, len, lo, hi, plan, false);
  if (!err.empty()) return fail(P1HIP_ERR_ARGS, "planner: " + err);
  if (plan.launches.size() > kSmallMaxSegs || plan.total_blocks > kSmallMaxBlocks)
    return fail(P1HIP_ERR_ARGS, "internal: small plan exceeds its argument block");
  SmallArgs a;
  memset(&a, 0, sizeof a);
  uint32_t block0 = 0;
  for (size_t i = 0; i < plan.launches.size(); ++i) {
    const Launch& L = plan.launches[i];
    a.ga[i] = L.ga;
    a.block0[i] = block0;
    block0 += L.blocks;
    d.gen_launches++;
    d.gen_nonces += L.nonces;
    d.scan_ops += L.nonces * kAlgOpsPerCompression * (uint64_t)L.btail;
  }
  a.nseg = (uint32_t)plan.launches.size();
  a.nblocks = block0;
  a.part = d.d_small_part;
  a.ticket = d.d_ticket;
  a.out_dev = d.d_res;
  a.out_host = to_host ? d.h_res : nullptr;
  if (profiling) {
    while (d.evs.size() < 2) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      d.evs.push_back(e);
    }
    HIPCHK(hipEventRecord(d.evs[0], d.stream));
  }
  HIPCHK(launch(d.f_small, a.nblocks, kBlock, d.stream, a));
  if (profiling) {
    float ms = 0.f;
    HIPCHK(hipEventRecord(d.evs[1], d.stream));
    HIPCHK(hipEventSynchronize(d.evs[1]));
    HIPCHK(hipEventElapsedTime(&ms, d.evs[0], d.evs[1]));
    d.scan_ms = ms;
  }
  d.scan_launches = 1;
  d.scan_nonces = plan.total_nonces;
  return P1HIP_OK;
}

// Device copy of a MODE 5 launch's K+W table (cached, least recently used
// evicted: the same layout in later scans reuses it; scans are synchronous,
// so an evicted table is idle).
constexpr size_t kMaxKwTabs = 8;
// ... and at most this many bytes of them (a 7-digit table is 2.56 GB; one
// scan needs at most one table per MODE 5 decade, < 2.9 GB in all)
constexpr size_t kMaxKwTabBytes = (size_t)8 << 30;
// kNoTable: the table cannot be had (larger than the cap, or the device is
// out of memory); the caller re-plans the share without MODE 5.
constexpr int kNoTable = 1;

int kwtable_for(Dev& d, const Launch& L, uint64_t* dptr) {
  for (size_t i = 0; i < d.kwtabs.size(); ++i) {
    Dev::KwTab t = d.kwtabs[i];
    if (t.k == L.tabk && memcmp(t.w, L.tabw, sizeof t.w) == 0) {
      t.used_in = d.range_id;
      // least recently used first: a scan touches at most 7 tables (one per
      // MODE 5 decade), so it never evicts one it is about to launch with
      d.kwtabs.erase(d.kwtabs.begin() + (long)i);
      d.kwtabs.push_back(t);
      *dptr = (uint64_t)(uintptr_t)t.dptr;
      return P1HIP_OK;
    }
  }
  const size_t need = (size_t)pow10u(L.tabk) * 64u * sizeof(uint32_t);
  // P1HIP_KWTAB_MAX_BYTES (tests only): a lower cap, to exercise the re-plan
  const char* capv = test_knob("P1HIP_KWTAB_MAX_BYTES");
  const size_t cap = capv ? (size_t)strtoull(capv, nullptr, 10) : kMaxKwTabBytes;
  if (need > cap) return kNoTable;
  for (;;) {
    size_t held = 0;
    for (const Dev::KwTab& t : d.kwtabs) held += (size_t)pow10u(t.k) * 64u * sizeof(uint32_t);
    if (d.kwtabs.empty() || (d.kwtabs.size() < kMaxKwTabs && held + need <= cap)) break;
    // evict the least recently used table this share has not referenced yet
    size_t v = 0;
    while (v < d.kwtabs.size() && d.kwtabs[v].used_in == d.range_id) ++v;
    if (v == d.kwtabs.size()) return kNoTable;  // everything held is in use by this share
    HIPCHK(hipFree(d.kwtabs[v].dptr));
    d.kwtabs.erase(d.kwtabs.begin() + (long)v);
  }
  // built on the device by k_kwtable, on the scan's stream (so the k_scan
  // launch that reads it is ordered after it): no host work, no upload
  Dev::KwTab t;
  memcpy(t.w, L.tabw, sizeof t.w);
  t.k = L.tabk;
  t.dptr = nullptr;
  t.used_in = d.range_id;
  const uint32_t rows = (uint32_t)pow10u(L.tabk);
  const hipError_t me = hipMalloc(&t.dptr, (size_t)rows * 64u * sizeof(uint32_t));
  if (me == hipErrorOutOfMemory) {
    (void)hipGetLastError();  // not sticky: clear it and scan without the table
    return kNoTable;
  }
  HIPCHK(me);
  KwTableArgs a;
  memset(&a, 0, sizeof a);
  memcpy(a.tabw, L.tabw, sizeof a.tabw);
  a.k = (uint32_t)L.tabk;
  a.qv = (uint32_t)(L.Y.q - 64);
  a.rows = rows;
  a.out = t.dptr;
  const hipError_t e = launch(d.f_kwtable, (rows + kBlock - 1) / kBlock, kBlock, d.stream, a);
  if (e != hipSuccess) {  // never cache a table that was not built
    (void)hipFree(t.dptr);
    return fail(P1HIP_ERR_HIP, std::string("k_kwtable launch: ") + hipGetErrorString(e));
  }
  d.kwtabs.push_back(t);
  *dptr = (uint64_t)(uintptr_t)t.dptr;
  return P1HIP_OK;
}

// P1HIP_SCAN_GRID (tests / A/B only, read per scan): k_scan's grid instead of
// the device's workgroup slots; at or above a launch's tile count every
// workgroup runs one tile and the queue hands out none (the round-5
// dispatch, on the same code object).
uint32_t scan_grid_for(const Dev& d, uint32_t tiles) {
  const char* v = test_knob("P1HIP_SCAN_GRID");
  const uint64_t g = v ? strtoull(v, nullptr, 10) : 0;
  const uint32_t slots = g > 0 ? (uint32_t)std::min<uint64_t>(g, kMaxLaunchBlocks) : d.scan_grid;
  return std::min(tiles, slots);
}

// Run one device's share [lo, hi] (lo <= hi) and leave its Key in d.d_res.
int run_range(Dev& d, const uint8_t* msg, size_t len, uint64_t lo, uint64_t hi, bool profiling,
              uint64_t min_fast_threads, bool split, bool tabulate) {
  HIPCHK(hipSetDevice(d.ordinal));
  d.range_id++;  // tables referenced from here on are pinned until the next call
  d.fast_launches = d.fast_nonces = d.fast_ops = d.gen_launches = d.gen_nonces = 0;
  d.scan_launches = d.scan_nonces = d.scan_ops = 0;
  d.scan_ms = 0.0;
  Plan plan;
  // plan -> every MODE 5 table -> launches: a table that cannot be had makes
  // the share re-plan without MODE 5 here, before any k_scan of it (or any
  // segment-table copy) is enqueued, so nothing is scanned twice and no
  // buffer is reallocated behind queued work.  Tables already built stay
  // cached (their k_kwtable launches are complete work, not scan work).
  std::vector<uint64_t> tabptr;
  for (;;) {
    std::string err = make_plan(msg, len, lo, hi, plan, true, min_fast_threads, split, tabulate);
    if (!err.empty()) return fail(P1HIP_ERR_ARGS, "planner: " + err);
    tabptr.assign(plan.launches.size(), 0);
    bool replan = false;
    for (size_t i = 0; i < plan.launches.size() && !replan; ++i) {
      const Launch& L = plan.launches[i];
      if (!L.fast || (L.mode != 5 && L.mode != 7)) continue;
      const int rt = kwtable_for(d, L, &tabptr[i]);
      if (rt == kNoTable) replan = true;
      else if (rt != P1HIP_OK) return rt;
    }
    if (!replan) break;
    tabulate = false;  // the re-plan has no MODE 5 launch, so this loop ends
    d.replans++;
    plan = Plan();
  }
  // Longest-running workgroups first: fast pieces by lo-loop length (10^k),
  // then generic pieces, so short work fills the grid's drain.
  std::vector<size_t> order(plan.launches.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = i;
  auto weight = [&](size_t i) -> uint64_t {
    const Launch& L = plan.launches[i];
    return L.fast ? (uint64_t)(L.fa.kpow / L.fa.nsub) * (uint64_t)L.btail : (uint64_t)L.btail - 1;
  };
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return weight(a) > weight(b); });
  // Pack into launches of <= kMaxSegs segments / kMaxLaunchBlocks workgroups.
  // When a scan needs several launches (e.g. configs[3]'s 2^38 nonces on one
  // GPU), balance them: each batch closes once it reaches total/launches
  // workgroups, so the launches are near-equal rather than one full and one
  // small one (equal drains, and a per-launch average that means something).
  struct Batch { size_t first, count; uint32_t blocks; };
  std::vector<Batch> batches;
  uint64_t all_blocks = 0;
  for (const Launch& L : plan.launches) all_blocks += L.blocks;
  const uint64_t max_blocks = launch_block_limit();
  const uint64_t nlaunch = (all_blocks + max_blocks - 1) / max_blocks;
  const uint64_t target = nlaunch > 1 ? (all_blocks + nlaunch - 1) / nlaunch : max_blocks;
  uint32_t total_blocks = 0;
  for (size_t r = 0; r < order.size(); ++r) {
    const Launch& L = plan.launches[order[r]];
    const uint64_t cur = batches.empty() ? 0 : batches.back().blocks;
    if (batches.empty() || batches.back().count == kMaxSegs || cur + (uint64_t)L.blocks > max_blocks ||
        (cur > 0 && cur + L.blocks / 2 > target && batches.size() < nlaunch))  // fits the next batch better
      batches.push_back({r, 0, 0});
    batches.back().count++;
    batches.back().blocks += L.blocks;
    total_blocks += L.blocks;
  }
  if (total_blocks > d.part_cap) {
    if (d.d_part) HIPCHK(hipFree(d.d_part));
    d.d_part = nullptr;
    size_t cap = 1;
    while (cap < total_blocks) cap <<= 1;
    HIPCHK(hipMalloc(&d.d_part, cap * sizeof(Key)));
    d.part_cap = cap;
  }
  if (batches.size() > d.seg_cap) {
    if (d.d_seg) HIPCHK(hipFree(d.d_seg));
    if (d.h_seg) HIPCHK(hipHostFree(d.h_seg));
    d.d_seg = nullptr;
    d.h_seg = nullptr;
    size_t cap = 4;
    while (cap < batches.size()) cap <<= 1;
    HIPCHK(hipMalloc(&d.d_seg, cap * kMaxSegs * sizeof(Segment)));
    HIPCHK(hipHostMalloc(&d.h_seg, cap * kMaxSegs * sizeof(Segment), hipHostMallocDefault));
    d.seg_cap = cap;
  }
  size_t nev = 0;
  uint32_t part_off = 0;
  for (size_t bi = 0; bi < batches.size(); ++bi) {
    const Batch& B = batches[bi];
    Segment* hs = d.h_seg + bi * kMaxSegs;
    uint64_t ops = 0, nonces = 0;
    uint32_t block0 = 0;
    for (size_t j = 0; j < B.count; ++j) {
      const Launch& L = plan.launches[order[B.first + j]];
      Segment& S = hs[j];
      memset(&S, 0, sizeof S);
      S.block0 = block0;
      block0 += L.blocks;
      if (L.fast) {
        if (!has_variant(L.fv, L.mode, L.trail)) return fail(P1HIP_ERR_ARGS, "no fast kernel variant");
        S.kind = variant_id(L.fv, L.mode, L.trail);
        S.fa = L.fa;
        if (L.mode == 5 || L.mode == 7) S.fa.kwtab = tabptr[order[B.first + j]];
        d.fast_launches++;
        d.fast_nonces += L.nonces;
        d.fast_ops += L.nonces * kAlgOpsPerCompression * (uint64_t)L.btail;
      } else {
        S.kind = kGenericKind;
        S.ga = L.ga;
        d.gen_launches++;
        d.gen_nonces += L.nonces;
      }
      nonces += L.nonces;
      ops += L.nonces * kAlgOpsPerCompression * (uint64_t)L.btail;
    }
    Segment* ds = d.d_seg + bi * kMaxSegs;
    HIPCHK(hipMemcpyAsync(ds, hs, B.count * sizeof(Segment), hipMemcpyHostToDevice, d.stream));
    if (profiling) {
      while (d.evs.size() < nev + 2) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        d.evs.push_back(e);
      }
      HIPCHK(hipEventRecord(d.evs[nev], d.stream));
    }
#ifdef P1_STATIC_GRID
    HIPCHK(launch(d.f_scan, B.blocks, kBlock, d.stream, (const Segment*)ds, (uint32_t)B.count,
                  (Key*)(d.d_part + part_off)));
#else
    // B.blocks tiles through a work queue on min(tiles, slots) workgroups
    HIPCHK(launch(d.f_scan, scan_grid_for(d, B.blocks), kBlock, d.stream, (const Segment*)ds,
                  (uint32_t)B.count, (Key*)(d.d_part + part_off), (uint32_t)B.blocks, d.d_scan_ticket));
#endif
    if (profiling) {
      HIPCHK(hipEventRecord(d.evs[nev + 1], d.stream));
      nev += 2;
    }
    part_off += B.blocks;
    d.scan_launches++;
    d.scan_nonces += nonces;
    d.scan_ops += ops;
  }
  HIPCHK(launch(d.f_reduce, 1, kReduceThreads, d.stream, (const Key*)d.d_part, total_blocks, d.d_res));
  if (profiling && nev) {
    HIPCHK(hipEventSynchronize(d.evs[nev - 1]));
    for (size_t i = 0; i < nev; i += 2) {
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, d.evs[i], d.evs[i + 1]));
      d.scan_ms += ms;
    }
  }
  return P1HIP_OK;
}

// A device's share, in pieces of at most kMaxScanSpan nonces: the plan of a
// share is O(its size / 2^26 hi values), so a share as large as the whole
// u64 range (which the Go loop never finishes either) would need ~10^8
// pieces.  Each piece is a full run_range; the keys are combined on the host
// and the result written back to d.d_res.  Shares up to 2^40 nonces (about
// 30 s of one GPU) are a single piece, with no extra copy.
constexpr uint64_t kMaxScanSpan = 1ull << 40;
int run_share(Dev& d, const uint8_t* msg, size_t len, uint64_t lo, uint64_t hi, const Runtime& R) {
  // P1HIP_MAX_SCAN_SPAN (tests only, read per scan): smaller pieces
  const char* sv = test_knob("P1HIP_MAX_SCAN_SPAN");
  const uint64_t span = sv && strtoull(sv, nullptr, 10) > 0 ? strtoull(sv, nullptr, 10) : kMaxScanSpan;
  if (hi - lo < span)
    return run_range(d, msg, len, lo, hi, R.profiling, R.min_fast_threads, R.split, R.tabulate);
  Key best = {~0ull, ~0ull};
  uint64_t fl = 0, fn = 0, fo = 0, gl = 0, gn = 0, sl = 0, sn = 0, so = 0;
  double sms = 0.0;
  for (uint64_t a = lo;;) {
    const uint64_t b = hi - a < span ? hi : a + (span - 1);
    int r = run_range(d, msg, len, a, b, R.profiling, R.min_fast_threads, R.split, R.tabulate);
    if (r != P1HIP_OK) return r;
    Key k;
    HIPCHK(hipMemcpyAsync(&k, d.d_res, sizeof(Key), hipMemcpyDeviceToHost, d.stream));
    HIPCHK(hipStreamSynchronize(d.stream));
    if (key_lt(k, best)) best = k;
    fl += d.fast_launches; fn += d.fast_nonces; fo += d.fast_ops; gl += d.gen_launches; gn += d.gen_nonces;
    sl += d.scan_launches; sn += d.scan_nonces; so += d.scan_ops; sms += d.scan_ms;
    if (b == hi) break;
    a = b + 1;
  }
  d.fast_launches = fl; d.fast_nonces = fn; d.fast_ops = fo; d.gen_launches = gl; d.gen_nonces = gn;
  d.scan_launches = sl; d.scan_nonces = sn; d.scan_ops = so; d.scan_ms = sms;
  HIPCHK(hipMemcpyAsync(d.d_res, &best, sizeof(Key), hipMemcpyHostToDevice, d.stream));
  HIPCHK(hipStreamSynchronize(d.stream));  // `best` lives on this stack frame
  return P1HIP_OK;
}

Key finish_key(Key k) {
  if (k.h == ~0ull) k.n = 0;  // identity (MaxUint64, 0) of miner.go:56
  return k;
}

int scan_locked(const uint8_t* msg, size_t msg_len, uint64_t lower, uint64_t upper, uint64_t* out_hash,
                uint64_t* out_nonce);
int reduce_pairs_locked(const uint64_t* hashes, const uint64_t* nonces, size_t n, uint64_t* out_hash,
                        uint64_t* out_nonce);

}  // namespace

// ----------------------------------------------------------------------------
// C ABI
// ----------------------------------------------------------------------------
extern "C" {

int p1hip_init(int want_devices, int* got_devices) {
  if (got_devices) *got_devices = 0;
  return guarded([&]() {
    Runtime& R = rt();
    std::lock_guard<std::mutex> g(R.mu);
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
      return fail(P1HIP_ERR_NO_DEVICE, "no HIP device visible");
    int n = want_devices <= 0 ? count : want_devices;
    if (n > count) return fail(P1HIP_ERR_NO_DEVICE, "asked for more devices than visible");
    std::vector<int> ords;
    for (int i = 0; i < n; ++i) ords.push_back(i);
    int rc = init_locked(R, ords);
    if (got_devices) *got_devices = rc == 0 ? (int)R.devs.size() : 0;
    return rc;
  });
}

int p1hip_init_devices(const int* ordinals, int n) {
  if (!ordinals || n <= 0) return fail(P1HIP_ERR_ARGS, "empty device list");
  return guarded([&]() {
    Runtime& R = rt();
    std::lock_guard<std::mutex> g(R.mu);
    return init_locked(R, std::vector<int>(ordinals, ordinals + n));
  });
}

int p1hip_device_count(void) {
  Runtime& R = rt();
  std::lock_guard<std::mutex> g(R.mu);
  return (int)R.devs.size();
}

int p1hip_scan(const uint8_t* msg, size_t msg_len, uint64_t lower, uint64_t upper, uint64_t* out_hash,
               uint64_t* out_nonce) {
  if (!out_hash || !out_nonce) return fail(P1HIP_ERR_ARGS, "null output pointer");
  if (!msg && msg_len > 0) return fail(P1HIP_ERR_ARGS, "msg == NULL with msg_len > 0");
  if (msg_len > P1HIP_MAX_MSG_LEN) return fail(P1HIP_ERR_ARGS, "msg_len exceeds P1HIP_MAX_MSG_LEN");
  return guarded([&]() { return scan_locked(msg, msg_len, lower, upper, out_hash, out_nonce); });
}

}  // extern "C"

namespace {

int scan_locked(const uint8_t* msg, size_t msg_len, uint64_t lower, uint64_t upper, uint64_t* out_hash,
                uint64_t* out_nonce) {
  Runtime& R = rt();
  std::lock_guard<std::mutex> g(R.mu);
  const auto t0 = std::chrono::steady_clock::now();
  int rc = ensure_init(R);
  if (rc) return rc;
  Key res = {~0ull, 0};
  if (lower <= upper) {
    const size_t nd = R.devs.size();
    // contiguous shards of near-equal predicted cost (planner.hpp plan_shards)
    std::vector<uint64_t> slo(nd), shi(nd);
    std::vector<char> active(nd, 0);
    plan_shards(msg, msg_len, lower, upper, (int)nd, slo.data(), shi.data());
    for (size_t i = 0; i < nd; ++i) active[i] = slo[i] <= shi[i];
    // Phase 1: every device scans its shard and synchronises its stream.
    // Phase 2 (the collective) starts only when every device succeeded, so a
    // failing device can never leave its peers blocked inside ncclAllGather.
    std::vector<int> rcs(nd, 0);
    std::vector<std::string> errs(nd);
    auto run_threads = [&](auto&& fn) {
      if (nd == 1) {
        fn(0);
      } else {
        // every thread is created before any of them runs `fn`: if one cannot
        // start, none enters the scan or the collective (a peer blocked in
        // ncclAllGather waiting for a thread that never started would hang)
        std::atomic<int> go{0};  // 0 wait, 1 run, -1 abort
        std::vector<std::thread> th;
        try {
          for (size_t i = 0; i < nd; ++i)
            th.emplace_back([&, i]() {
              while (go.load(std::memory_order_acquire) == 0) std::this_thread::yield();
              if (go.load(std::memory_order_acquire) == 1) fn(i);
            });
        } catch (...) {
          go.store(-1, std::memory_order_release);
          for (auto& t : th) t.join();
          throw;
        }
        go.store(1, std::memory_order_release);
        for (auto& t : th) t.join();
      }
    };
    auto first_error = [&]() -> int {
      for (size_t i = 0; i < nd; ++i)
        if (rcs[i]) return fail(rcs[i], "device " + std::to_string(R.devs[i].ordinal) + ": " + errs[i]);
      return P1HIP_OK;
    };
    const bool coll = (nd > 1 || R.rccl_one) && R.use_rccl;
    const uint64_t small_max = small_limit();
    run_threads([&](size_t i) {
      Dev& d = R.devs[i];
      int r = P1HIP_OK;
      const auto p0 = std::chrono::steady_clock::now();
      // per-scan accounting starts empty on every device (an inactive shard
      // must not re-report its previous scan)
      d.fast_launches = d.fast_nonces = d.fast_ops = d.gen_launches = d.gen_nonces = 0;
      d.scan_launches = d.scan_nonces = d.scan_ops = 0;
      d.scan_ms = 0.0;
      d.replans = 0;
      d.small_used = false;
      d.acc.shard_first = slo[i];
      d.acc.shard_last = shi[i];
      d.acc.active = active[i];
      // a host exception inside a device thread would end the process
      // (std::terminate): it becomes this device's error instead
      try {
      if ((int)i == R.fail_device) {
        r = fail(P1HIP_ERR_HIP, "injected failure (P1HIP_TEST_FAIL_DEVICE)");
      } else if (active[i] && shi[i] - slo[i] < small_max) {
        d.small_used = true;
        r = run_small(d, msg, msg_len, slo[i], shi[i], !coll && nd == 1, R.profiling);
      } else if (active[i]) {
        r = run_share(d, msg, msg_len, slo[i], shi[i], R);
      } else {
        // empty shard: contribute the identity key (all ones)
        if (hipSetDevice(d.ordinal) != hipSuccess) r = fail(P1HIP_ERR_HIP, "hipSetDevice");
        if (!r && hipMemsetAsync(d.d_res, 0xFF, sizeof(Key), d.stream) != hipSuccess)
          r = fail(P1HIP_ERR_HIP, "hipMemsetAsync(identity)");
      }
      if (!r && !coll && nd > 1) {  // host combine (P1HIP_NO_RCCL, tests)
        if (hipMemcpyAsync(R.devs[0].h_res + i, d.d_res, sizeof(Key), hipMemcpyDeviceToHost, d.stream) != hipSuccess)
          r = fail(P1HIP_ERR_HIP, "hipMemcpyAsync(result)");
      } else if (!r && !coll && !(active[i] && d.small_used)) {  // the small kernel wrote h_res itself
        if (hipMemcpyAsync(d.h_res, d.d_res, sizeof(Key), hipMemcpyDeviceToHost, d.stream) != hipSuccess)
          r = fail(P1HIP_ERR_HIP, "hipMemcpyAsync(result)");
      }
      if (!r && hipStreamSynchronize(d.stream) != hipSuccess) r = fail(P1HIP_ERR_HIP, "hipStreamSynchronize");
      } catch (const std::exception& ex) {
        try {
          r = fail(P1HIP_ERR_HIP, std::string("host: ") + ex.what());
        } catch (...) {
          r = P1HIP_ERR_HIP;
        }
      } catch (...) {
        r = P1HIP_ERR_HIP;
      }
      d.acc.phase1_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - p0).count();
      rcs[i] = r;
      if (r) {
        try {
          errs[i] = g_err;
        } catch (...) {  // the copy allocates; rcs[i] already says what matters
        }
      }
    });
    if ((rc = first_error()) != P1HIP_OK) return rc;
    if (coll) {
      // Phase 2: all-gather the 16-byte partials (2 x u64 per device) over
      // RCCL; device 0 copies the gathered table to the host.  One group call
      // per device thread is not needed: each thread enqueues on its own
      // communicator and the collective completes when all have joined.
      run_threads([&](size_t i) {
        Dev& d = R.devs[i];
        int r = P1HIP_OK;
        const auto g0 = std::chrono::steady_clock::now();
        // as in phase 1: a host exception (the error strings below allocate)
        // becomes this device's rc, never std::terminate
        try {
        if (hipSetDevice(d.ordinal) != hipSuccess) r = fail(P1HIP_ERR_HIP, "hipSetDevice");
        if (!r) {
          ncclResult_t nr = ncclAllGather(d.d_res, d.d_gather, 2, ncclUint64, d.comm, d.stream);
          if (nr != ncclSuccess) r = fail(P1HIP_ERR_RCCL, std::string("ncclAllGather: ") + ncclGetErrorString(nr));
        }
        if (!r && i == 0 &&
            hipMemcpyAsync(d.h_res, d.d_gather, sizeof(Key) * nd, hipMemcpyDeviceToHost, d.stream) != hipSuccess)
          r = fail(P1HIP_ERR_HIP, "hipMemcpyAsync(gathered)");
        if (!r && hipStreamSynchronize(d.stream) != hipSuccess) r = fail(P1HIP_ERR_HIP, "hipStreamSynchronize");
        d.acc.gather_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - g0).count();
        rcs[i] = r;
        if (r) errs[i] = g_err;
        } catch (...) {
          rcs[i] = P1HIP_ERR_HIP;  // errs[i] stays empty: building it may be what threw
        }
      });
      if ((rc = first_error()) != P1HIP_OK) return rc;
    }
    Key b = {~0ull, ~0ull};
    for (size_t i = 0; i < nd; ++i) b = key_lt(R.devs[0].h_res[i], b) ? R.devs[0].h_res[i] : b;
    res = finish_key(b);
    for (Dev& d : R.devs) {
      R.stats.fast_launches += d.fast_launches;
      R.stats.fast_nonces += d.fast_nonces;
      R.stats.fast_alg_ops += d.fast_ops;
      R.stats.generic_launches += d.gen_launches;
      R.stats.generic_nonces += d.gen_nonces;
      R.stats.scan_launches += d.scan_launches;
      R.stats.scan_nonces += d.scan_nonces;
      R.stats.scan_alg_ops += d.scan_ops;
      R.stats.scan_kernel_ms += d.scan_ms;
      if (d.small_used && d.scan_launches) R.stats.small_scans++;
      R.stats.table_replans += d.replans;
      d.acc.scans++;
      d.acc.scan_launches += d.scan_launches;
      d.acc.scan_nonces += d.scan_nonces;
      d.acc.scan_alg_ops += d.scan_ops;
      d.acc.scan_kernel_ms += d.scan_ms;
    }
  }
  R.stats.scans++;
  R.stats.scan_wall_ms +=
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *out_hash = res.h;
  *out_nonce = res.n;
  return P1HIP_OK;
}

}  // namespace

extern "C" {

int p1hip_plan_shards(const uint8_t* msg, size_t msg_len, uint64_t lower, uint64_t upper, int n,
                      uint64_t* first, uint64_t* last) {
  if (n <= 0 || !first || !last) return fail(P1HIP_ERR_ARGS, "n <= 0 or null output");
  if (!msg && msg_len > 0) return fail(P1HIP_ERR_ARGS, "msg == NULL with msg_len > 0");
  if (msg_len > P1HIP_MAX_MSG_LEN) return fail(P1HIP_ERR_ARGS, "msg_len exceeds P1HIP_MAX_MSG_LEN");
  if (lower > upper) {
    for (int i = 0; i < n; ++i) { first[i] = 1; last[i] = 0; }
    return P1HIP_OK;
  }
  return guarded([&]() {
    plan_shards(msg, msg_len, lower, upper, n, first, last);
    return P1HIP_OK;
  });
}

int p1hip_hash(const uint8_t* msg, size_t msg_len, uint64_t nonce, uint64_t* out_hash) {
  uint64_t n = 0;
  return p1hip_scan(msg, msg_len, nonce, nonce, out_hash, &n);
}

int p1hip_reduce_pairs(const uint64_t* hashes, const uint64_t* nonces, size_t n, uint64_t* out_hash,
                       uint64_t* out_nonce) {
  if (!out_hash || !out_nonce || (n && (!hashes || !nonces))) return fail(P1HIP_ERR_ARGS, "null pointer");
  return guarded([&]() { return reduce_pairs_locked(hashes, nonces, n, out_hash, out_nonce); });
}

}  // extern "C"

namespace {
int reduce_pairs_locked(const uint64_t* hashes, const uint64_t* nonces, size_t n, uint64_t* out_hash,
                        uint64_t* out_nonce) {
  Runtime& R = rt();
  std::lock_guard<std::mutex> g(R.mu);
  int rc = ensure_init(R);
  if (rc) return rc;
  Dev& d = R.devs[0];
  HIPCHK(hipSetDevice(d.ordinal));
  Key res = {~0ull, ~0ull};
  if (n > (size_t)kMaxLaunchBlocks * kBlock) return fail(P1HIP_ERR_ARGS, "too many pairs");
  if (n) {
    uint64_t *dh = nullptr, *dn = nullptr;
    Key* dp = nullptr;
    // frees the scratch buffers on every exit path (HIPCHK returns early)
    struct Scratch {
      uint64_t **a, **b;
      Key** c;
      ~Scratch() {
        if (*a) (void)hipFree(*a);
        if (*b) (void)hipFree(*b);
        if (*c) (void)hipFree(*c);
      }
    } scratch{&dh, &dn, &dp};
    const uint32_t blocks = (uint32_t)((n + kBlock - 1) / kBlock);
    HIPCHK(hipMalloc(&dh, n * 8));
    HIPCHK(hipMalloc(&dn, n * 8));
    HIPCHK(hipMalloc(&dp, (size_t)blocks * sizeof(Key)));
    HIPCHK(hipMemcpyAsync(dh, hashes, n * 8, hipMemcpyHostToDevice, d.stream));
    HIPCHK(hipMemcpyAsync(dn, nonces, n * 8, hipMemcpyHostToDevice, d.stream));
    HIPCHK(launch(d.f_pairs, blocks, kBlock, d.stream, (const uint64_t*)dh, (const uint64_t*)dn, (uint64_t)n, dp));
    HIPCHK(launch(d.f_reduce, 1, kReduceThreads, d.stream, (const Key*)dp, blocks, d.d_res));
    HIPCHK(hipMemcpyAsync(d.h_res, d.d_res, sizeof(Key), hipMemcpyDeviceToHost, d.stream));
    HIPCHK(hipStreamSynchronize(d.stream));
    res = d.h_res[0];
  }
  res = finish_key(res);
  *out_hash = res.h;
  *out_nonce = res.n;
  return P1HIP_OK;
}
}  // namespace

extern "C" {

int p1hip_set_profiling(int on) {
  Runtime& R = rt();
  std::lock_guard<std::mutex> g(R.mu);
  R.profiling = on != 0;
  return P1HIP_OK;
}

int p1hip_get_stats(p1hip_stats_t* out) {
  if (!out) return fail(P1HIP_ERR_ARGS, "null stats pointer");
  Runtime& R = rt();
  std::lock_guard<std::mutex> g(R.mu);
  *out = R.stats;
  return P1HIP_OK;
}

void p1hip_reset_stats(void) {
  Runtime& R = rt();
  std::lock_guard<std::mutex> g(R.mu);
  R.stats = p1hip_stats_t{};
  for (Dev& d : R.devs) {
    d.acc = p1hip_device_stats_t{};
    d.acc.shard_first = 1;  // empty until the next scan
  }
}

int p1hip_get_device_stats(int index, p1hip_device_stats_t* out) {
  if (!out) return fail(P1HIP_ERR_ARGS, "null stats pointer");
  Runtime& R = rt();
  std::lock_guard<std::mutex> g(R.mu);
  if (index < 0 || (size_t)index >= R.devs.size()) return fail(P1HIP_ERR_ARGS, "device index out of range");
  *out = R.devs[(size_t)index].acc;
  out->ordinal = R.devs[(size_t)index].ordinal;
  return P1HIP_OK;
}

int p1hip_comm_info(int index, int* nranks, int* rank) {
  if (!nranks || !rank) return fail(P1HIP_ERR_ARGS, "null comm-info pointer");
  *nranks = 0;
  *rank = -1;
  Runtime& R = rt();
  std::lock_guard<std::mutex> g(R.mu);
  if (index < 0 || (size_t)index >= R.devs.size()) return fail(P1HIP_ERR_ARGS, "device index out of range");
  const Dev& d = R.devs[(size_t)index];
  if (!d.comm) return P1HIP_OK;  // one device without P1HIP_FORCE_RCCL, or host combine
  // what RCCL itself says, not what init asked for
  int count = 0, user = -1;
  NCCLCHK(ncclCommCount(d.comm, &count));
  NCCLCHK(ncclCommUserRank(d.comm, &user));
  *nranks = count;
  *rank = user;
  return P1HIP_OK;
}

int p1hip_abi_version(void) { return P1HIP_ABI_VERSION; }

const char* p1hip_last_error(void) { return g_err.c_str(); }

const char* p1hip_version(void) { return "p1hip 0.5 gfx950"; }

const char* p1hip_test_knobs(void) {
  static thread_local std::string s;
  s.clear();
  try {
    // the knobs the environment sets now (read per scan, or at the next init)
    std::vector<std::pair<std::string, std::string>> kv;
    if (test_knobs_on()) {
      kv.push_back({"P1HIP_TEST_KNOBS", "1"});
      for (const char* k : kTestKnobs)
        if (const char* v = test_knob(k)) kv.push_back({k, v});
    }
    // ... and the ones read at init that the open devices still run with,
    // even if the environment has changed since
    Runtime& R = rt();
    std::lock_guard<std::mutex> g(R.mu);
    auto add = [&](const char* k, const std::string& v) {
      for (auto& e : kv)
        if (e.first == k) {
          if (e.second != v) e.second += " (init: " + v + ")";
          return;
        }
      kv.push_back({k, "(init: " + v + ")"});
    };
    if (!R.devs.empty()) {
      if (R.min_fast_threads != kMinFastThreads) add("P1HIP_MIN_FAST_THREADS", std::to_string(R.min_fast_threads));
      if (R.fail_device >= 0) add("P1HIP_TEST_FAIL_DEVICE", std::to_string(R.fail_device));
      if (!R.tabulate) add("P1HIP_NO_TABLE", "1");
      if (!R.split) add("P1HIP_NO_SPLIT", "1");
      if (!R.use_rccl) add("P1HIP_NO_RCCL", "1");
      if (R.rccl_one) add("P1HIP_FORCE_RCCL", "1");
    }
    for (size_t i = 0; i < kv.size(); ++i) s += (i ? ";" : "") + kv[i].first + "=" + kv[i].second;
  } catch (...) {
    s = "?";  // never empty when the state could not be read
  }
  return s.c_str();
}

int p1hip_device_info(int index, p1hip_device_info_t* out) {
  if (!out) return fail(P1HIP_ERR_ARGS, "null info pointer");
  return guarded([&]() {
    Runtime& R = rt();
    std::lock_guard<std::mutex> g(R.mu);
    if (index < 0 || (size_t)index >= R.devs.size()) return fail(P1HIP_ERR_ARGS, "device index out of range");
    const int o = R.devs[(size_t)index].ordinal;
    memset(out, 0, sizeof *out);
    out->ordinal = o;
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, o));
    HIPCHK(hipDeviceGetPCIBusId(out->pci_bus_id, (int)sizeof out->pci_bus_id - 1, o));
    out->cu_count = prop.multiProcessorCount;
    out->clock_khz = prop.clockRate;
    out->hbm_bytes = (uint64_t)prop.totalGlobalMem;
    strncpy(out->arch, prop.gcnArchName, sizeof out->arch - 1);
    static_assert(sizeof(prop.uuid.bytes) == sizeof(out->uuid), "uuid size");
    memcpy(out->uuid, prop.uuid.bytes, sizeof out->uuid);
    return P1HIP_OK;
  });
}

void p1hip_shutdown(void) {
  Runtime& R = rt();
  std::lock_guard<std::mutex> g(R.mu);
  shutdown_locked(R);
}

}  // extern "C"
