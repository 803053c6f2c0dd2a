// p1hip_kernels.hip -- the gfx950 device code of libp1hip.so.
//
// Built on its own (device-only) into assembly, passed through
// tools/isa_post.py, assembled and linked into a code object that
// libp1hip.so embeds and loads with hipModuleLoadData (see Makefile and
// DESIGN.md "Build").  The ABI with the host runtime is scan_abi.hpp.
//
// Replaces the miner's scan loop /root/reference/src/github.com/cmu440/bitcoin/
// miner/miner.go:56-63:
//   k_scan    -> one launch, one segment per planner piece (variant chosen per
//                tile from the segment table: fast_thread<FV,NV,TRAIL>
//                or generic_thread); a work queue of workgroup-sized tiles
//                over a grid the device holds at once
//             -> per-thread best (hash, nonce) -> wave argmin with DPP
//                (quad_perm, row_ror) + ds_swizzle + readlane -> LDS across
//                the 4 waves -> one 16-byte partial per workgroup
//   k_reduce  -> one workgroup folds all partials into the device result
//   k_pairs   -> test hook: the same argmin over crafted (hash, nonce) pairs
#include <hip/hip_runtime.h>

#include "scan_abi.hpp"

using namespace p1;

// ----------------------------------------------------------------------------
// Wave / workgroup argmin over Key = (hash, nonce), lexicographic.
// ----------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}

template <int CTRL>
__device__ __forceinline__ Key key_dpp(const Key& k) {
  Key o;
  o.h = ((uint64_t)dpp<CTRL>((uint32_t)(k.h >> 32)) << 32) | dpp<CTRL>((uint32_t)k.h);
  o.n = ((uint64_t)dpp<CTRL>((uint32_t)(k.n >> 32)) << 32) | dpp<CTRL>((uint32_t)k.n);
  return o;
}

__device__ __forceinline__ uint32_t swz_xor16(uint32_t v) {
  // ds_swizzle bit-mask mode: and 0x1f, or 0, xor 0x10 (within 32 lanes)
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);
}

__device__ __forceinline__ Key key_min(const Key& a, const Key& b) { return key_lt(b, a) ? b : a; }

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

// All 64 lanes must be active.  Returns the wave minimum (wave-uniform).
__device__ __forceinline__ Key wave_min(Key k) {
  k = key_min(k, key_dpp<0xB1>(k));   // quad_perm [1,0,3,2]  (xor 1)
  k = key_min(k, key_dpp<0x4E>(k));   // quad_perm [2,3,0,1]  (xor 2)
  k = key_min(k, key_dpp<0x124>(k));  // row_ror:4
  k = key_min(k, key_dpp<0x128>(k));  // row_ror:8  -> every lane holds its row min
  Key o;
  o.h = ((uint64_t)swz_xor16((uint32_t)(k.h >> 32)) << 32) | swz_xor16((uint32_t)k.h);
  o.n = ((uint64_t)swz_xor16((uint32_t)(k.n >> 32)) << 32) | swz_xor16((uint32_t)k.n);
  k = key_min(k, o);                  // halves of 32 lanes
  Key a, b;
  a.h = readlane64(k.h, 0);  a.n = readlane64(k.n, 0);
  b.h = readlane64(k.h, 32); b.n = readlane64(k.n, 32);
  return key_min(a, b);
}

template <int NT>
__device__ __forceinline__ void block_min_store(Key k, Key* out) {
  __shared__ Key sk[NT / 64];
  k = wave_min(k);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) sk[wid] = k;
  __syncthreads();
  if (threadIdx.x == 0) {
    Key b = sk[0];
#pragma unroll
    for (int w = 1; w < NT / 64; ++w) b = key_min(b, sk[w]);
    *out = b;
  }
}

// ----------------------------------------------------------------------------
// Kernels
// ----------------------------------------------------------------------------
// Minimum waves per SIMD the register allocator must leave room for
// (tuned on MI355X); override with -DP1_FAST_WAVES=n.
#ifndef P1_FAST_WAVES
#define P1_FAST_WAVES 4
#endif

// One tile of a scan: workgroup-sized work `b` finds its segment
// (wave-uniform scalar loop over the table), runs that segment's per-thread
// work and writes one 16-byte partial.  All decades of a scan -- and their
// ragged edges -- share one launch, so there is one grid drain per scan,
// filled by the short segments that are placed last.
__device__ __forceinline__ void scan_tile(const Segment* __restrict__ segs, uint32_t nseg, Key* __restrict__ part,
                                          uint32_t b) {
  uint32_t si = 0;
  while (si + 1 < nseg && segs[si + 1].block0 <= b) ++si;
  const Segment& S = segs[si];
  const uint32_t local = (b - S.block0) * kBlock + threadIdx.x;
  Key k;
  switch (S.kind) {
#define P1_CASE(FV, NV, TR)                         \
  case variant_id(FV, NV, TR):                      \
    k = fast_thread<FV, NV, TR>(S.fa, local);       \
    break;
// P1_VARIANTS_INC: a subset of the variant list (tools/variant_report.py
// builds one variant per code object to read its registers and loop mix)
#ifdef P1_VARIANTS_INC
#include P1_VARIANTS_INC
#else
#include "fast_variants.inc"
#endif
#undef P1_CASE
    default:
      k = generic_thread(S.ga, local);
      break;
  }
  block_min_store<kBlock>(k, part + b);
}

#ifdef P1_STATIC_GRID
// A/B (round 5 and before): one workgroup per tile, the grid is the tiles.
extern "C" __global__ __launch_bounds__(kBlock, P1_FAST_WAVES) void k_scan(const Segment* __restrict__ segs,
                                                                           uint32_t nseg, Key* __restrict__ part) {
  scan_tile(segs, nseg, part, blockIdx.x);
}
#else
// The scan kernel as a work queue over `ntiles` tiles (round 6).  The
// hardware hands workgroup i to XCD i mod 8, and under this load the XCDs
// do not run at one clock (tools/xcd_probe: the odd XCDs 1.5% below the
// even ones, profiles/r06b_xcd.jsonl), so a grid of one workgroup per tile
// waits for the slowest XCD's eighth of the work.  Here the grid is what
// the device holds at once (p1hip.hip: occupancy x CUs, or ntiles if
// fewer); each workgroup runs tile blockIdx.x, then takes the next tile
// from an agent-scope counter until none is left, so a faster XCD simply
// runs more tiles.  Every tile is still one workgroup's work with its own
// partial at part[tile].  Every wave reads the same next tile from LDS, so
// the whole workgroup leaves the loop together once the tiles run out.
// ticket[0] counts tiles handed out, ticket[1] workgroups done; the last
// workgroup to finish zeroes both for the stream's next launch.
extern "C" __global__ __launch_bounds__(kBlock, P1_FAST_WAVES) void k_scan(const Segment* __restrict__ segs,
                                                                           uint32_t nseg, Key* __restrict__ part,
                                                                           uint32_t ntiles,
                                                                           uint32_t* __restrict__ ticket) {
  __shared__ uint32_t s_next;
  uint32_t b = blockIdx.x;
  for (;;) {
    scan_tile(segs, nseg, part, b);
    if (threadIdx.x == 0)
      s_next = gridDim.x + __hip_atomic_fetch_add(&ticket[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    b = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_next);
    if (b >= ntiles) break;
  }
  if (threadIdx.x == 0 &&
      __hip_atomic_fetch_add(&ticket[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
    // every other workgroup has taken its last tile: nobody reads the counter again
    __hip_atomic_store(&ticket[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&ticket[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
#endif

extern "C" __global__ __launch_bounds__(kReduceThreads) void k_reduce(const Key* __restrict__ part, uint32_t n,
                                                                      Key* __restrict__ out) {
  Key b = {~0ull, ~0ull};
  for (uint32_t i = threadIdx.x; i < n; i += kReduceThreads) b = key_min(b, part[i]);
  block_min_store<kReduceThreads>(b, out);
}

// Small scans: one launch, whole plan in the kernel arguments (generic pieces,
// one nonce per thread), the last workgroup to finish folds every partial.
// Partials cross XCDs (each XCD has its own L2), so the writers release at
// agent scope before taking a ticket and the last workgroup acquires after.
extern "C" __global__ __launch_bounds__(kBlock) void k_scan_small(SmallArgs a) {
  const uint32_t b = blockIdx.x;
  uint32_t si = 0;
  while (si + 1 < a.nseg && a.block0[si + 1] <= b) ++si;
  const Key k = generic_thread(a.ga[si], (uint64_t)(b - a.block0[si]) * kBlock + threadIdx.x);
  block_min_store<kBlock>(k, a.part + b);
  __shared__ uint32_t last;
  if (threadIdx.x == 0) {
    __atomic_thread_fence(__ATOMIC_RELEASE);
    last = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == a.nblocks - 1;
  }
  __syncthreads();
  if (!last) return;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  Key m = {~0ull, ~0ull};
  for (uint32_t i = threadIdx.x; i < a.nblocks; i += kBlock) {
    Key p;
    p.h = __hip_atomic_load(&a.part[i].h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    p.n = __hip_atomic_load(&a.part[i].n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    m = key_min(m, p);
  }
  block_min_store<kBlock>(m, a.out_dev);
  if (threadIdx.x == 0) {
    *a.ticket = 0;  // ready for the next scan (launches on the stream are ordered)
    if (a.out_host) {
      *a.out_host = *a.out_dev;
      __atomic_thread_fence(__ATOMIC_RELEASE);  // system-visible before the kernel ends
    }
  }
}

// MODE 5 table: row c = K + W of tail block 1 for lo value c
extern "C" __global__ __launch_bounds__(kBlock) void k_kwtable(KwTableArgs a) {
  const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
  if (c >= a.rows) return;
  uint32_t row[64];
  kwtable_row(a.tabw, (int)a.k, (int)a.qv, c, row);
  uint4* out = (uint4*)(a.out + (size_t)c * 64u);
#pragma unroll
  for (int i = 0; i < 16; ++i) out[i] = make_uint4(row[4 * i], row[4 * i + 1], row[4 * i + 2], row[4 * i + 3]);
}

// test hook: one crafted pair per thread -> per-workgroup partials
extern "C" __global__ __launch_bounds__(kBlock) void k_pairs(const uint64_t* __restrict__ hs,
                                                             const uint64_t* __restrict__ ns, uint64_t n,
                                                             Key* __restrict__ part) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  Key k = {~0ull, ~0ull};
  if (i < n) { k.h = hs[i]; k.n = ns[i]; }
  block_min_store<kBlock>(k, part + blockIdx.x);
}
