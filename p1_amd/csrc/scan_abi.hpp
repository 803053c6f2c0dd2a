// scan_abi.hpp -- what the host runtime (p1hip.hip) and the device code
// object (p1hip_kernels.hip) agree on: the segment table of one k_scan launch,
// variant ids and launch shapes.  The kernels are loaded by name from the
// embedded code object (hipModuleLoadData), so this header IS their ABI.
#pragma once
#include "scan_core.hpp"

namespace p1 {

// Variant id of a fast segment <FV, MODE, TRAIL> (MODE: scan_core.hpp
// fast_thread); kGenericKind marks a generic segment.
P1_HD constexpr uint32_t variant_id(int fv, int mode, bool trail) {
  return mode == 5   ? 128u + (uint32_t)fv
         : mode == 7 ? 192u + (uint32_t)fv
         : mode == 6 ? 160u + (trail ? 16u : 0u) + (uint32_t)fv
                     : (trail ? 64u : 0u) + (uint32_t)fv * 4u + (uint32_t)(mode - 1);
}
constexpr uint32_t kGenericKind = 255;

// One segment of a scan launch: a contiguous run of workgroups that all do
// the same kind of work (one decade piece).
struct Segment {
  uint32_t kind;    // variant_id(...) or kGenericKind
  uint32_t block0;  // first workgroup of the segment within the launch
  uint32_t pad[2];
  FastArgs fa;
  GenArgs ga;
};

constexpr int kReduceThreads = 1024;  // k_reduce: one workgroup

// k_kwtable: builds a MODE 5 table on the device, one row per thread
// (scan_core.hpp kwtable_row).
struct KwTableArgs {
  uint32_t tabw[16];  // tail block 1, '0' at the lo digit bytes
  uint32_t k, qv, rows;
  uint32_t pad_;
  uint32_t* out;      // rows x 64 words
};

// Small scans (configs[0]-sized requests, single nonces of p1hip_hash): one
// launch of k_scan_small with the whole plan in its kernel arguments (no
// table copy), generic pieces only, and the grid's last workgroup folding the
// partials (no k_reduce launch) and writing the result straight to pinned
// host memory (no copy back).  [lower, upper] with at most kSmallMaxNonces
// nonces spans at most 5 decades, so at most kSmallMaxSegs pieces.
constexpr uint32_t kSmallMaxSegs = 6;
constexpr uint64_t kSmallMaxNonces = 1u << 16;
constexpr uint32_t kSmallMaxBlocks = (uint32_t)(kSmallMaxNonces / kBlock) + kSmallMaxSegs;
struct SmallArgs {
  GenArgs ga[kSmallMaxSegs];
  uint32_t block0[kSmallMaxSegs];  // first workgroup of each piece
  uint32_t nseg;
  uint32_t nblocks;                // workgroups in the grid
  Key* part;                       // kSmallMaxBlocks partials (device)
  uint32_t* ticket;                // device counter, 0 between scans
  Key* out_dev;                    // result (device, for the multi-device combine)
  Key* out_host;                   // result (pinned host) or null
};

// Kernel entry points (extern "C" names in the code object):
//   k_scan(const Segment* segs, uint32_t nseg, Key* part, uint32_t ntiles, uint32_t* ticket)
//                                     grid: min(ntiles, occupancy x CUs) x kBlock; tiles = sum of segment
//                                     blocks, handed out through ticket[0..1] (0 between launches)
//                                     (-DP1_STATIC_GRID: the first three arguments, grid = ntiles)
//   k_reduce(const Key* part, uint32_t n, Key* out)                  grid: 1 x kReduceThreads
//   k_pairs(const uint64_t* hs, const uint64_t* ns, uint64_t n, Key* part)  grid: ceil(n/kBlock) x kBlock
//   k_scan_small(SmallArgs a)                                        grid: a.nblocks x kBlock
//   k_kwtable(KwTableArgs a)                                         grid: ceil(a.rows/kBlock) x kBlock
}  // namespace p1
