// XCD-aware workgroup remap (MI355X: 8 XCDs, each with a private L2; cdna_hip_programming.md
// §5.5 T1).  Dispatch hands consecutive blockIdx values to different XCDs, so neighbouring
// macroblocks -- whose motion-search windows and interpolation footprints share most of
// their reference lines -- would each pull those lines into a different L2.  Remapping gives
// every XCD one contiguous band of work items instead.  Bijective for any grid size (the
// blocks with label bid % 8 == k are treated as XCD k's; a wrong guess about placement only
// costs speed, never correctness).
#pragma once
#include <hip/hip_runtime.h>

namespace mx {

constexpr int kNumXcd = 8;

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int xcd = bid % kNumXcd, q = nwg / kNumXcd, r = nwg % kNumXcd;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / kNumXcd;
}

// Row-interleaved variant for work whose cost varies across the picture (motion search exits
// early on static blocks, noise costs the most): XCD k takes chunks (e.g. MB rows) k, k+8,
// k+16, ... so horizontal neighbours share an L2 while every XCD still samples the whole
// frame.  Blocks past the last full group of 8 chunks keep the identity mapping (bijective).
__device__ __forceinline__ int xcd_interleave(int bid, int nwg, int chunk) {
    const int group = kNumXcd * chunk, main = nwg - nwg % group;
    if (bid >= main) return bid;
    const int xcd = bid % kNumXcd, j = bid / kNumXcd;
    return ((j / chunk) * kNumXcd + xcd) * chunk + j % chunk;
}

}  // namespace mx
