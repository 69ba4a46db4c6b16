// scan.hpp -- block-level scan helpers for 256-lane (4-wave) workgroups.
#pragma once
#include "common.hpp"

namespace crdt {

// Exclusive scan of one uint64 per lane across a 256-lane block; *total gets
// the block sum.  Every lane of the block must call it (contains barriers).
__device__ __forceinline__ uint64_t block_exclusive_scan_u64(uint64_t v, uint64_t *total) {
    __shared__ uint64_t wsum[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint64_t off = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint64_t s = wsum[k];
        off += (k < w) ? s : 0;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return off + x - v;
}

// Exclusive rank of a per-lane predicate across the 256-lane block using
// wave ballots (mbcnt) -- cheaper than the generic scan for 0/1 flags.
__device__ __forceinline__ uint32_t block_rank_flag(bool f, uint32_t *total) {
    __shared__ uint32_t wcnt[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t m = __ballot(f);
    const uint32_t below = (uint32_t)__popcll(m & ((lane == 0) ? 0ULL : (~0ULL >> (64 - lane))));
    if (lane == 0) wcnt[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t s = wcnt[k];
        off += (k < w) ? s : 0;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return off + below;
}

}  // namespace crdt
