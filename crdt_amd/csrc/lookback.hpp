// lookback.hpp -- single-pass decoupled look-back over per-tile status words
// (used by the set merges and the RefMerge walk).
#pragma once
#include "common.hpp"

namespace crdt {

constexpr uint64_t kFlagAgg = 1ULL << 62;     // tile count available
constexpr uint64_t kFlagInc = 2ULL << 62;     // inclusive prefix available
constexpr uint64_t kValMask = (1ULL << 62) - 1;

__device__ __forceinline__ uint64_t ld_status(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Called by ONE whole wave (the control wave; no barriers inside).
// Exclusive prefix of tile t = sum of the counts of tiles 0..t-1.  One round
// trip reads 256 predecessors (4 per lane, nearest first); it stops at the
// nearest inclusive prefix and spins only while a nearer predecessor has not
// published its count.  The {flag, count} word is one 8-byte agent-scope
// atomic: the data is the flag.  Bounded: sets *err.
static __device__ uint64_t wave_look_back(const uint64_t *status, uint32_t t, uint32_t *err, uint32_t *nspin = nullptr,
                                   uint32_t *nround = nullptr) {
    const int lane = threadIdx.x & 63;
    uint64_t excl = 0;
    int64_t base = (int64_t)t - 1;
    unsigned spins = 0;
    while (base >= 0) {
        uint64_t s[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t idx = base - (j * 64 + lane);
            s[j] = idx >= 0 ? ld_status(status + idx) : kFlagInc;   // virtual inclusive 0 before tile 0
        }
        int fi = 256, fv = 256;
#pragma unroll
        for (int j = 3; j >= 0; --j) {
            const uint64_t inc = __ballot((s[j] >> 62) == 2), inv = __ballot((s[j] >> 62) == 0);
            if (inc) fi = j * 64 + __ffsll((unsigned long long)inc) - 1;
            if (inv) fv = j * 64 + __ffsll((unsigned long long)inv) - 1;
        }
        if (nround) ++*nround;
        if (fv < fi) {                               // a nearer predecessor has not published yet
            if (nspin) ++*nspin;
            if (++spins > (1u << 22)) {
                if (lane == 0) atomicOr(err, CRDT_DEV_LOOKBACK);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint64_t v = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) v += (j * 64 + lane <= fi) ? (s[j] & kValMask) : 0;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
        excl += v;
        if (fi < 256) break;
        base -= 256;
    }
    return excl;
}

}  // namespace crdt
