// vclock.hip -- vector-clock dominance / concurrency classification.
//
// Build-defined (no reference code): per pair (a, b) of [nodes] uint64 clocks,
//   le = all_k a[k] <= b[k],  ge = all_k a[k] >= b[k]
//   EQUAL if le && ge, BEFORE if le only, AFTER if ge only, else CONCURRENT.
// With nodes == 1 this is the sign of the reference comparator
// (utils.Int64Comparator, main.go:106) applied to unsigned clocks.
//
// Layout: a, b row-major [pairs x nodes].  A pair's row is spread over
// NODES/2 lanes (16 B per lane), so one wave-load of a 128-node clock is the
// whole 1 KiB row; the "for all" is a 64-bit wave ballot.  U pairs-groups
// are loaded before any is reduced (all of a's rows, then all of b's), so
// each lane keeps 2*U 16-B loads in flight -- at U = 32 (the default) 256
// VGPRs, one wave per SIMD and 256 KiB in flight per CU.  HBM-bound:
// 2 * nodes * 8 + 1 bytes per pair.
#include "common.hpp"

namespace crdt {

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint8_t vc_class(bool le, bool ge) {
    return (uint8_t)(le ? (ge ? CRDT_VC_EQUAL : CRDT_VC_BEFORE) : (ge ? CRDT_VC_AFTER : CRDT_VC_CONCURRENT));
}

template <int NODES, int U>
__global__ __launch_bounds__(256) void k_vclock(const u64x2 *__restrict__ a, const u64x2 *__restrict__ b,
                                                uint8_t *__restrict__ cls, size_t pairs) {
    constexpr int LPR = NODES / 2;          // lanes per pair
    constexpr int PPL = kWave / LPR;        // pairs per wave-load
    constexpr int PPW = PPL * U;            // pairs per wave per iteration
    const int lane = threadIdx.x & 63;
    const int sub = lane / LPR, col = lane % LPR;
    const uint64_t gmask = (LPR == 64) ? ~0ULL : ((1ULL << LPR) - 1) << (sub * LPR);
    const size_t wave = ((size_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * 256) >> 6;
    for (size_t p0 = wave * PPW; p0 < pairs; p0 += nwaves * PPW) {
        u64x2 x[U], y[U];
        // all of a's rows, then all of b's: each operand's U rows (U KiB at
        // 128 nodes) one contiguous burst
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t p = p0 + (size_t)u * PPL + sub;
            x[u] = p < pairs ? __builtin_nontemporal_load(a + p * LPR + col) : (u64x2){0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t p = p0 + (size_t)u * PPL + sub;
            y[u] = p < pairs ? __builtin_nontemporal_load(b + p * LPR + col) : (u64x2){0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool nle = (x[u].x > y[u].x) || (x[u].y > y[u].y);   // violates a <= b
            const bool nge = (x[u].x < y[u].x) || (x[u].y < y[u].y);   // violates a >= b
            const uint64_t mnle = __ballot(nle) & gmask;
            const uint64_t mnge = __ballot(nge) & gmask;
            const size_t p = p0 + (size_t)u * PPL + sub;
            if (col == 0 && p < pairs) cls[p] = vc_class(mnle == 0, mnge == 0);
        }
    }
}

// Any node count: one wave per pair, lanes stride over the clock.
__global__ __launch_bounds__(256) void k_vclock_generic(const uint64_t *__restrict__ a,
                                                        const uint64_t *__restrict__ b,
                                                        uint8_t *__restrict__ cls, size_t pairs,
                                                        size_t nodes) {
    const int lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * 256) >> 6;
    for (size_t p = wave; p < pairs; p += nwaves) {
        bool nle = false, nge = false;
        for (size_t k = lane; k < nodes; k += 64) {
            const uint64_t x = a[p * nodes + k], y = b[p * nodes + k];
            nle |= x > y;
            nge |= x < y;
        }
        const bool le = __ballot(nle) == 0, ge = __ballot(nge) == 0;
        if (lane == 0) cls[p] = vc_class(le, ge);
    }
}

template <int NODES>
static void launch_vc(int ppw, unsigned grid, hipStream_t s, const u64x2 *a, const u64x2 *b,
                      uint8_t *c, size_t pairs) {
    switch (ppw) {
        case 1: k_vclock<NODES, 1><<<grid, 256, 0, s>>>(a, b, c, pairs); break;
        case 2: k_vclock<NODES, 2><<<grid, 256, 0, s>>>(a, b, c, pairs); break;
        case 8: k_vclock<NODES, 8><<<grid, 256, 0, s>>>(a, b, c, pairs); break;
        case 16: k_vclock<NODES, 16><<<grid, 256, 0, s>>>(a, b, c, pairs); break;
        case 32: k_vclock<NODES, 32><<<grid, 256, 0, s>>>(a, b, c, pairs); break;
        default: k_vclock<NODES, 4><<<grid, 256, 0, s>>>(a, b, c, pairs); break;
    }
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_vclock_classify(crdt_ctx *ctx, const uint64_t *a, const uint64_t *b, uint8_t *cls,
                                    size_t pairs, size_t nodes) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (nodes == 0 || mul_overflows(pairs, nodes)) return CRDT_E_INVAL;
    if (pairs == 0) return CRDT_OK;
    if (!a || !b || !cls) return CRDT_E_INVAL;
    const bool vec = (((uintptr_t)a | (uintptr_t)b) & 15) == 0;
    const hipStream_t s = ctx->stream;
    const unsigned grid = grid_for(pairs * 64, 256, (unsigned)(ctx->num_cus * g_vclock_blocks_per_cu));
    const u64x2 *va = (const u64x2 *)a, *vb = (const u64x2 *)b;
    const int ppw = g_vclock_pairs_per_wave;
    if (vec && nodes == 128) launch_vc<128>(ppw, grid, s, va, vb, cls, pairs);
    else if (vec && nodes == 64) launch_vc<64>(ppw, grid, s, va, vb, cls, pairs);
    else if (vec && nodes == 32) launch_vc<32>(ppw, grid, s, va, vb, cls, pairs);
    else k_vclock_generic<<<grid, 256, 0, s>>>(a, b, cls, pairs, nodes);
    return check_launch(ctx);
}
