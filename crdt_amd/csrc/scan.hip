// scan.hip -- device-wide exclusive scan (uint32 counts -> uint64 offsets).
// Used by the set merges (tile output counts) and RefMerge (inclusion flags).
// Three launches: per-chunk totals, one-block scan of the totals, per-chunk
// rescan + offset.  Chunk = 256 lanes x 8 items.
#include "scan.hpp"

namespace crdt {

constexpr int kScanItems = 8;
constexpr size_t kScanChunk = 256 * kScanItems;

__global__ __launch_bounds__(256) void k_chunk_totals(const uint32_t *__restrict__ in, size_t n,
                                                      uint64_t *__restrict__ totals) {
    const size_t base = (size_t)blockIdx.x * kScanChunk;
    uint64_t s = 0;
#pragma unroll
    for (int u = 0; u < kScanItems; ++u) {
        size_t i = base + (size_t)u * 256 + threadIdx.x;
        if (i < n) s += in[i];
    }
    uint64_t tot;
    block_exclusive_scan_u64(s, &tot);
    if (threadIdx.x == 0) totals[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void k_scan_totals(uint64_t *__restrict__ totals, size_t nb,
                                                     uint64_t *__restrict__ grand) {
    uint64_t carry = 0;
    for (size_t b0 = 0; b0 < nb; b0 += 256) {
        size_t i = b0 + threadIdx.x;
        uint64_t v = i < nb ? totals[i] : 0;
        uint64_t tot;
        uint64_t ex = block_exclusive_scan_u64(v, &tot);
        if (i < nb) totals[i] = carry + ex;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) *grand = carry;
}

__global__ __launch_bounds__(256) void k_chunk_scan(const uint32_t *__restrict__ in, size_t n,
                                                    const uint64_t *__restrict__ offs,
                                                    uint64_t *__restrict__ out) {
    const size_t base = (size_t)blockIdx.x * kScanChunk + (size_t)threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    uint64_t s = 0;
#pragma unroll
    for (int u = 0; u < kScanItems; ++u) {
        size_t i = base + u;
        v[u] = i < n ? in[i] : 0;
        s += v[u];
    }
    uint64_t tot;
    uint64_t run = offs[blockIdx.x] + block_exclusive_scan_u64(s, &tot);
#pragma unroll
    for (int u = 0; u < kScanItems; ++u) {
        size_t i = base + u;
        if (i < n) out[i] = run;
        run += v[u];
    }
}

size_t scan_tmp_bytes(size_t n) {
    size_t nb = (n + kScanChunk - 1) / kScanChunk;
    return Carve::round((nb + 1) * sizeof(uint64_t));
}

int exclusive_scan_u32(crdt_ctx *ctx, const uint32_t *in, uint64_t *out, size_t n, void *tmp) {
    if (n == 0) {
        hipError_t e = hipMemsetAsync(out, 0, sizeof(uint64_t), ctx->stream);
        return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
    }
    const size_t nb = (n + kScanChunk - 1) / kScanChunk;
    if (nb > 0x7fffffffULL) return CRDT_E_RANGE;
    uint64_t *totals = (uint64_t *)tmp;
    k_chunk_totals<<<(unsigned)nb, 256, 0, ctx->stream>>>(in, n, totals);
    k_scan_totals<<<1, 256, 0, ctx->stream>>>(totals, nb, out + n);
    k_chunk_scan<<<(unsigned)nb, 256, 0, ctx->stream>>>(in, n, totals, out);
    return check_launch(ctx);
}

}  // namespace crdt
