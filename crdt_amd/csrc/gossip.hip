// gossip.hip -- device assembly for anti-entropy rounds.
//
// The reference pulls a random friend's whole Diff over HTTP every round
// (main.go:226-261: GET /gossip -> Diff.ToJSON, decode into RemoteDiff,
// merge).  Here a replica population lives in HBM in the crdt_refmerge_in
// layout and a round is assembled on the device from segmented copies:
//   RemoteDiff of replica p  = the Diff segment of its peer q (entries, then
//                              their kv pairs, slot ids re-based from q's
//                              key slots to p's);
//   the merge                = crdt_refmerge_batch (the bit-exact merge());
//   the next Diff            = the merge's new Diff, its kv pairs gathered by
//                              `src` from the L or R arena.
// One primitive does all of it: a segmented copy with two sources, where
// segment s copies source segment code[s] (>= 0: source A, < 0: source B
// segment -code[s]-1) to dst[dst_off[s]..).  Short segments (kv lists) take
// a thread each, long ones (per-replica entry ranges) a workgroup each.
#include <algorithm>

#include "scan.hpp"

namespace crdt {

__device__ __forceinline__ void seg_src(int64_t c, const uint64_t *a_off, const uint64_t *b_off, uint64_t *b,
                                        uint64_t *e, bool *from_b) {
    *from_b = c < 0;
    const uint64_t k = c < 0 ? (uint64_t)(-(c + 1)) : (uint64_t)c;
    const uint64_t *o = c < 0 ? b_off : a_off;
    *b = o[k];
    *e = o[k + 1];
}

__global__ void k_seg_len(uint64_t n, const int64_t *__restrict__ code, const uint64_t *__restrict__ a_off,
                          const uint64_t *__restrict__ b_off, uint32_t *__restrict__ len) {
    for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < n; s += (uint64_t)gridDim.x * 256) {
        uint64_t b, e;
        bool fb;
        seg_src(code[s], a_off, b_off, &b, &e, &fb);
        len[s] = e > b ? (uint32_t)(e - b) : 0u;
    }
}

__global__ void k_add_base(uint64_t *__restrict__ v, uint64_t n, uint64_t base) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) v[i] += base;
}

__global__ void k_off_to_counts(const uint64_t *__restrict__ off, uint64_t n, uint32_t *__restrict__ cnt) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        cnt[i] = (uint32_t)(off[i + 1] - off[i]);
}

// dst[x] = src[x] (+ delta[s] for 4-byte elements when delta != nullptr)
template <typename T>
__device__ __forceinline__ T add_delta(T x, const uint32_t *delta, uint64_t s) {
    if constexpr (sizeof(T) == 4) return delta ? (T)((uint32_t)x + delta[s]) : x;
    return x;
}

template <typename T>
__global__ void k_seg_copy_thread(uint64_t n, const int64_t *__restrict__ code, const uint64_t *__restrict__ a_off,
                                  const uint64_t *__restrict__ b_off, const uint64_t *__restrict__ dst_off,
                                  const T *__restrict__ a, const T *__restrict__ b, T *__restrict__ dst,
                                  const uint32_t *__restrict__ delta) {
    for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < n; s += (uint64_t)gridDim.x * 256) {
        uint64_t sb, se;
        bool fb;
        seg_src(code[s], a_off, b_off, &sb, &se, &fb);
        const T *src = fb ? b : a;
        const uint64_t o = dst_off[s];
        for (uint64_t i = sb; i < se; ++i) dst[o + (i - sb)] = add_delta(src[i], delta, s);
    }
}

// long segments (per-replica entry ranges): a whole workgroup per segment
template <typename T>
__global__ void k_seg_copy_block(uint64_t n, const int64_t *__restrict__ code, const uint64_t *__restrict__ a_off,
                                 const uint64_t *__restrict__ b_off, const uint64_t *__restrict__ dst_off,
                                 const T *__restrict__ a, const T *__restrict__ b, T *__restrict__ dst,
                                 const uint32_t *__restrict__ delta) {
    for (uint64_t s = blockIdx.x; s < n; s += gridDim.x) {
        uint64_t sb, se;
        bool fb;
        seg_src(code[s], a_off, b_off, &sb, &se, &fb);
        const T *src = fb ? b : a;
        const uint64_t o = dst_off[s];
        for (uint64_t i = sb + threadIdx.x; i < se; i += 256) dst[o + (i - sb)] = add_delta(src[i], delta, s);
    }
}

__global__ void k_seg_fill_u32(uint64_t n, const uint64_t *__restrict__ dst_off, const uint32_t *__restrict__ val,
                               uint32_t *__restrict__ dst) {
    const int lane = threadIdx.x & 63;
    for (uint64_t s = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6; s < n; s += ((uint64_t)gridDim.x * 256) >> 6) {
        const uint32_t v = val[s];
        for (uint64_t i = dst_off[s] + lane; i < dst_off[s + 1]; i += 64) dst[i] = v;
    }
}

template <typename T>
static void launch_copy(crdt_ctx *ctx, uint64_t n, const int64_t *code, const uint64_t *a_off, const uint64_t *b_off,
                        const uint64_t *dst_off, const void *a, const void *b, void *dst, const uint32_t *delta,
                        int wide) {
    const unsigned cap = (unsigned)ctx->num_cus * 8;
    if (wide)
        k_seg_copy_block<T><<<(unsigned)std::min<uint64_t>(n, 65535), 256, 0, ctx->stream>>>(
            n, code, a_off, b_off, dst_off, (const T *)a, (const T *)b, (T *)dst, delta);
    else
        k_seg_copy_thread<T><<<grid_for(n, 256, cap), 256, 0, ctx->stream>>>(
            n, code, a_off, b_off, dst_off, (const T *)a, (const T *)b, (T *)dst, delta);
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_counts_to_offsets(crdt_ctx *ctx, const uint32_t *counts, size_t n, uint64_t base,
                                      uint64_t *off) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!off || (n && !counts)) return CRDT_E_INVAL;
    rc = ws_reserve(ctx, scan_tmp_bytes(n) + 4096);
    if (rc) return rc;
    Carve w(ctx->ws);
    void *tmp = w.take<char>(scan_tmp_bytes(n));
    rc = exclusive_scan_u32(ctx, counts, off, n, tmp);           // off[n] = total
    if (rc) return rc;
    if (base) k_add_base<<<grid_for(n + 1, 256, (unsigned)ctx->num_cus * 8), 256, 0, ctx->stream>>>(off, n + 1, base);
    return check_launch(ctx);
}

extern "C" int crdt_offsets_to_counts(crdt_ctx *ctx, const uint64_t *off, size_t n, uint32_t *counts) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (n == 0) return CRDT_OK;
    if (!off || !counts) return CRDT_E_INVAL;
    k_off_to_counts<<<grid_for(n, 256, (unsigned)ctx->num_cus * 8), 256, 0, ctx->stream>>>(off, n, counts);
    return check_launch(ctx);
}

extern "C" int crdt_seg_offsets(crdt_ctx *ctx, size_t n_seg, const int64_t *code, const uint64_t *a_off,
                                const uint64_t *b_off, uint64_t base, uint64_t *dst_off) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!dst_off || (n_seg && (!code || !a_off))) return CRDT_E_INVAL;
    rc = ws_reserve(ctx, Carve::round(n_seg * 4 + 4) + scan_tmp_bytes(n_seg) + 4096);
    if (rc) return rc;
    Carve w(ctx->ws);
    uint32_t *len = w.take<uint32_t>(n_seg + 1);
    void *tmp = w.take<char>(scan_tmp_bytes(n_seg));
    if (n_seg)
        k_seg_len<<<grid_for(n_seg, 256, (unsigned)ctx->num_cus * 8), 256, 0, ctx->stream>>>(n_seg, code, a_off,
                                                                                            b_off, len);
    rc = exclusive_scan_u32(ctx, len, dst_off, n_seg, tmp);
    if (rc) return rc;
    if (base)
        k_add_base<<<grid_for(n_seg + 1, 256, (unsigned)ctx->num_cus * 8), 256, 0, ctx->stream>>>(dst_off, n_seg + 1,
                                                                                                 base);
    return check_launch(ctx);
}

extern "C" int crdt_seg_copy(crdt_ctx *ctx, size_t n_seg, const int64_t *code, const uint64_t *a_off,
                             const uint64_t *b_off, const uint64_t *dst_off, size_t elem_size, const void *a,
                             const void *b, void *dst, const uint32_t *delta, int wide) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (n_seg == 0) return CRDT_OK;
    if (!code || !a_off || !dst_off || !dst) return CRDT_E_INVAL;
    if (delta && elem_size != 4) return CRDT_E_INVAL;
    switch (elem_size) {
        case 1: launch_copy<uint8_t>(ctx, n_seg, code, a_off, b_off, dst_off, a, b, dst, nullptr, wide); break;
        case 4: launch_copy<uint32_t>(ctx, n_seg, code, a_off, b_off, dst_off, a, b, dst, delta, wide); break;
        case 8: launch_copy<uint64_t>(ctx, n_seg, code, a_off, b_off, dst_off, a, b, dst, nullptr, wide); break;
        default: return CRDT_E_INVAL;
    }
    return check_launch(ctx);
}

extern "C" int crdt_seg_fill_u32(crdt_ctx *ctx, size_t n_seg, const uint64_t *dst_off, const uint32_t *val,
                                 uint32_t *dst) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (n_seg == 0) return CRDT_OK;
    if (!dst_off || !val || !dst) return CRDT_E_INVAL;
    k_seg_fill_u32<<<grid_for(n_seg * 64, 256, (unsigned)ctx->num_cus * 8), 256, 0, ctx->stream>>>(n_seg, dst_off, val,
                                                                                                   dst);
    return check_launch(ctx);
}
