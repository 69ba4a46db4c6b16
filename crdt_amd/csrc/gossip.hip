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
// a thread each, long ones (per-replica entry and kv ranges) a workgroup
// each; one pass can move two arrays (kv keys and values) by the same map.
// The pulled kv pairs of replica p are the contiguous kv range of q's
// entries, so R's kv offsets are q's offsets plus one per-replica delta and
// the assembly needs no per-entry scan.
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

__global__ void k_off_to_counts(const uint64_t *__restrict__ off, uint64_t n, uint32_t *__restrict__ cnt) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        cnt[i] = (uint32_t)(off[i + 1] - off[i]);
}

// One or two arrays moved by the same segment map; every element of segment s
// of array 0 gets + delta[s] (mod 2^(8*sizeof(T)): key-slot and kv-offset
// re-basing), array 1 is copied verbatim.
template <typename T>
struct SegArrays {
    const T *a0, *b0;
    T *d0;
    const T *delta;
    const T *a1, *b1;
    T *d1;
};

// short segments (kv lists): one thread per segment
template <typename T, bool kTwo>
__global__ void k_seg_copy_thread(uint64_t n, const int64_t *__restrict__ code, const uint64_t *__restrict__ a_off,
                                  const uint64_t *__restrict__ b_off, const uint64_t *__restrict__ dst_off,
                                  SegArrays<T> p) {
    for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < n; s += (uint64_t)gridDim.x * 256) {
        uint64_t sb, se;
        bool fb;
        seg_src(code[s], a_off, b_off, &sb, &se, &fb);
        const T *s0 = fb ? p.b0 : p.a0;
        const T *s1 = fb ? p.b1 : p.a1;
        const T dl = p.delta ? p.delta[s] : (T)0;
        const uint64_t o = dst_off[s] - sb;
        for (uint64_t i = sb; i < se; ++i) {
            p.d0[o + i] = (T)(s0[i] + dl);
            if constexpr (kTwo) p.d1[o + i] = s1[i];
        }
    }
}

// long segments (per-replica entry and kv ranges): `parts` workgroups per segment
template <typename T, bool kTwo>
__global__ void k_seg_copy_block(uint64_t n, const int64_t *__restrict__ code, const uint64_t *__restrict__ a_off,
                                 const uint64_t *__restrict__ b_off, const uint64_t *__restrict__ dst_off,
                                 SegArrays<T> p, uint32_t parts) {
    for (uint64_t g = blockIdx.x; g < n * parts; g += gridDim.x) {
        const uint64_t s = g / parts, part = g % parts;
        uint64_t sb, se;
        bool fb;
        seg_src(code[s], a_off, b_off, &sb, &se, &fb);
        const T *s0 = fb ? p.b0 : p.a0;
        const T *s1 = fb ? p.b1 : p.a1;
        const T dl = p.delta ? p.delta[s] : (T)0;
        const uint64_t o = dst_off[s] - sb;
        T *__restrict__ d0 = p.d0;
        T *__restrict__ d1 = p.d1;
        const uint64_t st = (uint64_t)parts * 256;
        uint64_t i = sb + part * 256 + threadIdx.x;
        // U elements per thread in flight before the first store (a load /
        // store per element in turn waited on one HBM round trip each)
        constexpr int U = 4;
        for (; i + (U - 1) * st < se; i += U * st) {
            T x[U], y[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                x[k] = s0[i + k * st];
                if constexpr (kTwo) y[k] = s1[i + k * st];
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {
                d0[o + i + k * st] = (T)(x[k] + dl);
                if constexpr (kTwo) d1[o + i + k * st] = y[k];
            }
        }
        for (; i < se; i += st) {
            d0[o + i] = (T)(s0[i] + dl);
            if constexpr (kTwo) d1[o + i] = s1[i];
        }
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
                        const uint64_t *dst_off, const void *a0, const void *b0, void *d0, const void *delta,
                        const void *a1, const void *b1, void *d1, int wide) {
    const SegArrays<T> p{(const T *)a0, (const T *)b0, (T *)d0, (const T *)delta,
                         (const T *)a1, (const T *)b1, (T *)d1};
    const unsigned cap = (unsigned)ctx->num_cus * 8;
    // enough workgroups to fill the chip: a few long segments split into parts
    const uint32_t parts = (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(1, (cap + n - 1) / n));
    const unsigned gb = (unsigned)std::min<uint64_t>(n * parts, 65535);
    if (wide && d1)
        k_seg_copy_block<T, true><<<gb, 256, 0, ctx->stream>>>(n, code, a_off, b_off, dst_off, p, parts);
    else if (wide)
        k_seg_copy_block<T, false><<<gb, 256, 0, ctx->stream>>>(n, code, a_off, b_off, dst_off, p, parts);
    else if (d1)
        k_seg_copy_thread<T, true><<<grid_for(n, 256, cap), 256, 0, ctx->stream>>>(n, code, a_off, b_off, dst_off, p);
    else
        k_seg_copy_thread<T, false><<<grid_for(n, 256, cap), 256, 0, ctx->stream>>>(n, code, a_off, b_off, dst_off, p);
}

static int seg_copy_any(crdt_ctx *ctx, size_t n_seg, const int64_t *code, const uint64_t *a_off,
                        const uint64_t *b_off, const uint64_t *dst_off, size_t elem_size, const void *a0,
                        const void *b0, void *d0, const void *delta, const void *a1, const void *b1, void *d1,
                        int wide) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (n_seg == 0) return CRDT_OK;
    if (!code || !a_off || !dst_off || !a0 || !d0 || (d1 && !a1)) return CRDT_E_INVAL;
    switch (elem_size) {
        case 1: launch_copy<uint8_t>(ctx, n_seg, code, a_off, b_off, dst_off, a0, b0, d0, delta, a1, b1, d1, wide); break;
        case 4: launch_copy<uint32_t>(ctx, n_seg, code, a_off, b_off, dst_off, a0, b0, d0, delta, a1, b1, d1, wide); break;
        case 8: launch_copy<uint64_t>(ctx, n_seg, code, a_off, b_off, dst_off, a0, b0, d0, delta, a1, b1, d1, wide); break;
        default: return CRDT_E_INVAL;
    }
    return check_launch(ctx);
}

// scan_lb source: segment s's length and where it starts (gossip assembly)
struct SegSrc {
    const int64_t *code;
    const uint64_t *a_off, *b_off;
    const uint64_t *n_dev = nullptr;      // (optional) segments >= *n_dev are empty: a device-side count
    struct Item {
        uint64_t len = 0, sb = 0;
        bool fb = false;
    };
    __device__ Item load(uint64_t s) const {
        if (n_dev && s >= *n_dev) return Item{};
        uint64_t b, e;
        bool fb;
        seg_src(code[s], a_off, b_off, &b, &e, &fb);
        return Item{e > b ? e - b : 0, b, fb};
    }
};

// scan_lb action: copy the segment to its freshly scanned offset (one thread
// per segment: kv lists), array 1 alongside when kTwo
template <typename T, bool kTwo>
struct SegCopyAct {
    SegArrays<T> p;
    template <int N>
    __device__ void apply(const SegSrc::Item *it, const uint64_t *d) const {
        // first element of every segment: all loads in flight, then the stores
        T x0[N], x1[N];
#pragma unroll
        for (int r = 0; r < N; ++r) {
            if (it[r].len) {
                x0[r] = (it[r].fb ? p.b0 : p.a0)[it[r].sb];
                if constexpr (kTwo) x1[r] = (it[r].fb ? p.b1 : p.a1)[it[r].sb];
            }
        }
#pragma unroll
        for (int r = 0; r < N; ++r) {
            if (it[r].len) {
                p.d0[d[r]] = x0[r];
                if constexpr (kTwo) p.d1[d[r]] = x1[r];
            }
        }
        // the rest of longer kv lists
#pragma unroll
        for (int r = 0; r < N; ++r) {
            const T *s0 = it[r].fb ? p.b0 : p.a0;
            const T *s1 = it[r].fb ? p.b1 : p.a1;
            for (uint64_t j = 1; j < it[r].len; ++j) {
                p.d0[d[r] + j] = s0[it[r].sb + j];
                if constexpr (kTwo) p.d1[d[r] + j] = s1[it[r].sb + j];
            }
        }
    }
};

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_counts_to_offsets(crdt_ctx *ctx, const uint32_t *counts, size_t n, uint64_t base,
                                      uint64_t *off) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!off || (n && !counts)) return CRDT_E_INVAL;
    rc = ws_reserve(ctx, scan_lb_tmp_bytes(n) + 4096);
    if (rc) return rc;
    return scan_lb(ctx, CountSrc{counts}, NoAct{}, n, base, off, ctx->ws);      // off[n] = base + total
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
    rc = ws_reserve(ctx, scan_lb_tmp_bytes(n_seg) + 4096);
    if (rc) return rc;
    return scan_lb(ctx, SegSrc{code, a_off, b_off}, NoAct{}, n_seg, base, dst_off, ctx->ws);
}

template <typename T>
static int seg_gather(crdt_ctx *ctx, size_t n_seg, const int64_t *code, const uint64_t *a_off, const uint64_t *b_off,
                      uint64_t base, uint64_t *dst_off, const void *a0, const void *b0, void *d0, const void *a1,
                      const void *b1, void *d1, const uint64_t *n_dev = nullptr) {
    const SegArrays<T> p{(const T *)a0, (const T *)b0, (T *)d0, nullptr, (const T *)a1, (const T *)b1, (T *)d1};
    const SegSrc src{code, a_off, b_off, n_dev};
    if (d1) return scan_lb(ctx, src, SegCopyAct<T, true>{p}, n_seg, base, dst_off, ctx->ws);
    return scan_lb(ctx, src, SegCopyAct<T, false>{p}, n_seg, base, dst_off, ctx->ws);
}

extern "C" int crdt_seg_gather2(crdt_ctx *ctx, size_t n_seg, const int64_t *code, const uint64_t *a_off,
                                const uint64_t *b_off, uint64_t base, uint64_t *dst_off, size_t elem_size,
                                const void *a0, const void *b0, void *dst0, const void *a1, const void *b1,
                                void *dst1) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!dst_off || (n_seg && (!code || !a_off || !a0 || !dst0 || (dst1 && !a1)))) return CRDT_E_INVAL;
    rc = ws_reserve(ctx, scan_lb_tmp_bytes(n_seg) + 4096);
    if (rc) return rc;
    switch (elem_size) {
        case 1: return seg_gather<uint8_t>(ctx, n_seg, code, a_off, b_off, base, dst_off, a0, b0, dst0, a1, b1, dst1);
        case 4: return seg_gather<uint32_t>(ctx, n_seg, code, a_off, b_off, base, dst_off, a0, b0, dst0, a1, b1, dst1);
        case 8: return seg_gather<uint64_t>(ctx, n_seg, code, a_off, b_off, base, dst_off, a0, b0, dst0, a1, b1, dst1);
        default: return CRDT_E_INVAL;
    }
}

// crdt_seg_gather2 over n_max segments of which only the first *n_dev (a
// count still on the device, <= n_max) are real: the rest scan as empty, so
// dst_off[i] = base + total for every i in [*n_dev, n_max].  Lets a caller
// launch the gather behind the kernel that produces the count, without a
// host round trip for it (the batched Server.merge()).
int crdt::seg_gather2_dev_count(crdt_ctx *ctx, size_t n_max, const uint64_t *n_dev, const int64_t *code,
                                 const uint64_t *a_off, const uint64_t *b_off, uint64_t *dst_off, const uint32_t *a0,
                          const uint32_t *b0, uint32_t *dst0, const uint32_t *a1, const uint32_t *b1, uint32_t *dst1) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!dst_off || !n_dev || (n_max && (!code || !a_off || !a0 || !dst0 || (dst1 && !a1)))) return CRDT_E_INVAL;
    rc = ws_reserve(ctx, scan_lb_tmp_bytes(n_max) + 4096);
    if (rc) return rc;
    return seg_gather<uint32_t>(ctx, n_max, code, a_off, b_off, 0, dst_off, a0, b0, dst0, a1, b1, dst1, n_dev);
}

extern "C" int crdt_seg_gather2_n(crdt_ctx *ctx, size_t n_max, const uint64_t *n_dev, const int64_t *code,
                                  const uint64_t *a_off, const uint64_t *b_off, uint64_t *dst_off, const uint32_t *a0,
                                  const uint32_t *b0, uint32_t *dst0, const uint32_t *a1, const uint32_t *b1,
                                  uint32_t *dst1) {
    return crdt::seg_gather2_dev_count(ctx, n_max, n_dev, code, a_off, b_off, dst_off, a0, b0, dst0, a1, b1, dst1);
}

extern "C" int crdt_seg_copy(crdt_ctx *ctx, size_t n_seg, const int64_t *code, const uint64_t *a_off,
                             const uint64_t *b_off, const uint64_t *dst_off, size_t elem_size, const void *a,
                             const void *b, void *dst, const uint32_t *delta, int wide) {
    if (delta && elem_size != 4) return CRDT_E_INVAL;
    return seg_copy_any(ctx, n_seg, code, a_off, b_off, dst_off, elem_size, a, b, dst, delta, nullptr, nullptr,
                        nullptr, wide);
}

extern "C" int crdt_seg_copy2(crdt_ctx *ctx, size_t n_seg, const int64_t *code, const uint64_t *a_off,
                              const uint64_t *b_off, const uint64_t *dst_off, size_t elem_size, const void *a0,
                              const void *b0, void *dst0, const void *delta0, const void *a1, const void *b1,
                              void *dst1, int wide) {
    return seg_copy_any(ctx, n_seg, code, a_off, b_off, dst_off, elem_size, a0, b0, dst0, delta0, a1, b1, dst1,
                        wide);
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
