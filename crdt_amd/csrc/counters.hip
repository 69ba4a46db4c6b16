// counters.hip -- G-Counter / PN-Counter / vector-clock join kernels.
//
// No reference code exists for these types: they are the
// standard state-based CRDT joins (elementwise unsigned max) over a replica
// population stored row-major [rows x nodes] uint64 in HBM.  Everything here
// is HBM-bound integer streaming: 16-byte (dwordx4) loads per lane, several
// independent loads in flight per lane, no LDS, no MFMA.
#include "common.hpp"

namespace crdt {

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

template <bool NT> __device__ __forceinline__ u64x2 ld(const u64x2 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT> __device__ __forceinline__ void st(u64x2 *p, u64x2 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
__device__ __forceinline__ u64x2 vmax(u64x2 x, u64x2 y) {
    return __builtin_elementwise_max(x, y);  // unsigned 64-bit max per lane
}

// out = max(a, b) elementwise over n2 16-byte vectors.  Grid-stride: at each
// step the whole grid touches one contiguous window of U * grid * 4 KiB.
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_join(const u64x2 *__restrict__ a,
                                              const u64x2 *__restrict__ b,
                                              u64x2 *__restrict__ o, size_t n2) {
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (size_t)(U - 1) * stride < n2; i += (size_t)U * stride) {
        u64x2 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld<NT>(a + i + (size_t)u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) y[u] = ld<NT>(b + i + (size_t)u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(o + i + (size_t)u * stride, vmax(x[u], y[u]));
    }
    for (; i < n2; i += stride) st<NT>(o + i, vmax(ld<NT>(a + i), ld<NT>(b + i)));
}

// Scalar tail (odd element count).
__global__ void k_join_tail(const uint64_t *a, const uint64_t *b, uint64_t *o, size_t idx) {
    uint64_t x = a[idx], y = b[idx];
    o[idx] = x > y ? x : y;
}

// ---------------------------------------------------------------- fold
// Column max over rows.  Fast path: nodes a power of two in [2, 512], so a
// 256-lane block covers 512 uint64 = 512/nodes whole rows per load and every
// lane keeps the same column pair for the whole grid-stride loop.
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_fold_pow2(const u64x2 *__restrict__ a, size_t n2,
                                                   int nodes, uint64_t *__restrict__ partial) {
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    u64x2 m = {0, 0};
    for (; i + (size_t)(U - 1) * stride < n2; i += (size_t)U * stride) {
        u64x2 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld<NT>(a + i + (size_t)u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) m = vmax(m, x[u]);
    }
    for (; i < n2; i += stride) m = vmax(m, ld<NT>(a + i));
    __shared__ u64x2 red[256];
    red[threadIdx.x] = m;
    __syncthreads();
    const int lanes_per_row = nodes >> 1;          // vectors per row
    if ((int)threadIdx.x < lanes_per_row) {
        u64x2 r = red[threadIdx.x];
        for (int t = threadIdx.x + lanes_per_row; t < 256; t += lanes_per_row) r = vmax(r, red[t]);
        partial[(size_t)blockIdx.x * nodes + 2 * threadIdx.x] = r.x;
        partial[(size_t)blockIdx.x * nodes + 2 * threadIdx.x + 1] = r.y;
    }
}

// Generic nodes: lanes stride over columns, blocks over rows.
__global__ __launch_bounds__(256) void k_fold_generic(const uint64_t *__restrict__ a, size_t rows,
                                                      size_t nodes, uint64_t *__restrict__ partial) {
    for (size_t c = threadIdx.x; c < nodes; c += 256) {
        uint64_t m = 0;
        for (size_t r = blockIdx.x; r < rows; r += gridDim.x) {
            uint64_t v = a[r * nodes + c];
            m = v > m ? v : m;
        }
        partial[(size_t)blockIdx.x * nodes + c] = m;
    }
}

// partial [g x nodes] -> out[nodes] via unsigned 64-bit atomicMax (out pre-zeroed).
__global__ __launch_bounds__(256) void k_fold_finish(const uint64_t *__restrict__ partial, size_t g,
                                                     size_t nodes, uint64_t *__restrict__ out) {
    for (size_t c = threadIdx.x; c < nodes; c += 256) {
        uint64_t m = 0;
        for (size_t r = blockIdx.x; r < g; r += gridDim.x) {
            uint64_t v = partial[r * nodes + c];
            m = v > m ? v : m;
        }
        if (m) atomicMax((unsigned long long *)&out[c], (unsigned long long)m);
    }
}

// ---------------------------------------------------------------- row sums
// out[r] = sum_n a[r][n] (- sum_n n[r][n] for PN), uint64 wrap.  NODES/2 lanes
// per row (16 B each), 64/(NODES/2) rows per wave-load, butterfly reduction
// inside the row's lane group.
template <int NODES, bool PN>
__global__ __launch_bounds__(256) void k_rowsum(const u64x2 *__restrict__ p,
                                                const u64x2 *__restrict__ n, uint64_t *__restrict__ out,
                                                size_t rows) {
    constexpr int LPR = NODES / 2;               // lanes per row
    constexpr int RPW = kWave / LPR;             // rows per wave per step
    const int lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * 256) >> 6;
    const int sub = lane / LPR, col = lane % LPR;
    for (size_t r0 = wave * RPW; r0 < rows; r0 += nwaves * RPW) {
        const size_t r = r0 + sub;
        uint64_t s = 0;
        if (r < rows) {
            u64x2 v = ld<true>(p + r * LPR + col);
            s = v.x + v.y;
            if constexpr (PN) {
                u64x2 w = ld<true>(n + r * LPR + col);
                s -= w.x + w.y;
            }
        }
#pragma unroll
        for (int m = LPR / 2; m >= 1; m >>= 1) s += __shfl_xor(s, m, LPR);
        if (col == 0 && r < rows) out[r] = s;
    }
}

// Generic nodes: one wave per row, lanes stride over columns.
template <bool PN>
__global__ __launch_bounds__(256) void k_rowsum_generic(const uint64_t *__restrict__ p,
                                                        const uint64_t *__restrict__ n,
                                                        uint64_t *__restrict__ out, size_t rows,
                                                        size_t nodes) {
    const int lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * 256) >> 6;
    for (size_t r = wave; r < rows; r += nwaves) {
        uint64_t s = 0;
        for (size_t c = lane; c < nodes; c += 64) {
            s += p[r * nodes + c];
            if constexpr (PN) s -= n[r * nodes + c];
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
        if (lane == 0) out[r] = s;
    }
}

// ---------------------------------------------------------------- order maps
__global__ void k_u64_to_i64(const uint64_t *in, int64_t *out, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        out[i] = (int64_t)(in[i] ^ 0x8000000000000000ULL);
}
__global__ void k_i64_to_u64(const int64_t *in, uint64_t *out, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        out[i] = (uint64_t)in[i] ^ 0x8000000000000000ULL;
}

// ---------------------------------------------------------------- launchers
template <int U, bool NT>
static void launch_join(unsigned grid, hipStream_t s, const u64x2 *a, const u64x2 *b, u64x2 *o,
                        size_t n2) {
    k_join<U, NT><<<grid, 256, 0, s>>>(a, b, o, n2);
}

static int join_impl(crdt_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *o, size_t n) {
    const size_t n2 = n / 2;
    const unsigned grid = grid_for(n2, 256, (unsigned)(ctx->num_cus * g_join_blocks_per_cu));
    const hipStream_t s = ctx->stream;
    if (n2) {
        const u64x2 *va = (const u64x2 *)a, *vb = (const u64x2 *)b;
        u64x2 *vo = (u64x2 *)o;
        const bool nt = g_join_nontemporal != 0;
        switch (g_join_unroll) {
            case 1: nt ? launch_join<1, true>(grid, s, va, vb, vo, n2) : launch_join<1, false>(grid, s, va, vb, vo, n2); break;
            case 2: nt ? launch_join<2, true>(grid, s, va, vb, vo, n2) : launch_join<2, false>(grid, s, va, vb, vo, n2); break;
            case 8: nt ? launch_join<8, true>(grid, s, va, vb, vo, n2) : launch_join<8, false>(grid, s, va, vb, vo, n2); break;
            default: nt ? launch_join<4, true>(grid, s, va, vb, vo, n2) : launch_join<4, false>(grid, s, va, vb, vo, n2); break;
        }
    }
    if (n & 1) k_join_tail<<<1, 1, 0, s>>>(a, b, o, n - 1);
    return check_launch(ctx);
}

// ---------------------------------------------------------------- streaming peaks
// the bench reports each kernel's fraction of a SELF-MEASURED
// copy-kernel peak beside the 8 TB/s spec.  A plain copy (16-B loads and
// stores, U vectors in flight per lane) and a read-only sweep (xor-reduced
// over the workgroup, one store per workgroup) of the same form as the join / fold loops.
template <int U>
__global__ __launch_bounds__(256) void k_stream_copy(const u64x2 *__restrict__ a, u64x2 *__restrict__ o, size_t n2) {
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (size_t)(U - 1) * stride < n2; i += (size_t)U * stride) {
        u64x2 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld<true>(a + i + (size_t)u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) st<true>(o + i + (size_t)u * stride, x[u]);
    }
    for (; i < n2; i += stride) st<true>(o + i, ld<true>(a + i));
}

template <int U>
__global__ __launch_bounds__(256) void k_stream_read(const u64x2 *__restrict__ a, size_t n2,
                                                     uint64_t *__restrict__ sink) {
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    u64x2 m = {0, 0};
    for (; i + (size_t)(U - 1) * stride < n2; i += (size_t)U * stride) {
        u64x2 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld<true>(a + i + (size_t)u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) m ^= x[u];
    }
    for (; i < n2; i += stride) m ^= ld<true>(a + i);
    // xor over the workgroup (every lane's loads feed the stored word)
    uint64_t v = m.x ^ m.y;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o);
    __shared__ uint64_t red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) sink[blockIdx.x] = red[0] ^ red[1] ^ red[2] ^ red[3];
}

}  // namespace crdt

using namespace crdt;

static bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

extern "C" int crdt_stream_copy(crdt_ctx *ctx, const void *src, void *dst, size_t bytes, int unroll,
                                int blocks_per_cu) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!src || !dst || !aligned16(src) || !aligned16(dst) || (bytes & 15)) return CRDT_E_INVAL;
    if (blocks_per_cu < 1 || blocks_per_cu > 64) return CRDT_E_INVAL;
    const size_t n2 = bytes / 16;
    if (n2 == 0) return CRDT_OK;
    const unsigned grid = grid_for(n2, 256, (unsigned)(ctx->num_cus * blocks_per_cu));
    const u64x2 *a = (const u64x2 *)src;
    u64x2 *o = (u64x2 *)dst;
    const hipStream_t s = ctx->stream;
    switch (unroll) {
        case 1: k_stream_copy<1><<<grid, 256, 0, s>>>(a, o, n2); break;
        case 2: k_stream_copy<2><<<grid, 256, 0, s>>>(a, o, n2); break;
        case 4: k_stream_copy<4><<<grid, 256, 0, s>>>(a, o, n2); break;
        case 8: k_stream_copy<8><<<grid, 256, 0, s>>>(a, o, n2); break;
        default: return CRDT_E_INVAL;
    }
    return check_launch(ctx);
}

extern "C" int crdt_stream_read(crdt_ctx *ctx, const void *src, size_t bytes, uint64_t *sink_dev, size_t sink_words,
                                int unroll, int blocks_per_cu) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!src || !sink_dev || !aligned16(src) || (bytes & 15)) return CRDT_E_INVAL;
    if (blocks_per_cu < 1 || blocks_per_cu > 64) return CRDT_E_INVAL;
    const size_t n2 = bytes / 16;
    if (n2 == 0) return CRDT_OK;
    const unsigned grid = grid_for(n2, 256, (unsigned)(ctx->num_cus * blocks_per_cu));
    if (sink_words < grid) return CRDT_E_INVAL;         // one word per workgroup
    const u64x2 *a = (const u64x2 *)src;
    const hipStream_t s = ctx->stream;
    switch (unroll) {
        case 1: k_stream_read<1><<<grid, 256, 0, s>>>(a, n2, sink_dev); break;
        case 2: k_stream_read<2><<<grid, 256, 0, s>>>(a, n2, sink_dev); break;
        case 4: k_stream_read<4><<<grid, 256, 0, s>>>(a, n2, sink_dev); break;
        case 8: k_stream_read<8><<<grid, 256, 0, s>>>(a, n2, sink_dev); break;
        default: return CRDT_E_INVAL;
    }
    return check_launch(ctx);
}

extern "C" int crdt_gcounter_join(crdt_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *out,
                                  size_t rows, size_t nodes) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (mul_overflows(rows, nodes)) return CRDT_E_INVAL;
    const size_t n = rows * nodes;
    if (n == 0) return CRDT_OK;
    if (!a || !b || !out || !aligned16(a) || !aligned16(b) || !aligned16(out)) return CRDT_E_INVAL;
    return join_impl(ctx, a, b, out, n);
}

extern "C" int crdt_pncounter_join(crdt_ctx *ctx, const uint64_t *pa, const uint64_t *na,
                                   const uint64_t *pb, const uint64_t *nb, uint64_t *po,
                                   uint64_t *no, size_t rows, size_t nodes) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (mul_overflows(rows, nodes)) return CRDT_E_INVAL;
    const size_t n = rows * nodes;
    if (n == 0) return CRDT_OK;
    const void *ps[6] = {pa, na, pb, nb, po, no};
    for (const void *p : ps)
        if (!p || !aligned16(p)) return CRDT_E_INVAL;
    // the P and N halves as two passes of the tuned G-Counter join: a fused
    // single pass keeps four 16-B loads per lane in flight, past the ~16 KiB
    // per CU the HBM system prefers (measured 65% vs 80% of peak)
    rc = join_impl(ctx, pa, pb, po, n);
    if (rc) return rc;
    return join_impl(ctx, na, nb, no, n);
}

extern "C" int crdt_gcounter_fold(crdt_ctx *ctx, const uint64_t *a, size_t rows, size_t nodes,
                                  uint64_t *out) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!out || nodes == 0 || mul_overflows(rows, nodes)) return CRDT_E_INVAL;
    hipError_t e = hipMemsetAsync(out, 0, nodes * sizeof(uint64_t), ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
    if (rows == 0) return CRDT_OK;
    if (!a) return CRDT_E_INVAL;
    const bool pow2 = nodes >= 2 && nodes <= 512 && (nodes & (nodes - 1)) == 0 && aligned16(a);
    unsigned grid;
    const unsigned bpc = (unsigned)g_fold_blocks_per_cu;
    if (pow2) grid = grid_for(rows * nodes / 2, 256 * (unsigned)g_fold_unroll, (unsigned)ctx->num_cus * bpc);
    else grid = grid_for(rows, 1, (unsigned)(ctx->num_cus * 4));
    const size_t part_bytes = (size_t)grid * nodes * sizeof(uint64_t);
    rc = ws_reserve(ctx, part_bytes);
    if (rc) return rc;
    uint64_t *partial = (uint64_t *)ctx->ws;
    if (pow2) {
        const u64x2 *va = (const u64x2 *)a;
        const size_t n2 = rows * nodes / 2;
        const hipStream_t s = ctx->stream;
        const bool nt = g_fold_nontemporal != 0;
#define FOLD(U) (nt ? k_fold_pow2<U, true><<<grid, 256, 0, s>>>(va, n2, (int)nodes, partial) \
                    : k_fold_pow2<U, false><<<grid, 256, 0, s>>>(va, n2, (int)nodes, partial))
        switch (g_fold_unroll) {
            case 1: FOLD(1); break;
            case 2: FOLD(2); break;
            case 8: FOLD(8); break;
            case 16: FOLD(16); break;
            default: FOLD(4); break;
        }
#undef FOLD
    } else {
        k_fold_generic<<<grid, 256, 0, ctx->stream>>>(a, rows, nodes, partial);
    }
    rc = check_launch(ctx);
    if (rc) return rc;
    const unsigned g2 = grid < 32 ? grid : 32;
    k_fold_finish<<<g2, 256, 0, ctx->stream>>>(partial, grid, nodes, out);
    return check_launch(ctx);
}

template <bool PN>
static int rowsum(crdt_ctx *ctx, const uint64_t *p, const uint64_t *n, uint64_t *out, size_t rows,
                  size_t nodes) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (mul_overflows(rows, nodes)) return CRDT_E_INVAL;
    if (rows == 0) return CRDT_OK;
    if (!p || !out || (PN && !n)) return CRDT_E_INVAL;
    const bool vec = aligned16(p) && (!PN || aligned16(n));
    const unsigned grid = grid_for(rows * 64, 256, (unsigned)(ctx->num_cus * 8));
    const hipStream_t s = ctx->stream;
    const u64x2 *vp = (const u64x2 *)p, *vn = (const u64x2 *)n;
    if (vec && nodes == 64) k_rowsum<64, PN><<<grid, 256, 0, s>>>(vp, vn, out, rows);
    else if (vec && nodes == 128) k_rowsum<128, PN><<<grid, 256, 0, s>>>(vp, vn, out, rows);
    else if (vec && nodes == 32) k_rowsum<32, PN><<<grid, 256, 0, s>>>(vp, vn, out, rows);
    else if (vec && nodes == 16) k_rowsum<16, PN><<<grid, 256, 0, s>>>(vp, vn, out, rows);
    else k_rowsum_generic<PN><<<grid, 256, 0, s>>>(p, n, out, rows, nodes);
    return check_launch(ctx);
}

extern "C" int crdt_gcounter_value(crdt_ctx *ctx, const uint64_t *a, size_t rows, size_t nodes,
                                   uint64_t *out) {
    return rowsum<false>(ctx, a, nullptr, out, rows, nodes);
}

extern "C" int crdt_pncounter_value(crdt_ctx *ctx, const uint64_t *p, const uint64_t *n, int64_t *out,
                                    size_t rows, size_t nodes) {
    return rowsum<true>(ctx, p, n, (uint64_t *)out, rows, nodes);
}

extern "C" int crdt_u64_to_ordered_i64(crdt_ctx *ctx, const uint64_t *in, int64_t *out, size_t n) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (n == 0) return CRDT_OK;
    if (!in || !out) return CRDT_E_INVAL;
    k_u64_to_i64<<<grid_for(n, 256, 4096), 256, 0, ctx->stream>>>(in, out, n);
    return check_launch(ctx);
}

extern "C" int crdt_ordered_i64_to_u64(crdt_ctx *ctx, const int64_t *in, uint64_t *out, size_t n) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (n == 0) return CRDT_OK;
    if (!in || !out) return CRDT_E_INVAL;
    k_i64_to_u64<<<grid_for(n, 256, 4096), 256, 0, ctx->stream>>>(in, out, n);
    return check_launch(ctx);
}
