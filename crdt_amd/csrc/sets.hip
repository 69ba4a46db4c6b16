// sets.hip -- LWW-Element-Set and OR-Set merge.
//
// Build-defined semantics (no reference code), tie rule from the reference:
// on an exactly equal timestamp the local/left value is kept (main.go:54-65).
// Inputs A (local) and B (remote) are SoA tuples (key u64, ts u64, rep u32,
// tomb u8) sorted ascending by (key, ts, rep).  The merged order is the
// STABLE merge: on an equal tuple A's element precedes B's.
//   LWW    : one output per distinct key = the first element (in merged
//            order) carrying the key's maximal (ts, rep); tombstoned winners
//            are kept (they are state).
//   OR-Set : one output per distinct tag (key, ts, rep); tomb = OR over the
//            tag's elements (add-wins only if some copy is not removed).
//
// GPU structure (merge path, Odeh et al. / Green et al.):
//   1. k_partition : binary search of each tile's diagonal -> (i, j) split.
//   2. k_set_tile<count> : per tile, stage the A and B slices in LDS, merge
//      in LDS (per-lane merge-path search + ITEMS-long serial merge), flag
//      emitting positions, write the tile's output count.  LWW counting needs
//      keys only (8 of 21 bytes per tuple).
//   3. exclusive scan of tile counts.
//   4. k_set_tile<write> : re-merge, rank emitters with wave ballots, resolve
//      the winner / tomb-OR (runs crossing a tile edge continue in global
//      memory), write coalesced SoA output.
#include "scan.hpp"

namespace crdt {

enum { SET_LWW = 0, SET_OR = 1 };

struct Tag {
    uint64_t k, t;
    uint32_t r;
};
__device__ __forceinline__ bool tag_le(const Tag &a, const Tag &b) {
    if (a.k != b.k) return a.k < b.k;
    if (a.t != b.t) return a.t < b.t;
    return a.r <= b.r;
}
__device__ __forceinline__ bool tag_eq(const Tag &a, const Tag &b) {
    return a.k == b.k && a.t == b.t && a.r == b.r;
}
__device__ __forceinline__ Tag gtag(const crdt_tuples &s, size_t i) { return Tag{s.key[i], s.ts[i], s.rep[i]}; }

// Merge-path split of diagonal d: number of A elements among the first d
// merged elements.  A[x] precedes B[y] iff A[x] <= B[y] (stable, A first).
__global__ void k_partition(crdt_tuples A, crdt_tuples B, size_t na, size_t nb, size_t tile, size_t ntiles,
                            uint64_t *__restrict__ split) {
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (t > ntiles) return;
    const size_t n = na + nb;
    size_t d = t * tile;
    if (d > n) d = n;
    size_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
    while (lo < hi) {
        const size_t mid = (lo + hi) >> 1;
        if (tag_le(gtag(A, mid), gtag(B, d - 1 - mid))) lo = mid + 1;
        else hi = mid;
    }
    split[t] = lo;
}

template <int MODE, bool WRITE, int ITEMS>
__global__ __launch_bounds__(256) void k_set_tile(crdt_tuples A, crdt_tuples B, size_t na, size_t nb,
                                                  const uint64_t *__restrict__ split,
                                                  uint32_t *__restrict__ tile_count,
                                                  const uint64_t *__restrict__ tile_off, crdt_tuples out) {
    constexpr int TILE = 256 * ITEMS;
    constexpr bool KEYS_ONLY = (MODE == SET_LWW) && !WRITE;   // counting key-run ends needs keys only
    __shared__ uint64_t skey[TILE];
    __shared__ uint64_t sts[KEYS_ONLY ? 1 : TILE];
    __shared__ uint32_t srep[KEYS_ONLY ? 1 : TILE];
    __shared__ uint8_t stomb[WRITE ? TILE : 1];
    __shared__ uint16_t smi[TILE];
    __shared__ Tag edge_prev, edge_next;
    __shared__ int has_prev, has_next;

    const size_t n = na + nb;
    const size_t t = blockIdx.x;
    const size_t d0 = t * (size_t)TILE;
    const size_t d1 = d0 + TILE < n ? d0 + TILE : n;
    const size_t i0 = split[t], i1 = split[t + 1];
    const size_t j0 = d0 - i0, j1 = d1 - i1;
    const int na_t = (int)(i1 - i0), len = (int)(d1 - d0);
    const int nb_t = len - na_t;
    const int tid = threadIdx.x;

    // ---- stage the tile's A slice then B slice in LDS (coalesced)
    for (int x = tid; x < len; x += 256) {
        const bool fromA = x < na_t;
        const size_t g = fromA ? i0 + x : j0 + (x - na_t);
        skey[x] = (fromA ? A.key : B.key)[g];
        if constexpr (!KEYS_ONLY) {
            sts[x] = (fromA ? A.ts : B.ts)[g];
            srep[x] = (fromA ? A.rep : B.rep)[g];
        }
        if constexpr (WRITE) stomb[x] = (fromA ? A.tomb : B.tomb)[g];
    }
    // ---- neighbours across the tile edges (merged positions d0-1 and d1)
    if (tid == 0) {
        has_prev = 0;
        if (d0 > 0) {
            if (i0 > 0 && j0 > 0) {
                const Tag a = gtag(A, i0 - 1), b = gtag(B, j0 - 1);
                const bool lb = tag_le(a, b);              // the later one in merged order
                edge_prev = Tag{lb ? b.k : a.k, lb ? b.t : a.t, lb ? b.r : a.r};
            } else if (i0 > 0) {
                edge_prev = gtag(A, i0 - 1);
            } else {
                edge_prev = gtag(B, j0 - 1);
            }
            has_prev = 1;
        }
        has_next = 0;
        if (d1 < n) {
            if (i1 < na && j1 < nb) {
                const Tag a = gtag(A, i1), b = gtag(B, j1);
                const bool la = tag_le(a, b);              // the earlier one in merged order
                edge_next = Tag{la ? a.k : b.k, la ? a.t : b.t, la ? a.r : b.r};
            } else if (i1 < na) {
                edge_next = gtag(A, i1);
            } else {
                edge_next = gtag(B, j1);
            }
            has_next = 1;
        }
    }
    __syncthreads();

    // ---- per-lane merge path inside the tile, then ITEMS serial merge steps
    auto ltag = [&](int x) -> Tag {
        if constexpr (KEYS_ONLY) return Tag{skey[x], 0, 0};
        else return Tag{skey[x], sts[x], srep[x]};
    };
    {
        const int dd = tid * ITEMS < len ? tid * ITEMS : len;
        int lo = dd > nb_t ? dd - nb_t : 0, hi = dd < na_t ? dd : na_t;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (tag_le(ltag(mid), ltag(na_t + dd - 1 - mid))) lo = mid + 1;
            else hi = mid;
        }
        int ia = lo, ib = dd - lo;
#pragma unroll
        for (int u = 0; u < ITEMS; ++u) {
            const int k = dd + u;
            if (k < len) {
                const bool takeA = ib >= nb_t || (ia < na_t && tag_le(ltag(ia), ltag(na_t + ib)));
                smi[k] = (uint16_t)(takeA ? ia++ : na_t + ib++);
            }
        }
    }
    __syncthreads();

    // ---- emit flags: OR -> first of a tag run; LWW -> last of a key run
    uint64_t run = WRITE ? tile_off[t] : 0;
    uint32_t cnt = 0;
#pragma unroll 1
    for (int u = 0; u < ITEMS; ++u) {
        const int k = u * 256 + tid;
        bool emit = false;
        int e = 0;
        if (k < len) {
            e = smi[k];
            if constexpr (MODE == SET_OR) {
                if (k > 0) emit = !tag_eq(ltag(smi[k - 1]), ltag(e));
                else emit = !has_prev || !tag_eq(edge_prev, ltag(e));
            } else {
                if (k + 1 < len) emit = skey[smi[k + 1]] != skey[e];
                else emit = !has_next || edge_next.k != skey[e];
            }
        }
        if constexpr (!WRITE) {
            cnt += emit ? 1u : 0u;
        } else {
            uint32_t tot;
            const uint32_t rank = block_rank_flag(emit, &tot);
            if (emit) {
                const size_t pos = run + rank;
                const Tag tg = ltag(e);
                uint8_t tomb;
                if constexpr (MODE == SET_OR) {
                    // tomb-OR over the tag's run, continuing past the tile end
                    tomb = stomb[e];
                    int m = k;
                    while (m + 1 < len && tag_eq(ltag(smi[m + 1]), tg)) tomb |= stomb[smi[++m]];
                    if (m + 1 == len) {
                        for (size_t x = i1; x < na && tag_eq(gtag(A, x), tg); ++x) tomb |= A.tomb[x];
                        for (size_t y = j1; y < nb && tag_eq(gtag(B, y), tg); ++y) tomb |= B.tomb[y];
                    }
                } else {
                    // winner = earliest element (merged order) carrying this tag
                    int m = k;
                    while (m > 0 && tag_eq(ltag(smi[m - 1]), tg)) --m;
                    tomb = stomb[smi[m]];
                    if (m == 0 && has_prev && tag_eq(edge_prev, tg)) {
                        if (i0 > 0 && tag_eq(gtag(A, i0 - 1), tg)) {
                            size_t x = i0 - 1;
                            while (x > 0 && tag_eq(gtag(A, x - 1), tg)) --x;
                            tomb = A.tomb[x];
                        } else {
                            size_t y = j0 - 1;
                            while (y > 0 && tag_eq(gtag(B, y - 1), tg)) --y;
                            tomb = B.tomb[y];
                        }
                    }
                }
                out.key[pos] = tg.k;
                out.ts[pos] = tg.t;
                out.rep[pos] = tg.r;
                out.tomb[pos] = tomb;
            }
            run += tot;
        }
    }
    if constexpr (!WRITE) {
        uint64_t tot;
        block_exclusive_scan_u64(cnt, &tot);
        if (tid == 0) tile_count[t] = (uint32_t)tot;
    }
}

__global__ void k_store_count(const uint64_t *__restrict__ offs, size_t ntiles, uint64_t *__restrict__ out_count) {
    *out_count = offs[ntiles];
}

// Adjacent pairs out of (key, ts, rep) order.
__global__ void k_count_unsorted(crdt_tuples T, size_t n, unsigned long long *bad) {
    unsigned long long c = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i + 1 < n; i += (size_t)gridDim.x * 256)
        c += tag_le(gtag(T, i), gtag(T, i + 1)) ? 0 : 1;
    if (c) atomicAdd(bad, c);
}

template <int MODE, int ITEMS>
static int set_merge_impl(crdt_ctx *ctx, const crdt_tuples &A, size_t na, const crdt_tuples &B, size_t nb,
                          const crdt_tuples &O, uint64_t *out_count) {
    constexpr size_t TILE = 256 * ITEMS;
    const size_t n = na + nb;
    const size_t ntiles = (n + TILE - 1) / TILE;
    if (ntiles > 0x7fffffffULL) return CRDT_E_RANGE;
    const size_t b_split = Carve::round((ntiles + 1) * sizeof(uint64_t));
    const size_t b_cnt = Carve::round(ntiles * sizeof(uint32_t));
    const size_t b_off = Carve::round((ntiles + 1) * sizeof(uint64_t));
    const size_t b_tmp = scan_tmp_bytes(ntiles);
    int rc = ws_reserve(ctx, b_split + b_cnt + b_off + b_tmp + 1024);
    if (rc) return rc;
    Carve w(ctx->ws);
    uint64_t *split = w.take<uint64_t>(ntiles + 1);
    uint32_t *cnt = w.take<uint32_t>(ntiles);
    uint64_t *off = w.take<uint64_t>(ntiles + 1);
    void *tmp = w.take<char>(b_tmp);
    const hipStream_t s = ctx->stream;
    k_partition<<<grid_for(ntiles + 1, 256, 0x7fffffff), 256, 0, s>>>(A, B, na, nb, TILE, ntiles, split);
    k_set_tile<MODE, false, ITEMS><<<(unsigned)ntiles, 256, 0, s>>>(A, B, na, nb, split, cnt, nullptr, O);
    rc = check_launch(ctx);
    if (rc) return rc;
    rc = exclusive_scan_u32(ctx, cnt, off, ntiles, tmp);
    if (rc) return rc;
    k_set_tile<MODE, true, ITEMS><<<(unsigned)ntiles, 256, 0, s>>>(A, B, na, nb, split, nullptr, off, O);
    k_store_count<<<1, 1, 0, s>>>(off, ntiles, out_count);
    return check_launch(ctx);
}

static bool tuples_ok(const crdt_tuples *t) { return t && t->key && t->ts && t->rep && t->tomb; }

template <int MODE>
static int set_merge(crdt_ctx *ctx, const crdt_tuples *a, size_t na, const crdt_tuples *b, size_t nb,
                     crdt_tuples *out, uint64_t *out_count) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!out_count || !tuples_ok(out)) return CRDT_E_INVAL;
    if ((na && !tuples_ok(a)) || (nb && !tuples_ok(b))) return CRDT_E_INVAL;
    if (na + nb == 0) {
        hipError_t e = hipMemsetAsync(out_count, 0, sizeof(uint64_t), ctx->stream);
        return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
    }
    crdt_tuples empty{nullptr, nullptr, nullptr, nullptr};
    const crdt_tuples &A = na ? *a : empty;
    const crdt_tuples &B = nb ? *b : empty;
    if (g_sets_items == 4) return set_merge_impl<MODE, 4>(ctx, A, na, B, nb, *out, out_count);
    return set_merge_impl<MODE, 8>(ctx, A, na, B, nb, *out, out_count);
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_lww_merge(crdt_ctx *ctx, const crdt_tuples *a, size_t na, const crdt_tuples *b, size_t nb,
                              crdt_tuples *out, uint64_t *out_count_dev) {
    return set_merge<SET_LWW>(ctx, a, na, b, nb, out, out_count_dev);
}

extern "C" int crdt_orset_merge(crdt_ctx *ctx, const crdt_tuples *a, size_t na, const crdt_tuples *b, size_t nb,
                                crdt_tuples *out, uint64_t *out_count_dev) {
    return set_merge<SET_OR>(ctx, a, na, b, nb, out, out_count_dev);
}

extern "C" int crdt_tuples_count_unsorted(crdt_ctx *ctx, const crdt_tuples *t, size_t n, uint64_t *bad) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!bad) return CRDT_E_INVAL;
    hipError_t e = hipMemsetAsync(bad, 0, sizeof(uint64_t), ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
    if (n < 2) return CRDT_OK;
    if (!tuples_ok(t)) return CRDT_E_INVAL;
    k_count_unsorted<<<grid_for(n, 256, (unsigned)ctx->num_cus * 8), 256, 0, ctx->stream>>>(
        *t, n, (unsigned long long *)bad);
    return check_launch(ctx);
}
