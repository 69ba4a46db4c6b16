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
//            tag's elements.
//
// GPU structure (merge path + single-pass decoupled look-back):
//   1. k_partition: 16-ary searches, four tile diagonals per wave (one per
//      16-lane group), comparing keys first and loading ts/rep only on a key
//      tie.
//   2. k_set_merge: each workgroup takes the next tile id from an atomic
//      counter (a look-back then never waits on a tile that no running
//      workgroup owns), issues all of the tile's A/B loads before any LDS
//      store, finds its lane's merge-path split in LDS and merges ITEMS
//      elements keeping the merged tags in REGISTERS (the two heads are the
//      only LDS reads per step), derives emit flags / LWW winners / OR-Set
//      tomb-ORs from registers (runs that cross a lane, tile edge continue
//      through the merged-order index in LDS and then global memory: rare),
//      publishes its count and looks back 256 predecessors per round trip
//      ({flag, count} 8-byte agent-scope atomics: the data is the flag),
//      stages the output in LDS and writes it with coalesced stores.
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

// A[i] <= B[j] in tuple order, reading ts / rep only on a tie.
__device__ __forceinline__ bool g_le_lazy(const crdt_tuples &A, size_t i, const crdt_tuples &B, size_t j) {
    const uint64_t ka = A.key[i], kb = B.key[j];
    if (ka != kb) return ka < kb;
    const uint64_t ta = A.ts[i], tb = B.ts[j];
    if (ta != tb) return ta < tb;
    return A.rep[i] <= B.rep[j];
}

// ---------------------------------------------------------------- partition
// split[t] = number of A elements among the first min(t*TILE, n) merged
// elements.  P(i) = A[i] <= B[d-1-i] is true for i < answer, false after.
__global__ __launch_bounds__(256) void k_partition(crdt_tuples A, crdt_tuples B, size_t na, size_t nb,
                                                   size_t tile, size_t ntiles, uint64_t *__restrict__ split) {
    const int lane = threadIdx.x & 63, grp = lane >> 4, gl = lane & 15;
    const size_t t = ((((size_t)blockIdx.x * 256 + threadIdx.x) >> 6) << 2) + (size_t)grp;
    const size_t n = na + nb;
    const size_t d = t * tile < n ? t * tile : n;
    size_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
    bool done = t > ntiles || hi <= lo;
    while (__ballot(!done)) {
        const size_t span = hi - lo;
        const bool small = span <= 16;
        const size_t c = small ? lo + (size_t)gl : lo + ((size_t)gl * span) / 16;
        const bool valid = !done && (small ? (size_t)gl < span : true);
        const bool p = valid && g_le_lazy(A, c, B, d - 1 - c);
        const unsigned m = (unsigned)((__ballot(p) >> (grp * 16)) & 0xFFFF);
        const unsigned cnt = (unsigned)__popc(m);
        if (!done) {
            if (small) {
                lo += cnt;
                done = true;
            } else {
                const size_t nlo = cnt > 0 ? lo + (((size_t)(cnt - 1)) * span) / 16 + 1 : lo;
                const size_t nhi = cnt < 16 ? lo + ((size_t)cnt * span) / 16 : hi;
                lo = nlo;
                hi = nhi;
                done = hi <= lo;
            }
        }
    }
    if (gl == 0 && t <= ntiles) split[t] = lo;
}

// ---------------------------------------------------------------- look-back
constexpr uint64_t kFlagAgg = 1ULL << 62;     // tile count available
constexpr uint64_t kFlagInc = 2ULL << 62;     // inclusive prefix available
constexpr uint64_t kValMask = (1ULL << 62) - 1;

__device__ __forceinline__ uint64_t ld_status(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Called by the WHOLE 256-lane block (contains barriers; every loop decision
// is block-uniform).  Exclusive prefix of tile t = sum of the counts of tiles
// 0..t-1.  One round trip reads 1024 predecessors (4 per lane, nearest
// first); it stops at the nearest inclusive prefix and spins only while a
// nearer predecessor has not published its count.  Bounded: sets *err.
__device__ uint64_t block_look_back(const uint64_t *status, uint32_t t, uint32_t *err, int *s_fi, int *s_fv,
                                    uint64_t *s_part) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t excl = 0;
    int64_t base = (int64_t)t - 1;
    unsigned spins = 0;
    while (base >= 0) {
        uint64_t s[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t idx = base - (w * 256 + j * 64 + lane);
            s[j] = idx >= 0 ? ld_status(status + idx) : kFlagInc;   // virtual inclusive 0 before tile 0
        }
        int fi = 1024, fv = 1024;
#pragma unroll
        for (int j = 3; j >= 0; --j) {
            const uint64_t inc = __ballot((s[j] >> 62) == 2), inv = __ballot((s[j] >> 62) == 0);
            if (inc) fi = w * 256 + j * 64 + __ffsll((unsigned long long)inc) - 1;
            if (inv) fv = w * 256 + j * 64 + __ffsll((unsigned long long)inv) - 1;
        }
        if (lane == 0) { s_fi[w] = fi; s_fv[w] = fv; }
        __syncthreads();
        int FI = s_fi[0], FV = s_fv[0];
#pragma unroll
        for (int k = 1; k < 4; ++k) { FI = s_fi[k] < FI ? s_fi[k] : FI; FV = s_fv[k] < FV ? s_fv[k] : FV; }
        __syncthreads();
        if (FV < FI) {                               // a nearer predecessor has not published yet
            if (++spins > (1u << 22)) {
                if (threadIdx.x == 0) atomicOr(err, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint64_t v = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) v += (w * 256 + j * 64 + lane <= FI) ? (s[j] & kValMask) : 0;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
        if (lane == 0) s_part[w] = v;
        __syncthreads();
        excl += s_part[0] + s_part[1] + s_part[2] + s_part[3];
        __syncthreads();
        if (FI < 1024) break;
        base -= 1024;
    }
    return excl;
}

// ---------------------------------------------------------------- tile merge
template <int MODE, int ITEMS>
__global__ __launch_bounds__(256) void k_set_merge(crdt_tuples A, crdt_tuples B, size_t na, size_t nb,
                                                   const uint64_t *__restrict__ split, uint64_t *status,
                                                   uint32_t *tile_ctr, uint32_t *err, uint32_t ntiles, int ablate,
                                                   crdt_tuples out, uint64_t *__restrict__ out_count,
                                                   uint64_t *stamps) {
    // Diagnostic build only (stamps != nullptr): per-tile s_memtime at phase
    // boundaries, written to a buffer nothing else reads.
#define STAMP(i) \
    do { if (stamps && threadIdx.x == 0) stamps[(size_t)s_tile * 8 + (i)] = __builtin_amdgcn_s_memtime(); } while (0)
    constexpr int TILE = 256 * ITEMS;
    __shared__ uint64_t skey[TILE];
    __shared__ uint64_t sts[TILE];
    __shared__ uint32_t srep[TILE];
    __shared__ uint8_t stomb[TILE];
    __shared__ uint16_t smi[TILE];
    __shared__ uint64_t s_edge_k[2], s_edge_t[2];
    __shared__ uint32_t s_edge_r[2];
    __shared__ int s_has[2];
    __shared__ uint32_t s_tile;
    __shared__ int s_fi[4], s_fv[4];
    __shared__ uint64_t s_part[4];

    const int tid = threadIdx.x;
    if (tid == 0) s_tile = (ablate & 4) ? blockIdx.x : atomicAdd(tile_ctr, 1u);   // 4: timing only, with 1
    __syncthreads();
    const uint32_t t = s_tile;
    STAMP(0);
    const size_t n = na + nb;
    const size_t d0 = (size_t)t * TILE;
    const size_t d1 = d0 + TILE < n ? d0 + TILE : n;
    const size_t i0 = split[t], i1 = split[t + 1];
    const size_t j0 = d0 - i0, j1 = d1 - i1;
    const int na_t = (int)(i1 - i0), len = (int)(d1 - d0);
    const int nb_t = len - na_t;

    // ---- issue every load of the tile (and its edge neighbours) before any LDS store
    uint64_t rk[ITEMS], rt[ITEMS];     // this lane's tile elements x = u*256 + tid (kept for the rank search)
    uint32_t rr[ITEMS];
    {
        uint8_t rb[ITEMS];
#pragma unroll
        for (int u = 0; u < ITEMS; ++u) {
            const int x = u * 256 + tid;
            if (x < len) {
                const bool fa = x < na_t;
                const size_t g = fa ? i0 + x : j0 + (x - na_t);
                rk[u] = (fa ? A.key : B.key)[g];
                rt[u] = (fa ? A.ts : B.ts)[g];
                rr[u] = (fa ? A.rep : B.rep)[g];
                rb[u] = (fa ? A.tomb : B.tomb)[g];
            }
        }
        if (tid == 0 || tid == 64) {                  // merged positions d0-1 (prev) and d1 (next)
            const bool prev = tid == 0;
            int has = 0;
            Tag e{0, 0, 0};
            if (prev && d0 > 0) {
                has = 1;
                if (i0 > 0 && j0 > 0) {
                    const Tag a = gtag(A, i0 - 1), b = gtag(B, j0 - 1);
                    const bool lb = tag_le(a, b);      // the later one in merged order
                    e = Tag{lb ? b.k : a.k, lb ? b.t : a.t, lb ? b.r : a.r};
                } else if (i0 > 0) {
                    e = gtag(A, i0 - 1);
                } else {
                    e = gtag(B, j0 - 1);
                }
            } else if (!prev && d1 < n) {
                has = 1;
                if (i1 < na && j1 < nb) {
                    const Tag a = gtag(A, i1), b = gtag(B, j1);
                    const bool la = tag_le(a, b);      // the earlier one in merged order
                    e = Tag{la ? a.k : b.k, la ? a.t : b.t, la ? a.r : b.r};
                } else if (i1 < na) {
                    e = gtag(A, i1);
                } else {
                    e = gtag(B, j1);
                }
            }
            const int w = prev ? 0 : 1;
            s_has[w] = has;
            s_edge_k[w] = e.k;
            s_edge_t[w] = e.t;
            s_edge_r[w] = e.r;
        }
#pragma unroll
        for (int u = 0; u < ITEMS; ++u) {
            const int x = u * 256 + tid;
            if (x < len) {
                skey[x] = rk[u];
                sts[x] = rt[u];
                srep[x] = rr[u];
                stomb[x] = rb[u];
            }
        }
    }
    __syncthreads();
    STAMP(1);

#define LTAG(x) Tag{skey[(x)], sts[(x)], srep[(x)]}
    // ---- merge path: this lane owns merged positions [dd, dd + nv); the
    // merged tags stay in registers, the two heads are the only LDS reads
    // per serial step.  (A per-element ILP rank search was measured 3.6x
    // slower here: 12 x 3 scattered LDS probes per element.)
    const int dd = tid * ITEMS < len ? tid * ITEMS : len;
    const int nv = len - dd < ITEMS ? len - dd : ITEMS;
    Tag it[ITEMS];
    uint8_t tb[ITEMS];
    {
        int lo = dd > nb_t ? dd - nb_t : 0, hi = dd < na_t ? dd : na_t;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            const int mb = na_t + dd - 1 - mid;
            bool le;
            const uint64_t ka = skey[mid], kb = skey[mb];
            if (ka != kb) le = ka < kb;
            else le = tag_le(LTAG(mid), LTAG(mb));
            if (le) lo = mid + 1;
            else hi = mid;
        }
        int ia = lo, ib = dd - lo;
        Tag ha = ia < na_t ? LTAG(ia) : Tag{0, 0, 0};
        Tag hb = ib < nb_t ? LTAG(na_t + ib) : Tag{0, 0, 0};
#pragma unroll
        for (int u = 0; u < ITEMS; ++u) {
            if (u < nv) {
                const bool takeA = ib >= nb_t || (ia < na_t && tag_le(ha, hb));
                const int src = takeA ? ia : na_t + ib;
                it[u] = takeA ? ha : hb;
                smi[dd + u] = (uint16_t)src;
                tb[u] = stomb[src];
                if (takeA) {
                    ++ia;
                    if (ia < na_t) ha = LTAG(ia);
                } else {
                    ++ib;
                    if (ib < nb_t) hb = LTAG(na_t + ib);
                }
            } else {
                it[u] = Tag{0, 0, 0};
                tb[u] = 0;
            }
        }
    }
    __syncthreads();
    STAMP(2);

    // ---- neighbours of this lane's run: merged positions dd-1 and dd+nv
    const Tag eprev{s_edge_k[0], s_edge_t[0], s_edge_r[0]};
    const Tag enext{s_edge_k[1], s_edge_t[1], s_edge_r[1]};
    const bool has_prev_edge = s_has[0] != 0, has_next_edge = s_has[1] != 0;
    bool hp = false, hn = false;
    Tag pv{0, 0, 0}, nx{0, 0, 0};
    if (nv > 0) {
        if (dd > 0) { pv = LTAG(smi[dd - 1]); hp = true; }
        else if (has_prev_edge) { pv = eprev; hp = true; }
        if (dd + nv < len) { nx = LTAG(smi[dd + nv]); hn = true; }
        else if (has_next_edge) { nx = enext; hn = true; }
    }

    // ---- emit flags from registers (OR: first of a tag run; LWW: last of a key run)
    uint32_t emask = 0;
#pragma unroll
    for (int u = 0; u < ITEMS; ++u) {
        if (u < nv) {
            bool emit;
            if constexpr (MODE == SET_OR) {
                emit = u > 0 ? !tag_eq(it[u - 1], it[u]) : !(hp && tag_eq(pv, it[0]));
            } else {
                emit = (u + 1 < nv) ? it[u + 1].k != it[u].k : !(hn && nx.k == it[u].k);
            }
            emask |= emit ? (1u << u) : 0u;
        }
    }
    uint64_t total;
    const uint64_t local_off = block_exclusive_scan_u64((uint64_t)__popc(emask), &total);
    STAMP(3);

    // ---- publish this tile's count now; its successors can look past it
    // while this tile resolves and stages (the look-back itself comes last)
    if (tid == 0) st_status(status + t, (t == 0 ? kFlagInc : kFlagAgg) | total);

    // ---- output tombs from registers; runs crossing this lane's edge are rare
    uint8_t ot[ITEMS];
    if constexpr (MODE == SET_OR) {
        // tomb-OR over the run that starts at each emitter (backward sweep)
        uint8_t carry = 0;
        Tag last = it[0];                                       // it[nv-1] without a runtime index
#pragma unroll
        for (int u = 1; u < ITEMS; ++u)
            if (u < nv) last = it[u];
        if (nv > 0 && hn && tag_eq(nx, last)) {                 // run continues past this lane
            const Tag tg = last;
            int m = dd + nv;
            while (m < len && tag_eq(LTAG(smi[m]), tg)) carry |= stomb[smi[m++]];
            if (m == len) {
                for (size_t x = i1; x < na && tag_eq(gtag(A, x), tg); ++x) carry |= A.tomb[x];
                for (size_t y = j1; y < nb && tag_eq(gtag(B, y), tg); ++y) carry |= B.tomb[y];
            }
        }
#pragma unroll
        for (int u = ITEMS - 1; u >= 0; --u) {
            if (u < nv) {
                const bool cont = (u + 1 < nv) ? tag_eq(it[u + 1], it[u]) : true;   // last valid: carry
                const uint8_t c = (u + 1 < nv) ? (cont ? ot[u + 1] : (uint8_t)0) : carry;
                ot[u] = (uint8_t)(tb[u] | c);
            } else {
                ot[u] = 0;
            }
        }
    } else {
        // LWW winner = earliest element carrying the emitter's tag (forward sweep)
        uint8_t first = 0;
        if (nv > 0 && hp && tag_eq(pv, it[0])) {                 // tag group began before this lane
            const Tag tg = it[0];
            int m = dd - 1;
            while (m > 0 && tag_eq(LTAG(smi[m - 1]), tg)) --m;
            first = (dd > 0) ? stomb[smi[m]] : 0;
            if ((dd == 0 || m == 0) && has_prev_edge && tag_eq(eprev, tg)) {   // ... or before the tile
                if (i0 > 0 && tag_eq(gtag(A, i0 - 1), tg)) {
                    size_t x = i0 - 1;
                    while (x > 0 && tag_eq(gtag(A, x - 1), tg)) --x;
                    first = A.tomb[x];
                } else {
                    size_t y = j0 - 1;
                    while (y > 0 && tag_eq(gtag(B, y - 1), tg)) --y;
                    first = B.tomb[y];
                }
            }
        } else {
            first = tb[0];
        }
#pragma unroll
        for (int u = 0; u < ITEMS; ++u) {
            if (u == 0) ot[0] = first;
            else ot[u] = (u < nv && tag_eq(it[u - 1], it[u])) ? ot[u - 1] : tb[u];
        }
    }
#undef LTAG
    __syncthreads();                                          // inputs in LDS are dead from here
    STAMP(5);

    // ---- stage the tile's output in LDS at its local offsets, then copy out coalesced
    {
        uint32_t o = (uint32_t)local_off;
#pragma unroll
        for (int u = 0; u < ITEMS; ++u) {
            if (emask & (1u << u)) {
                skey[o] = it[u].k;
                sts[o] = it[u].t;
                srep[o] = it[u].r;
                stomb[o] = ot[u];
                ++o;
            }
        }
    }
    __syncthreads();
    STAMP(6);
    // ---- output offset: decoupled look-back by the whole block (1024 predecessors per round trip)
    uint64_t P = 0;
    if (t > 0) {
        P = (ablate & 1) ? 0 : block_look_back(status, t, err, s_fi, s_fv, s_part);
        if (tid == 0) st_status(status + t, kFlagInc | (P + total));
    }
    if (tid == 0 && t == ntiles - 1) *out_count = P + total;
    STAMP(4);
    const int T = (int)total;
    if (!(ablate & 2)) {
#pragma unroll
        for (int u = 0; u < ITEMS; ++u) {
            const int x = u * 256 + tid;
            if (x < T) {
                out.key[P + x] = skey[x];
                out.ts[P + x] = sts[x];
                out.rep[P + x] = srep[x];
                out.tomb[P + x] = stomb[x];
            }
        }
    }
    if (stamps) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        STAMP(7);
    }
#undef STAMP
}

uint64_t *g_last_stamps = nullptr;   // diagnostic: stamps of the last set merge (8 per tile)
size_t g_last_stamps_n = 0;

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
    if (ntiles >= 0x7fffffffULL || n >= (1ULL << 62)) return CRDT_E_RANGE;
    // status words + tile counter + error word first (one memset), split after
    const size_t b_status = Carve::round((ntiles + 4) * sizeof(uint64_t));
    const size_t b_split = Carve::round((ntiles + 1) * sizeof(uint64_t));
    const size_t b_stamps = g_sets_stamps ? Carve::round(ntiles * 8 * sizeof(uint64_t)) : 0;
    int rc = ws_reserve(ctx, b_status + b_split + b_stamps + 768);
    if (rc) return rc;
    Carve w(ctx->ws);
    uint64_t *status = w.take<uint64_t>(ntiles + 4);
    uint32_t *ctr = (uint32_t *)(status + ntiles);        // status[ntiles]: tile counter + error word
    uint32_t *err = ctr + 1;
    uint64_t *split = w.take<uint64_t>(ntiles + 1);
    uint64_t *stamps = g_sets_stamps ? w.take<uint64_t>(ntiles * 8) : nullptr;
    g_last_stamps = stamps;
    g_last_stamps_n = stamps ? ntiles * 8 : 0;
    const hipStream_t s = ctx->stream;
    hipError_t e = hipMemsetAsync(status, 0, b_status, s);
    if (e != hipSuccess) return hip_fail(ctx, e);
    const size_t diags = ntiles + 1;                      // 4 diagonals per wave, 16 per block
    k_partition<<<(unsigned)((diags + 15) / 16), 256, 0, s>>>(A, B, na, nb, TILE, ntiles, split);
    k_set_merge<MODE, ITEMS><<<(unsigned)ntiles, 256, 0, s>>>(A, B, na, nb, split, status, ctr, err,
                                                              (uint32_t)ntiles, g_sets_ablate, O, out_count,
                                                              stamps);
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

// Diagnostic: copy the phase stamps of the last set merge (8 s_memtime values
// per tile) to host memory.  Enabled by crdt_set_option("sets.stamps", 1).
extern "C" int crdt_debug_set_stamps(crdt_ctx *ctx, uint64_t *host, size_t cap, size_t *n) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!n) return CRDT_E_INVAL;
    *n = g_last_stamps_n;
    if (!g_last_stamps || !host || cap == 0) return CRDT_OK;
    const size_t m = cap < g_last_stamps_n ? cap : g_last_stamps_n;
    hipError_t e = hipMemcpyAsync(host, g_last_stamps, m * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
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
