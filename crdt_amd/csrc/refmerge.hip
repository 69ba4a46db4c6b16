// refmerge.hip -- bit-exact batched (*Server).merge() of the reference
// (/root/reference/main.go:35-100), many replicas per launch.
//
// Closed form implemented (derivation in DESIGN.md "RefMerge"):
//  Walk (main.go:45-73): Diff' = L u {r in R : r not in L, r < max(L)}.
//    r is inserted iff lower_bound(L, r) < |L| and L[lb] != r: an equal ts
//    keeps the local entry (main.go:54-65); remote ts above max(L) are never
//    reached by the two-pointer loop (main.go:49) and are dropped.
//  Replay (main.go:75-98): CurrentState rebuilt from empty over the
//    remote-origin entries of Diff' (local *Command values fail the
//    map[string]string assertion, main.go:80), descending ts.  Per key:
//      base = value of the max-ts entry holding the key;
//      if Atoi(base) fails or no other holder's value parses -> base verbatim
//      else Itoa(sum of every parsable value), int64 wrap (main.go:95).
//    The sum is order-independent (mod 2^64), which is what lets the fold run
//    as parallel atomics instead of the reference's serial descending loop.
//
// Kernels: atoi over the string arena; tiled merge-path walk (count pass,
// device scan, write pass producing the new Diff and folding the replay into
// per-slot accumulators); per-slot closed form (k_slot_final).
#include <algorithm>

#include "scan.hpp"

namespace crdt {

// Go 1.18 strconv.Atoi (64-bit): ^[+-]?[0-9]+$ within int64, leading zeros ok.
__device__ __forceinline__ bool go_atoi(const uint8_t *s, uint64_t len, int64_t *out) {
    if (len == 0) return false;
    uint64_t i = 0;
    bool neg = false;
    if (s[0] == '+' || s[0] == '-') {
        neg = s[0] == '-';
        i = 1;
        if (len == 1) return false;
    }
    uint64_t acc = 0;
    for (; i < len; ++i) {
        const unsigned d = (unsigned)s[i] - (unsigned)'0';
        if (d > 9) return false;
        if (acc > (0xFFFFFFFFFFFFFFFFULL - d) / 10) return false;   // ParseUint range error
        acc = acc * 10 + d;
    }
    if (!neg && acc >= 0x8000000000000000ULL) return false;        // ParseInt range error
    if (neg && acc > 0x8000000000000000ULL) return false;
    *out = neg ? (int64_t)(0 - acc) : (int64_t)acc;
    return true;
}

__global__ void k_atoi(const uint8_t *__restrict__ bytes, const uint64_t *__restrict__ off, uint64_t n,
                       uint8_t *__restrict__ ok, int64_t *__restrict__ val) {
    for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < n; s += (uint64_t)gridDim.x * 256) {
        int64_t v = 0;
        const bool good = go_atoi(bytes + off[s], off[s + 1] - off[s], &v);
        ok[s] = good;
        val[s] = good ? v : 0;
    }
}

// ---------------------------------------------------------------- walk + replay
// Tiled merge path.  Per replica the new Diff is the merge of L and R (L
// first on an equal ts) keeping every L entry and the R entries that are
// "inserted" (below max(L), not equal to the L entry just before them in
// merge order).  Each replica's merge sequence (|L|+|R| items) is cut into
// tiles of MT items; every tile pass loads one 64-B descriptor and stages
// its L and R ranges in LDS with coalesced loads.
//   k_rm_plan_small / scan : tiles per replica;
//   k_rm_split : one wave per tile: its geometry and 16-ary merge-path split
//                -> descriptors (plus the Atoi / accumulator-reset prep);
//   k_rm_count : merge (512 threads x 8 items): inserted-R count per tile and
//                the merge-order bitmaps;
//   scan of the counts -> each tile's output offset, out.off;
//   k_rm_tile  : re-merge (512 threads x FI items), each entry's rank among
//                the tile's emitted entries; the tile's new-Diff slice
//                staged in LDS by rank and written coalesced; the replay
//                (main.go:75-98) of the tile's emitted remote-origin entries
//                into an LDS table keyed by slot, flushed with one set of
//                global atomics per (tile, slot);
//   k_slot_final: per-slot closed form.
// The replay's per-key state is order-free: best = max over holders of
// (rank in the replica's merge sequence) << 32 | string id (the max-ts
// holder, since the merge sequence is ts-ascending), plus the wrapped sum
// and count of the parsable values; so tiles fold independently.  (Per-entry
// binary searches over the logs, and a per-replica replay pass re-reading
// the new Diff, were each bound by chains of dependent global loads; every
// tile pass here is still latency-bound at 2-4 TB/s, see DESIGN.md.)
constexpr int MT = 4096;                  // merge items per tile
constexpr int MB = 512;                   // threads per tile (count pass)
constexpr int TT = 512;                   // LDS replay-table entries per tile
constexpr int FB = 1024;                  // threads of the tile pass (one tile each)
constexpr int NW = MT / 64;               // 64-bit words per merge bitmap of a tile
constexpr int FI = MT / FB;               // entries per fold thread
#ifndef RM_SPLIT_PW
#define RM_SPLIT_PW 16                    // merge-path search width (probing lanes)
#endif
constexpr uint32_t OKC = 256;             // string tables up to this size are staged in the fold's LDS
constexpr uint32_t kEmpty = 0xFFFFFFFFu;

struct TileGeo {                          // 64 B per tile (per-replica geometry)
    uint64_t lb, nl, rb, nr, d0, d1;
    int64_t maxl;
    uint32_t p, first;                    // replica; first tile of the replica
};

struct TileDesc {                         // 64 B per tile; a tile pass loads its own and the next one
    uint64_t l0, r0;                      // global index of the tile's first L / R entry
    uint64_t d0;                          // the tile's first diagonal in the replica's merge sequence
    int64_t maxl;                         // insert below this (max(L) of the replica)
    int64_t lprev;                        // L entry just before the tile (valid if has_prev)
    uint64_t lend;                        // end of the replica's L (global index)
    uint32_t n;                           // merge items of the tile; 0: no tile
    uint32_t has_prev;
    uint32_t rsd;                         // added (mod 2^32) to the key slot of every R pair (in-place pulls)
    uint32_t pad;
};

// The batch as the planning kernels see it: the ABI struct plus the
// in-place pull form (crdt_refmerge_batch_pull) -- replica p's R is
// r_ts[r_off[p] .. r_end[p]) (ranges may overlap: R aliases the peers'
// Diffs) and its R pairs' key slots are re-based by r_sd[p].
struct RmIn : crdt_refmerge_in {
    const uint64_t *r_end = nullptr;      // nullptr: CSR, r_off[p + 1]
    const uint32_t *r_sd = nullptr;
};
__device__ __forceinline__ uint64_t r_hi(const RmIn &in, uint32_t p) {
    return in.r_end ? in.r_end[p] : in.r_off[p + 1];
}
// R entries of replica p; a reversed range (r_end < r_off) counts as empty
// and the planning passes raise CRDT_DEV_RANGE for it
__device__ __forceinline__ uint64_t r_len(const RmIn &in, uint32_t p) {
    const uint64_t b = in.r_off[p], e = r_hi(in, p);
    return e > b ? e - b : 0;
}

// The tile's L / R entry counts: its L range ends where the next tile's
// begins (same replica: d0 > 0) or at the replica's L end.
__device__ __forceinline__ void tile_counts(const TileDesc &d, const TileDesc &dn, uint32_t *na, uint32_t *nb) {
    const uint64_t l1 = (dn.n && dn.d0 > 0) ? dn.l0 : d.lend;
    *na = (uint32_t)(l1 - d.l0);
    *nb = d.n - *na;
}

struct alignas(16) OkVal {                // Go Atoi of one arena string: one 16-B gather per lookup
    int64_t val;                          // 0 where !ok
    int64_t ok;
};

struct RpCand {                           // delta replay: a tile's max holder of one slot
    uint64_t key;                         // ts ^ 2^63
    uint32_t slot, str;
};

struct SlotAcc {                          // global replay accumulators, by slot
    unsigned long long *best;             // 0 = slot untouched
    unsigned long long *sum;
    unsigned *npar;
};

// The new Diff's kv pairs (crdt_refmerge_batch_kv): the count pass sums the
// kv pairs of each tile's emitted entries (tkv), the scan turns the sums into
// tile bases (ikv), and the tile pass writes each emitted entry's kv offset
// and copies its pairs -- no separate segmented gather over out.src.
struct KvOut {
    uint64_t *off;                        // nullptr: no kv output
    uint32_t *key, *val;
    uint64_t cap;
    const uint64_t *ikv;                  // per-tile kv base (exclusive scan of tkv)
    const uint32_t *tone;                 // per tile: every emitted entry has exactly one pair
    uint32_t affine = 0;                  // one-pair population: every entry one pair, entry e's at kv[0] + e
};

// kv pairs of an entry's range [kb, ke), clamped to the arena (malformed
// ranges stay in bounds); the count and tile passes both use this
__device__ __forceinline__ uint64_t kv_len(uint64_t kb, uint64_t ke, uint64_t n_kv) {
    const uint64_t e = ke < n_kv ? ke : n_kv;
    return kb < e ? e - kb : 0;
}

__global__ void k_rm_ntiles(RmIn in, uint32_t *__restrict__ nt, uint32_t *__restrict__ err) {
    for (uint32_t p = blockIdx.x * 256 + threadIdx.x; p < in.replicas; p += gridDim.x * 256) {
        if (r_hi(in, p) < in.r_off[p]) atomicOr(err, CRDT_DEV_RANGE);
        const uint64_t n = (in.l_off[p + 1] - in.l_off[p]) + r_len(in, p);
        nt[p] = (uint32_t)((n + MT - 1) / MT);
    }
}

// Go Atoi of strings i (okv) and the reset of replay accumulator i, for
// i = i0, i0 + stride, ...
__device__ __forceinline__ void prep_items(const uint8_t *__restrict__ bytes, const uint64_t *__restrict__ off,
                                           uint64_t nstr, OkVal *__restrict__ okv, SlotAcc acc, uint32_t ns,
                                           uint64_t i0, uint64_t stride) {
    const uint64_t n = nstr > ns ? nstr : ns;
    for (uint64_t i = i0; i < n; i += stride) {
        if (i < nstr) {
            int64_t v = 0;
            const bool good = go_atoi(bytes + off[i], off[i + 1] - off[i], &v);
            okv[i].val = good ? v : 0;
            okv[i].ok = good;
        }
        if (i < ns) {
            acc.best[i] = 0;
            acc.sum[i] = 0;
            acc.npar[i] = 0;
        }
    }
}

// Merge-path split of diagonal d (first d items of the merge): the number of
// L items among them.  One wave, PW-ary (lanes 0..PW-1 probe): the pass is
// bound by the scattered probe loads, not by the rounds -- 256-ary (4 probes
// per lane) took 53 us, 64-ary 23 us, 32-ary 18.6 us, 16-ary 15.2 us for
// 10.6k tiles of 10k-entry logs.
// pred(a) = L[a] <= R[d-1-a] holds for a < split and fails from it on.
// *lprev = L[split - 1] when split > 0: a raise of lo always comes from a
// probe of L[new lo - 1], so it is shuffled out of the search and only a
// split that never moved off its lower bound loads it.
template <int PW>
__device__ __forceinline__ uint64_t wave_split(const int64_t *L, uint64_t nl, const int64_t *R, uint64_t nr,
                                               uint64_t d, int lane, int64_t *lprev) {
    constexpr int K = 1;                                 // probe j = lane * K + k (lane < PW)
    uint64_t lo = d > nr ? d - nr : 0, hi = d < nl ? d : nl;
    const uint64_t lo0 = lo;
    int64_t lp = 0;
    while (lo < hi) {
        const uint64_t step = (hi - lo + PW * K - 1) / (PW * K);
        int64_t lv[K], rv[K];
        bool valid[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t a = lo + (uint64_t)(lane * K + k) * step;
            valid[k] = lane < PW && a < hi;
            lv[k] = valid[k] ? L[a] : 0;
            rv[k] = valid[k] ? R[d - 1 - a] : 0;
        }
        int c = 0, nv = 0;                               // monotone over j: probes 0..c-1 hold
#pragma unroll
        for (int k = 0; k < K; ++k) {
            c += __popcll(__ballot(valid[k] && lv[k] <= rv[k]));
            nv += __popcll(__ballot(valid[k]));
        }
        const int jc = c ? c - 1 : 0;
        int64_t mine = lv[0];
#pragma unroll
        for (int k = 1; k < K; ++k) mine = (jc % K) == k ? lv[k] : mine;
        const int64_t lc = __shfl(mine, jc / K);
        if (c) lp = lc;                                  // L[nlo - 1]
        const uint64_t nlo = c ? lo + (uint64_t)(c - 1) * step + 1 : lo;
        const uint64_t nhi = c < nv ? lo + (uint64_t)c * step : hi;
        lo = nlo;
        hi = nhi;
    }
    *lprev = lo > lo0 ? lp : lo > 0 ? L[lo - 1] : 0;
    return lo;
}

// The geometry of tile t from tbase (exclusive scan of the tiles per
// replica): its replica is the last p with tbase[p] <= t (replicas with no
// tile share their successor's tbase and are skipped by the search).
// maxl_ovr (nullable): per-replica max(L) to insert below, instead of the
// local L's last key (the ts-range-sharded merge passes the global max).
__device__ __forceinline__ TileGeo tile_geo(const RmIn &in, const uint64_t *__restrict__ tbase,
                                            const int64_t *__restrict__ maxl_ovr, uint64_t t) {
    uint32_t lo = 0, hi = in.replicas;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (tbase[mid] <= t) lo = mid;
        else hi = mid;
    }
    TileGeo g;
    g.p = lo;
    g.lb = in.l_off[lo];
    g.nl = in.l_off[lo + 1] - g.lb;
    g.rb = in.r_off[lo];
    g.nr = r_len(in, lo);
    g.maxl = maxl_ovr ? maxl_ovr[lo] : g.nl ? in.l_ts[g.lb + g.nl - 1] : INT64_MIN;   // empty L: nothing inserted
    g.first = (uint32_t)tbase[lo];
    g.d0 = (t - tbase[lo]) * MT;
    g.d1 = g.d0 + MT < g.nl + g.nr ? g.d0 + MT : g.nl + g.nr;
    return g;
}

// Tile descriptors: one wave per tile computes the tile's geometry and the
// merge-path split at its first diagonal and packs the tile's ranges (its
// end is the next descriptor's start); slots past the tile count get an
// empty descriptor.  The same launch runs the Atoi / accumulator-reset prep
// (independent work).
__global__ __launch_bounds__(256) void k_rm_split(RmIn in, uint32_t replicas,
                                                  const uint64_t *__restrict__ tbase,
                                                  const int64_t *__restrict__ maxl_ovr, uint64_t tmax,
                                                  TileDesc *__restrict__ desc, OkVal *__restrict__ okv, SlotAcc acc,
                                                  uint32_t ns, uint32_t *__restrict__ err) {
    const uint64_t t = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    prep_items(in.str_bytes, in.str_off, in.n_str, okv, acc, ns, (uint64_t)blockIdx.x * 256 + threadIdx.x,
               (uint64_t)gridDim.x * 256);
    if (t > tmax) return;                                // desc[tmax]: always an empty sentinel
    TileDesc d = {};
    // more tiles than planned (R ranges summing past n_r): every tile left
    // empty -- nothing is read or written past the sizes the call was given
    const uint64_t tiles = tbase[replicas];
    if (tiles > tmax && t == 0 && lane == 0) atomicOr(err, CRDT_DEV_RANGE);
    if (t < tiles && tiles <= tmax) {
        const TileGeo g = tile_geo(in, tbase, maxl_ovr, t);
        int64_t lprev;
        const uint64_t a0 = wave_split<RM_SPLIT_PW>(in.l_ts + g.lb, g.nl, in.r_ts + g.rb, g.nr, g.d0, lane, &lprev);
        d.l0 = g.lb + a0;
        d.r0 = g.rb + (g.d0 - a0);
        d.d0 = g.d0;
        d.maxl = g.maxl;
        d.lend = g.lb + g.nl;
        d.n = (uint32_t)(g.d1 - g.d0);
        d.has_prev = a0 > 0;
        d.lprev = lprev;
        d.rsd = in.r_sd ? in.r_sd[g.p] : 0u;
    }
    if (lane == 0) desc[t] = d;
}

// (A padded LDS image of the tile, element i at i + i / 8 against the
// 32-byte stride of a wave's merge-path probes, measured slower: count
// 45.9 -> 48.7 us.)

// Stage the tile's merge items in LDS: every thread issues its NT loads
// before the first store (a load / store per item in turn left the pass
// waiting on its serial HBM round trips).
template <int NT>
__device__ __forceinline__ void load_tile_ts(const crdt_refmerge_in &in, const TileDesc &d, uint32_t na, uint32_t n,
                                             int64_t *sm) {
    constexpr int NI = MT / NT;
    int64_t v[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) {
        const uint32_t k = threadIdx.x + (uint32_t)j * NT;
        v[j] = k < na ? in.l_ts[d.l0 + k] : k < n ? in.r_ts[d.r0 + (k - na)] : 0;
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
        const uint32_t k = threadIdx.x + (uint32_t)j * NT;
        if (k < n) sm[1 + k] = v[j];
    }
    if (threadIdx.x == 0) sm[0] = d.lprev;
    __syncthreads();
}

// SA[0..na) = L[a0..a1), SB[0..nb) = R[b0..b1) (LDS), lprev = L[a0-1] (when a0 > 0).
// Thread-level merge of diagonals [k0, k1) of the tile: bit i of *isl / *emit
// = item i is an L entry / is emitted.  Returns the split (ia) at k0.
__device__ __forceinline__ uint32_t thread_merge(const int64_t *SA, const int64_t *SB, int64_t lprev, uint32_t na,
                                                 uint32_t nb, uint32_t k0, uint32_t k1, bool has_prev0, int64_t maxl,
                                                 uint32_t *isl, uint32_t *emit) {
    uint32_t lo = k0 > nb ? k0 - nb : 0, hi = k0 < na ? k0 : na;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (SA[mid] <= SB[k0 - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    uint32_t ia = lo, ib = k0 - lo;
    const uint32_t ia0 = ia;
    uint32_t fl = 0, fe = 0;
    // the two heads and the L entry before the L head stay in registers: one
    // LDS read (the new head) per step
    int64_t ha = ia < na ? SA[ia] : 0, hb = ib < nb ? SB[ib] : 0;
    int64_t pl = ia ? SA[ia - 1] : lprev;                // L entry just before (global a0+ia-1)
    bool hp = ia > 0 || has_prev0;
    for (uint32_t k = k0, i = 0; k < k1; ++k, ++i) {
        const bool take_l = ia < na && (ib >= nb || ha <= hb);
        if (take_l) {
            fl |= 1u << i;
            fe |= 1u << i;
            pl = ha;
            hp = true;
            ++ia;
            if (ia < na) ha = SA[ia];
        } else {
            if (hb < maxl && !(hp && pl == hb)) fe |= 1u << i;
            ++ib;
            if (ib < nb) hb = SB[ib];
        }
    }
    *isl = fl;
    *emit = fe;
    return ia0;
}

template <int NT>
__device__ __forceinline__ uint32_t block_excl_sum(uint32_t v, uint32_t *s_w, uint32_t *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) {
        base += k < w ? s_w[k] : 0;
        tot += s_w[k];
    }
    *total = tot;
    return base + x - v;
}

__device__ __forceinline__ uint32_t table_find(uint32_t *t_slot, uint32_t slot) {
    uint32_t h = (slot * 2654435761u) >> 23;             // 9-bit hash
    for (int probe = 0; probe < 16; ++probe, h = (h + 1) & (TT - 1)) {
        uint32_t c = t_slot[h];                          // plain read first: most pairs hit a claimed entry
        if (c == kEmpty) c = atomicCAS(&t_slot[h], kEmpty, slot);
        if (c == kEmpty || c == slot) return h;
    }
    return kEmpty;
}

// Fold one (slot, string) pair of a remote-origin entry whose rank in the
// replica's merge sequence is `rank` (>= 1).
__device__ __forceinline__ void fold_pair(uint32_t *t_slot, unsigned long long *t_best, unsigned long long *t_sum,
                                          uint32_t *t_npar, const SlotAcc &acc, bool use_lds, uint32_t slot,
                                          uint32_t v, uint64_t rank, bool okv, int64_t x) {
    const unsigned long long best = (rank << 32) | v;
    const uint32_t idx = use_lds ? table_find(t_slot, slot) : kEmpty;
    if (idx != kEmpty) {
        atomicMax(&t_best[idx], best);
        if (okv) {
            atomicAdd(&t_sum[idx], (unsigned long long)x);   // mod 2^64 (main.go:95)
            atomicAdd(&t_npar[idx], 1u);
        }
    } else {                                             // table full: straight to the slot
        atomicMax(&acc.best[slot], best);
        if (okv) {
            atomicAdd(&acc.sum[slot], (unsigned long long)x);
            atomicAdd(&acc.npar[slot], 1u);
        }
    }
}

// Pass 1: the merge of each tile's ts in LDS (one merge per tile, the only
// one): its inserted-R count, and the merge written out as two bitmaps in
// merge order -- bit k of isl = merge item k is an L entry, bit k of emit =
// it is emitted (every L entry; the inserted R entries) -- 512 B per tile,
// bits[t * 64 + w] (w < 32: isl words, w >= 32: emit words).  The tile pass
// reads every entry's position from them instead of merging again (a
// second merge in the tile pass, or a 2-byte rank per entry written and
// read back, each cost more).  Grid = the tile-count upper bound.
template <int NT, bool KV = false>
__global__ __launch_bounds__(NT) void k_rm_count(crdt_refmerge_in in, const TileDesc *__restrict__ desc,
                                                 uint32_t *__restrict__ tcnt, uint64_t *__restrict__ bits,
                                                 uint32_t *__restrict__ zero, int dma, uint64_t *__restrict__ tkv,
                                                 uint32_t *__restrict__ tone, uint32_t *__restrict__ err,
                                                 int one_pair = 0) {
    constexpr int NI = MT / NT, LPW = 64 / NI;           // items per thread, lanes per bitmap word
    static_assert(NI * LPW == 64, "a bitmap word is LPW lanes' items");
    __shared__ alignas(16) int64_t sm[MT + 8];           // (DMA: each run from its 16-byte aligned-down start)
    __shared__ uint32_t s_w[NT / 64];
    __shared__ uint64_t s_k[KV ? NT / 64 : 1];
    __shared__ uint8_t s_emr[KV ? MT : 1];               // KV: emitted flag of each R entry of the tile
    const uint64_t t = blockIdx.x;
    if (zero && t == 0 && threadIdx.x == 0) *zero = 0;   // (the delta fold's overflow flag)
    const TileDesc d = desc[t], dn = desc[t + 1];
    uint32_t na, nb;
    tile_counts(d, dn, &na, &nb);
    const uint32_t n = na + nb;
    if (n == 0) {
        if (threadIdx.x == 0) {
            tcnt[t] = 0;                                 // the scans run over the whole grid
            if (KV) {
                tkv[t] = 0;
                tone[t] = 1;
            }
        }
        return;
    }
    const int64_t *SA, *SB;
    if (dma) {                                           // LDS-DMA staging (no VGPR round trip)
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), ln = threadIdx.x & 63;
        uint32_t at = 0;
        const int oa = dma_run<int64_t, NT / 64>(in.l_ts, d.l0, na, sm, &at, wv, ln);
        const int ob = dma_run<int64_t, NT / 64>(in.r_ts, d.r0, nb, sm, &at, wv, ln);
        SA = sm + oa;
        SB = sm + ob;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA has landed in LDS
        __syncthreads();
    } else {
        load_tile_ts<NT>(in, d, na, n, sm);
        SA = sm + 1;
        SB = sm + 1 + na;
    }
    const uint32_t k0 = threadIdx.x * NI < n ? threadIdx.x * NI : n;
    const uint32_t k1 = k0 + NI < n ? k0 + NI : n;
    uint32_t isl = 0, emit = 0, ia0 = 0;
    if (k0 < k1) ia0 = thread_merge(SA, SB, d.lprev, na, nb, k0, k1, d.has_prev, d.maxl, &isl, &emit);
    uint64_t ks = 0;                                     // KV: kv pairs of the tile's emitted entries
    int one = 1;                                         // KV: every emitted entry has exactly one pair
    if (KV && one_pair) {                                // (the caller's invariant: one pair per entry)
        ks = (uint64_t)__popc(emit);
    } else if (KV) {
        // the merge marks its emitted R entries by R index in LDS; then the
        // kv ranges are read in index order (coalesced, all loads in flight):
        // every L entry of the tile, the marked R entries
        if (k0 < k1) {
            const uint32_t ib0 = k0 - ia0;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const uint32_t nlb = (uint32_t)__popc(isl & ((1u << i) - 1u));
                if (k0 + i < k1 && !((isl >> i) & 1u)) s_emr[ib0 + (uint32_t)i - nlb] = (uint8_t)((emit >> i) & 1u);
            }
        }
        __syncthreads();
        // an item's range end is the next item's start (the next lane's
        // load) except at a wave's last lane and the ends of the L and R runs
        uint64_t kb[NI], ke[NI];
        bool on[NI];
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int j = 0; j < NI; ++j) {
            const uint32_t k = threadIdx.x + (uint32_t)j * NT;
            const bool il = k < na;
            const uint32_t idx = il ? k : k - na;
            on[j] = k < n && (il || s_emr[idx]);
            const uint64_t *kp = il ? in.l_kv + (d.l0 + idx) : in.r_kv + (d.r0 + idx);
            kb[j] = k < n ? kp[0] : 0;
            ke[j] = (k < n && (lane == 63 || k + 1 == na || k + 1 == n)) ? kp[1] : 0;
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
            const uint32_t k = threadIdx.x + (uint32_t)j * NT;
            const uint64_t nx = __shfl_down(kb[j], 1);
            if (!(lane == 63 || k + 1 == na || k + 1 == n)) ke[j] = nx;
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
            const uint64_t len = on[j] ? kv_len(kb[j], ke[j], in.n_kv) : 0;
            ks += len;
            one &= !on[j] || len == 1;
        }
    }
    // LPW lanes' item bits -> one 64-bit word of each bitmap
    const int lane = threadIdx.x & 63, sh = (lane % LPW) * NI;
    uint64_t wl = (uint64_t)isl << sh, we = (uint64_t)emit << sh;
#pragma unroll
    for (int o = 1; o < LPW; o <<= 1) {
        wl |= (uint64_t)__shfl_xor((unsigned long long)wl, o);
        we |= (uint64_t)__shfl_xor((unsigned long long)we, o);
    }
    if (lane % LPW == 0) {
        const uint32_t w = threadIdx.x / LPW;
        bits[t * 2 * NW + w] = wl;
        bits[t * 2 * NW + NW + w] = we;
    }
    uint32_t x = (uint32_t)__popc(emit & ~isl);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        x += __shfl_xor(x, o);
        if (KV) ks += __shfl_xor(ks, o);
    }
    if (lane == 0) {
        s_w[threadIdx.x >> 6] = x;
        if (KV) s_k[threadIdx.x >> 6] = ks;
    }
    if (KV) one = __syncthreads_and(one);
    else __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        uint64_t ktot = 0;
#pragma unroll
        for (int k = 0; k < NT / 64; ++k) {
            tot += s_w[k];
            if (KV) ktot += s_k[k];
        }
        tcnt[t] = tot;
        if (KV) {
            tkv[t] = ktot;
            tone[t] = (uint32_t)one;
            if (ktot >= 0xFFFFFFFFull) atomicOr(err, CRDT_DEV_RANGE);   // (the tile pass sums in 32 bits)
        }
    }
}

enum { RM_FOLD_NONE = 0, RM_FOLD_FULL = 1, RM_FOLD_DELTA = 2 };

// Pass 2, one workgroup per tile, in merge order: wave w's lanes take merge
// items k = 64 (w + NWV i) + lane (i < FI), so each load instruction covers 64
// consecutive merge items -- two contiguous runs, one of L and one of R.  An
// item's L / R index and its rank among the tile's emitted entries are
// prefix counts of the count pass's bitmaps (one word per wave and item
// slot: the word prefix by shuffles over the tile's 64 words, the bit
// prefix by mbcnt), so no merge, LDS staging or barrier stands before the
// entry loads.  Emitted entries are stored straight from registers at
// their rank in the tile's slice (consecutive across the emitting lanes).
// The replay fold (main.go:75-98) of the emitted remote-origin entries runs
// into an LDS table keyed by slot, flushed with one set of global atomics
// per (tile, slot).  An entry's rank in the replica's merge sequence (d0 +
// its 1-based rank in the tile) orders the replica's new Diff like its ts,
// so best = rank << 32 | string id picks the max-ts holder without knowing
// output positions.  Further kvs of an entry (rare: the reference's load
// generator writes one kv per entry) take a tail loop.
//   FOLD == RM_FOLD_NONE : slice write only (no slots, or the timing diag)
//   FOLD == RM_FOLD_FULL : + the replay fold into acc
//   FOLD == RM_FOLD_DELTA: + the incremental replay's first phase -- only
//        the inserted R entries, keyed by ts ^ 2^63, into the carried state st
//        (max, holder count, wrapped sum, parsable count); each R entry's
//        rank (0: not inserted) goes to r_dk for the holder pass's
//        overflow walk.
template <int FOLD, int PARTS, bool KV, bool ONE = false, bool NTH = true>
__device__ __forceinline__ void rm_tile(const crdt_refmerge_in &in, const TileDesc *__restrict__ desc,
                                        const uint64_t *__restrict__ bits, uint16_t *__restrict__ r_dk,
                                        const OkVal *__restrict__ okv, const SlotAcc &acc, int diag,
                                        const uint64_t *__restrict__ ic, const crdt_refmerge_out &out,
                                        const crdt_replay_state &st, RpCand *__restrict__ cand,
                                        uint32_t *__restrict__ cand_n, uint32_t *__restrict__ ovf,
                                        uint32_t *__restrict__ err, const KvOut &kvo) {
    // PARTS > 1: each workgroup takes 1/PARTS of the tile's items (words
    // WPP h .. WPP h + WPP - 1) with FB / PARTS threads and its own slot table
    constexpr int WT = FB / PARTS, NWV = WT / 64, WPP = NW / PARTS;   // threads, waves, words per workgroup
    static_assert(FI * NWV == WPP, "each wave takes FI words of 64 items");
    constexpr bool DELTA = FOLD == RM_FOLD_DELTA, FOLDS = FOLD != RM_FOLD_NONE;
    static_assert(!DELTA || PARTS == 1, "the delta fold keeps one candidate list per tile");
    static_assert(!KV || (PARTS == 1 && !DELTA), "the kv prefix spans the whole tile");
    static_assert(WT >= (int)OKC, "one thread per staged Atoi record");
    constexpr int TN = FOLDS ? TT : 1;
    __shared__ uint32_t t_slot[TN];
    __shared__ uint32_t t_nh[DELTA ? TT : 1];
    __shared__ unsigned long long t_key[DELTA ? TT : 1];   // DELTA: max ts ^ 2^63 of each entry
    __shared__ uint32_t s_nc, s_ovf;
    __shared__ unsigned long long t_best[TN];
    __shared__ unsigned long long t_sum[TN];
    __shared__ uint32_t t_npar[TN];
    __shared__ int64_t s_okval[FOLDS ? OKC : 1];
    __shared__ uint8_t s_okok[FOLDS ? OKC : 1];
    __shared__ uint32_t s_wk[KV ? NW : 1];              // KV: kv pairs per bitmap word
    const uint64_t t = blockIdx.x / PARTS;
    const int part = (int)(blockIdx.x % PARTS);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // KV: one-pair tiles (the common case: offset = tile base + rank, no
    // prefix pass) and the rest go to two launches of the pass
    if (KV && (kvo.tone[t] != 0) != ONE) return;
    // the descriptors, the tile's bitmap words (one of each bitmap per lane),
    // its offset and the staged Atoi records are independent loads: all issued
    // before the first use (the empty-tile exit would otherwise order them)
    static_assert(NW == 64, "one word of each bitmap per lane");
    const TileDesc d = desc[t], dn = desc[t + 1];
    const uint64_t word_l = bits[t * 2 * NW + lane], word_e = bits[t * 2 * NW + NW + lane];
    const uint64_t ict = ic[t];
    const uint64_t ikt = KV ? kvo.ikv[t] : 0;
    const bool okc = FOLDS && in.n_str <= OKC;
    OkVal ok0 = OkVal{0, 0};
    if (okc && threadIdx.x < in.n_str) ok0 = okv[threadIdx.x];
    uint32_t na, nb;
    tile_counts(d, dn, &na, &nb);
    const uint32_t n = na + nb;
    if (n == 0) {
        if (DELTA && threadIdx.x == 0) cand_n[t] = 0;
        return;
    }
    uint32_t pre_l = (uint32_t)__popcll(word_l), pre_e = (uint32_t)__popcll(word_e);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t yl = __shfl_up(pre_l, o), ye = __shfl_up(pre_e, o);
        if (lane >= o) {
            pre_l += yl;
            pre_e += ye;
        }
    }
    pre_l -= (uint32_t)__popcll(word_l);
    pre_e -= (uint32_t)__popcll(word_e);
    // every L / R index and output rank below derives from the bitmaps: a
    // tile whose bitmaps set a bit past its n items or do not hold exactly
    // its na L entries raises CRDT_DEV_RANGE instead of reading out of range
    {
        const uint32_t lo = 64u * (uint32_t)lane;
        const uint64_t valid = lo >= n ? 0ull : (n - lo >= 64u ? ~0ull : (1ull << (n - lo)) - 1);
        const bool bad = ((word_l | word_e) & ~valid) != 0;
        const uint32_t tot_l = (uint32_t)__builtin_amdgcn_readlane((int)(pre_l + (uint32_t)__popcll(word_l)), 63);
        if (__ballot(bad) != 0 || tot_l != na) {
            if (threadIdx.x == 0 && part == 0) atomicOr(err, CRDT_DEV_RANGE);
            if (DELTA && threadIdx.x == 0) cand_n[t] = 0;
            return;
        }
    }
    const uint64_t ob = d.l0 + ict;
    if (DELTA && threadIdx.x == 0) s_nc = s_ovf = 0;
    if (FOLDS)
        for (int h = threadIdx.x; h < TT; h += WT) {
            t_slot[h] = kEmpty;
            t_best[h] = 0;
            t_sum[h] = 0;
            t_npar[h] = 0;
            if (DELTA) {
                t_nh[h] = 0;
                t_key[h] = 0;
            }
        }
    // a small string table (the reference's load generator writes ten
    // values, main.go:282) is staged in LDS: the Atoi lookup leaves the
    // chain of dependent global loads (kv range -> kv pair -> Atoi record)
    if (okc && threadIdx.x < in.n_str) {
        s_okval[threadIdx.x] = ok0.val;
        s_okok[threadIdx.x] = (uint8_t)(ok0.ok != 0);
    }
    // per item slot f: merge item k = 64 * (wv + NWV f) + lane.  The words
    // and their prefixes are wave-uniform (scalar registers); an item's
    // flags, L / R index and rank are recomputed from them where used.
    uint64_t s_wl[FI], s_we[FI];
    uint32_t s_pl[FI], s_pe[FI];
    const int wvu = __builtin_amdgcn_readfirstlane(wv) + WPP * part;   // this wave's first word
#pragma unroll
    for (int f = 0; f < FI; ++f) {
        const int w = wvu + NWV * f;
        // (readlane returns int: widen through uint32_t, never sign-extend)
        s_wl[f] = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(word_l >> 32), w) << 32) |
                  (uint32_t)__builtin_amdgcn_readlane((uint32_t)word_l, w);
        s_we[f] = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(word_e >> 32), w) << 32) |
                  (uint32_t)__builtin_amdgcn_readlane((uint32_t)word_e, w);
        s_pl[f] = (uint32_t)__builtin_amdgcn_readlane(pre_l, w);
        s_pe[f] = (uint32_t)__builtin_amdgcn_readlane(pre_e, w);
    }
    auto below = [&](uint64_t m) -> uint32_t {          // set bits of m below this lane
        return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    };
    auto it_in = [&](int f) { return 64u * (uint32_t)(wvu + NWV * f) + (uint32_t)lane < n; };
    auto it_l = [&](int f) { return (bool)((s_wl[f] >> lane) & 1); };
    auto it_em = [&](int f) { return (bool)((s_we[f] >> lane) & 1); };
    auto it_rk = [&](int f) { return s_pe[f] + below(s_we[f]); };        // rank among the emitted (0-based)
    auto it_gi = [&](int f) -> uint64_t {                                // global L / R index
        const uint32_t li = s_pl[f] + below(s_wl[f]);
        return it_l(f) ? d.l0 + li : d.r0 + (64u * (uint32_t)(wvu + NWV * f) + (uint32_t)lane - li);
    };
    uint64_t e_kb[FI], e_ke[FI];
    uint32_t k_c[FI];
    int64_t e_ts[FI];
    uint32_t e_cnt[FI], e_slot[FI], e_v[FI];
    uint32_t cmask = 0;                                  // KV: bit f = replay candidate (its count is k_c[f])
    uint8_t e_org[FI];
    // ONE (one-pair populations): every entry of L and of the pulled ranges
    // holds exactly one pair and the pairs lie in entry order -- entry gi's
    // pair at kv[0] + gi -- so no range is loaded: the pair loads issue with
    // the ts loads instead of behind a kv range load
    uint64_t kl0 = 0, kr0 = 0;
    const bool aff = ONE && kvo.affine;                  // (uniform)
    if (aff) {
        kl0 = in.n_l ? in.l_kv[0] : 0;
        kr0 = in.n_r ? in.r_kv[0] : 0;
    }
#pragma unroll
    for (int f = 0; f < FI; ++f) {                       // every entry load issued before the first use
        // (only emitted entries are written or folded: an R entry whose ts L
        // already holds loads nothing)
        const bool in_tile = it_in(f) && it_em(f), il = it_l(f);
        const uint64_t gi = it_gi(f);
        const uint64_t *kv = (il ? in.l_kv : in.r_kv) + gi;
        e_ts[f] = in_tile ? (il ? in.l_ts[gi] : in.r_ts[gi]) : 0;
        // nontemporal hints on the once-touched origin and kv-range loads and on
        // the slice / kv stores (profiles/r06/ab/refmerge_nontemporal.txt: gossip
        // round -12 %, delta -3 %, RefMerge -1 %).  Not on the pair loads: they
        // lose their Infinity Cache hits (the gossip round's gain halves).  NTH =
        // false for a merge whose R side the device has just written (the wire
        // round's decode, crdt_ctx::rm_nt; hinted there: +2.5 %).  The choice is
        // a template parameter: a run-time select between a hinted and a plain
        // access of one address is merged by the compiler into a plain one.
        e_org[f] = (in_tile && il) ? (NTH ? __builtin_nontemporal_load(in.l_origin + gi) : in.l_origin[gi]) : 0;
        if (aff) e_kb[f] = (il ? kl0 : kr0) + gi;
        else e_kb[f] = ((FOLDS || KV) && in_tile) ? (NTH ? __builtin_nontemporal_load(kv) : kv[0]) : 0;
        e_ke[f] = ((FOLDS || KV) && !ONE && in_tile) ? (NTH ? __builtin_nontemporal_load(kv + 1) : kv[1]) : 0;   // (ONE: every emitted range has one pair)
    }
    if (FOLDS || KV) {
#pragma unroll
        for (int f = 0; f < FI; ++f) {
            // *Command values are skipped by the replay (main.go:80); the
            // delta folds only the inserted R entries
            const bool cand_e = FOLDS && it_em(f) && !e_org[f] && !(DELTA && it_l(f));
            const uint64_t len = ONE ? 1 : kv_len(e_kb[f], e_ke[f], in.n_kv);
            e_cnt[f] = (!KV && cand_e) ? (uint32_t)(len < 0xFFFFFFFFull ? len : 0xFFFFFFFFull) : 0;
            if (KV && cand_e) cmask |= 1u << f;
            // KV: every emitted entry's pairs are copied (a tile of >= 2^32
            // pairs is flagged below, so 32-bit counts are exact where used)
            k_c[f] = (KV && it_em(f)) ? (uint32_t)(len < 0xFFFFFFFFull ? len : 0xFFFFFFFFull) : 0;
        }
#pragma unroll
        for (int f = 0; f < FI; ++f) {
            const bool first = KV ? k_c[f] != 0 : e_cnt[f] != 0;
            e_slot[f] = first ? in.kv_key[e_kb[f]] + (it_l(f) ? 0u : d.rsd) : 0xFFFFFFFFu;
            e_v[f] = first ? in.kv_val[e_kb[f]] : 0xFFFFFFFFu;
        }
    }
    // KV: each emitted entry's kv offset = the tile's base + the pairs of the
    // emitted entries before it in merge order (word-major: word w, then
    // lane): a count per word through LDS (one barrier, while the kv pairs
    // are still in flight), its prefix over the words, then the lane's
    // prefix within its word.  (32-bit sums: a tile of >= 2^32 pairs is
    // flagged by the count pass; its offsets are then garbage, but every
    // write stays in bounds.)  One pair per entry (the reference's load
    // generator): the lane's prefix is a ballot count; otherwise a wave scan.
    auto lane_pre = [&](int f, uint32_t *tot) -> uint32_t {
        const uint64_t one = __ballot(k_c[f] != 0), multi = __ballot(k_c[f] > 1);
        if (!multi) {
            *tot = (uint32_t)__popcll(one);
            return below(one);
        }
        uint32_t x = k_c[f];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        *tot = (uint32_t)__builtin_amdgcn_readlane(x, 63);
        return x - k_c[f];
    };
    uint32_t wx = 0;                                     // KV: lane w = pairs of words before word w
    if constexpr (KV && !ONE) {
#pragma unroll
        for (int f = 0; f < FI; ++f) {
            uint32_t tot;
            (void)lane_pre(f, &tot);
            if (lane == 0) s_wk[wvu + NWV * f] = tot;
        }
        __syncthreads();
        uint32_t wi = s_wk[lane];
        wx = wi;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(wi, o);
            if (lane >= o) wi += y;
        }
        wx = wi - wx;
    }
    // the slice, straight from registers (every L entry of the tile and its
    // inserted R entries, at their rank), and (KV) each entry's kv offset and pairs
#pragma unroll
    for (int f = 0; f < FI; ++f) {
        const bool il = it_l(f), em = it_em(f);
        const uint64_t gi = it_gi(f);
        uint32_t wb = 0, lp = 0;
        if (KV && !ONE) {                                // (wave-uniform parts before any lane leaves)
            uint32_t tot;
            wb = (uint32_t)__builtin_amdgcn_readlane(wx, wvu + NWV * f);
            lp = lane_pre(f, &tot);
        }
        if (em) {
            const uint64_t o = ob + it_rk(f);
            if (o >= in.n_l + in.n_r) {                  // (consistent bitmaps never get here)
                atomicOr(err, CRDT_DEV_RANGE);
                continue;
            }
            if constexpr (NTH) {
                __builtin_nontemporal_store(e_ts[f], &out.ts[o]);
                __builtin_nontemporal_store(il ? (int64_t)gi : -(int64_t)gi - 1, &out.src[o]);
                __builtin_nontemporal_store(e_org[f], &out.origin[o]);
            } else {
                out.ts[o] = e_ts[f];
                out.src[o] = il ? (int64_t)gi : -(int64_t)gi - 1;
                out.origin[o] = e_org[f];
            }
            if (KV) {
                const uint64_t pos = ONE ? ikt + it_rk(f) : ikt + wb + lp;
                if constexpr (NTH) __builtin_nontemporal_store(pos, &kvo.off[o]);
                else kvo.off[o] = pos;
                if (k_c[f] && pos + k_c[f] > kvo.cap) {
                    atomicOr(err, CRDT_DEV_RANGE);
                } else if (k_c[f]) {
                    if constexpr (NTH) {
                        __builtin_nontemporal_store(e_slot[f], &kvo.key[pos]);
                        __builtin_nontemporal_store(e_v[f], &kvo.val[pos]);
                    } else {
                        kvo.key[pos] = e_slot[f];
                        kvo.val[pos] = e_v[f];
                    }
                    for (uint32_t j = 1; j < k_c[f]; ++j) {   // further kvs of the entry (rare)
                        kvo.key[pos + j] = in.kv_key[e_kb[f] + j] + (il ? 0u : d.rsd);
                        kvo.val[pos + j] = in.kv_val[e_kb[f] + j];
                    }
                }
            }
        }
        if (DELTA && it_in(f) && !il) r_dk[gi] = em ? (uint16_t)(it_rk(f) + 1) : (uint16_t)0;
    }
    if (!FOLDS) return;
    if constexpr (KV) {                                  // (the candidates' counts, from k_c)
#pragma unroll
        for (int f = 0; f < FI; ++f) e_cnt[f] = ((cmask >> f) & 1u) ? k_c[f] : 0;
    }
    OkVal e_o[FI];
    if (!okc)
#pragma unroll
        for (int f = 0; f < FI; ++f) {
            e_o[f] = OkVal{0, 0};
            if (e_cnt[f] && e_slot[f] < in.n_slots && e_v[f] < in.n_str) e_o[f] = okv[e_v[f]];
        }
    __syncthreads();                                     // table initialised, Atoi records staged
    if (okc)
#pragma unroll
        for (int f = 0; f < FI; ++f) {
            e_o[f] = OkVal{0, 0};
            if (e_cnt[f] && e_slot[f] < in.n_slots && e_v[f] < in.n_str)
                e_o[f] = OkVal{s_okval[e_v[f]], s_okok[e_v[f]]};
        }
#pragma unroll
    for (int f = 0; f < FI; ++f) {
        if (!e_cnt[f]) continue;
        const uint64_t rank = d.d0 + it_rk(f) + 1;
        const uint64_t key = (uint64_t)e_ts[f] ^ 0x8000000000000000ull;   // DELTA: the ts-keyed max
        const uint64_t kb = e_kb[f];
        for (uint32_t j = 0; j < e_cnt[f]; ++j) {
            uint32_t slot = e_slot[f], v = e_v[f];
            OkVal o = e_o[f];
            if (j) {                                     // further kvs of the entry (rare)
                slot = in.kv_key[kb + j] + (it_l(f) ? 0u : d.rsd);
                v = in.kv_val[kb + j];
                if (slot < in.n_slots && v < in.n_str) o = okv[v];
            }
            if (slot >= in.n_slots || v >= in.n_str) continue;
            if (!DELTA) {
                fold_pair(t_slot, t_best, t_sum, t_npar, acc, true, slot, v, rank, o.ok != 0, o.val);
                continue;
            }
            // within a tile the merge rank orders entries like their ts: the
            // max-rank holder (rank << 32 | string) is the max-ts holder
            const uint32_t idx = table_find(t_slot, slot);
            if (idx != kEmpty) {
                atomicMax(&t_best[idx], (unsigned long long)(rank << 32 | v));
                atomicMax(&t_key[idx], (unsigned long long)key);
                atomicAdd(&t_nh[idx], 1u);
                if (o.ok) {
                    atomicAdd(&t_sum[idx], (unsigned long long)o.val);   // mod 2^64 (main.go:95)
                    atomicAdd(&t_npar[idx], 1u);
                }
            } else {                                     // table full: straight to the state
                s_ovf = 1;                               // (the holder pass then walks the entries)
                atomicMax(reinterpret_cast<unsigned long long *>(&st.best_key[slot]), (unsigned long long)key);
                atomicAdd(&st.nhold[slot], 1u);
                if (o.ok) {
                    atomicAdd(reinterpret_cast<unsigned long long *>(&st.sum[slot]), (unsigned long long)o.val);
                    atomicAdd(&st.npar[slot], 1u);
                }
            }
        }
    }
    __syncthreads();
    if (kDiagBuild && (diag & 255) == 2) return;     // (timing diagnostic: diagnostic build only)
    for (int h = threadIdx.x; h < TT; h += WT) {
        const uint32_t slot = t_slot[h];
        if (slot == kEmpty) continue;
        if (DELTA) {
            const uint32_t c = atomicAdd(&s_nc, 1u);
            cand[t * TT + c] = RpCand{t_key[h], slot, (uint32_t)t_best[h]};
            atomicMax(reinterpret_cast<unsigned long long *>(&st.best_key[slot]), t_key[h]);
            atomicAdd(&st.nhold[slot], t_nh[h]);
            if (t_npar[h]) {
                atomicAdd(reinterpret_cast<unsigned long long *>(&st.sum[slot]), t_sum[h]);
                atomicAdd(&st.npar[slot], t_npar[h]);
            }
            continue;
        }
        atomicMax(&acc.best[slot], t_best[h]);
        if (t_npar[h]) {
            atomicAdd(&acc.sum[slot], t_sum[h]);
            atomicAdd(&acc.npar[slot], t_npar[h]);
        }
    }
    if (DELTA) {
        __syncthreads();
        if (threadIdx.x == 0) {
            cand_n[t] = s_nc;
            if (s_ovf) *ovf = 1;
        }
    }
}

template <int FOLD, int PARTS = 1>
__global__ __launch_bounds__(FB / PARTS, 8) void k_rm_tile(crdt_refmerge_in in, const TileDesc *__restrict__ desc,
                                                const uint64_t *__restrict__ bits, uint16_t *__restrict__ r_dk,
                                                const OkVal *__restrict__ okv, SlotAcc acc, int diag,
                                                const uint64_t *__restrict__ ic, crdt_refmerge_out out,
                                                crdt_replay_state st, RpCand *__restrict__ cand,
                                                uint32_t *__restrict__ cand_n, uint32_t *__restrict__ ovf,
                                                uint32_t *__restrict__ err) {
    rm_tile<FOLD, PARTS, false>(in, desc, bits, r_dk, okv, acc, diag, ic, out, st, cand, cand_n, ovf, err, KvOut{});
}

// the tile pass with the kv output, one-pair tiles (two workgroups per CU)
template <int FOLD, bool NTH = true>
__global__ __launch_bounds__(FB, 8) void k_rm_tile_kv1(crdt_refmerge_in in, const TileDesc *__restrict__ desc,
                                                       const uint64_t *__restrict__ bits, const OkVal *__restrict__ okv,
                                                       SlotAcc acc, int diag, const uint64_t *__restrict__ ic,
                                                       crdt_refmerge_out out, uint32_t *__restrict__ err, KvOut kvo) {
    rm_tile<FOLD, 1, true, true, NTH>(in, desc, bits, nullptr, okv, acc, diag, ic, out, crdt_replay_state{}, nullptr,
                                      nullptr, nullptr, err, kvo);
}

// ... and the other tiles: one workgroup per CU (the kv prefix pass needs
// more than the 64 registers two resident tiles leave a thread)
template <int FOLD, bool NTH = true>
__global__ __launch_bounds__(FB, 4) void k_rm_tile_kv(crdt_refmerge_in in, const TileDesc *__restrict__ desc,
                                                      const uint64_t *__restrict__ bits, const OkVal *__restrict__ okv,
                                                      SlotAcc acc, int diag, const uint64_t *__restrict__ ic,
                                                      crdt_refmerge_out out, uint32_t *__restrict__ err, KvOut kvo) {
    rm_tile<FOLD, 1, true, false, NTH>(in, desc, bits, nullptr, okv, acc, diag, ic, out, crdt_replay_state{}, nullptr,
                                       nullptr, nullptr, err, kvo);
}

// ... and both kinds of tile in one launch, for grids that fit the chip in one
// wave of workgroups (small batches: one launch fewer, occupancy moot)
template <int FOLD, bool NTH = true>
__global__ __launch_bounds__(FB, 4) void k_rm_tile_kvx(crdt_refmerge_in in, const TileDesc *__restrict__ desc,
                                                       const uint64_t *__restrict__ bits, const OkVal *__restrict__ okv,
                                                       SlotAcc acc, int diag, const uint64_t *__restrict__ ic,
                                                       crdt_refmerge_out out, uint32_t *__restrict__ err, KvOut kvo) {
    rm_tile<FOLD, 1, true, true, NTH>(in, desc, bits, nullptr, okv, acc, diag, ic, out, crdt_replay_state{}, nullptr,
                                      nullptr, nullptr, err, kvo);
    rm_tile<FOLD, 1, true, false, NTH>(in, desc, bits, nullptr, okv, acc, diag, ic, out, crdt_replay_state{}, nullptr,
                                       nullptr, nullptr, err, kvo);
}

// Delta replay, second phase: the global max holder of each slot writes its
// string.  Every tile left one candidate (its max holder) per slot it
// touched, so only those are checked -- unless some tile's LDS table
// overflowed (its pairs went straight to the state without a candidate):
// then every inserted R entry is checked.  ts are unique, so exactly one
// holder matches the max.
__global__ __launch_bounds__(64) void k_rp_holder(crdt_refmerge_in in, const uint16_t *__restrict__ r_dk,
                                                  crdt_replay_state st, const RpCand *__restrict__ cand,
                                                  const uint32_t *__restrict__ cand_n,
                                                  const uint32_t *__restrict__ ovf, uint64_t tmax) {
    if (*ovf) {
        for (uint64_t e = (uint64_t)blockIdx.x * 64 + threadIdx.x; e < in.n_r; e += (uint64_t)gridDim.x * 64) {
            if (!r_dk[e]) continue;
            const uint64_t kb = in.r_kv[e], ke = in.r_kv[e + 1] < in.n_kv ? in.r_kv[e + 1] : in.n_kv;
            const uint64_t key = (uint64_t)in.r_ts[e] ^ 0x8000000000000000ull;
            for (uint64_t q = kb; q < ke; ++q) {
                const uint32_t slot = in.kv_key[q], v = in.kv_val[q];
                if (slot >= in.n_slots || v >= in.n_str) continue;
                if (st.best_key[slot] == key) st.best_str[slot] = v;
            }
        }
        return;
    }
    for (uint64_t t = blockIdx.x; t < tmax; t += gridDim.x) {
        const uint32_t n = cand_n[t];
        for (uint32_t h = threadIdx.x; h < n; h += 64) {
            const RpCand c = cand[t * TT + h];
            if (st.best_key[c.slot] == c.key) st.best_str[c.slot] = c.str;
        }
    }
}

// ---- single-workgroup planning / scan for the common batch sizes (one
// launch instead of the multi-kernel device scan: every launch here costs
// ~4 us, more than the work)
constexpr int SB = 1024;                  // threads of the single-workgroup kernels
constexpr size_t kSmallPlan = 1u << 16;   // replicas / tiles handled by one workgroup

__device__ __forceinline__ uint64_t block_excl_u64(uint64_t v, uint64_t *s_w, uint64_t *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint64_t base = 0, tot = 0;
    for (int k = 0; k < SB / 64; ++k) {
        base += k < w ? s_w[k] : 0;
        tot += s_w[k];
    }
    __syncthreads();                                     // s_w reused by the next call
    *total = tot;
    return base + x - v;
}

// Exclusive scan of n <= kSmallPlan values by one workgroup: each thread
// holds a contiguous chunk in registers (independent loads), one block
// scan, then the chunk's prefixes are written.  out[n] = total.
template <typename Get>
__device__ __forceinline__ void small_scan(Get get, uint32_t n, uint64_t *__restrict__ out, uint64_t *s_w) {
    const uint32_t per = (n + SB - 1) / SB;
    const uint32_t b = threadIdx.x * per < n ? threadIdx.x * per : n;
    const uint32_t e = b + per < n ? b + per : n;
    if (per <= 16) {                                     // n <= 16k: one read, the chunk stays in registers
        uint64_t v[16], sum = 0, tot;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            v[k] = b + k < e ? get(b + k) : 0;
            sum += v[k];
        }
        uint64_t x = block_excl_u64(sum, s_w, &tot);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (b + k < e) out[b + k] = x;
            x += v[k];
        }
        if (threadIdx.x == 0) out[n] = tot;
        return;
    }
    // 8 loads in flight per thread per batch; the second pass re-reads (L2-hot)
    uint64_t sum = 0;
    for (uint32_t c = b; c < e; c += 8) {
        uint64_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = c + k < e ? get(c + k) : 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) sum += v[k];
    }
    uint64_t tot;
    uint64_t x = block_excl_u64(sum, s_w, &tot);
    for (uint32_t c = b; c < e; c += 8) {
        uint64_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = c + k < e ? get(c + k) : 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (c + k < e) out[c + k] = x;
            x += v[k];
        }
    }
    if (threadIdx.x == 0) out[n] = tot;
}

// tbase = exclusive scan of the per-replica tile counts (tbase[np] = tiles)
__global__ __launch_bounds__(SB) void k_rm_plan_small(RmIn in, uint64_t *__restrict__ tbase,
                                                      uint32_t *__restrict__ err) {
    __shared__ uint64_t s_w[SB / 64];
    small_scan([&](uint32_t p) -> uint64_t {
        if (r_hi(in, p) < in.r_off[p]) atomicOr(err, CRDT_DEV_RANGE);
        const uint64_t n = (in.l_off[p + 1] - in.l_off[p]) + r_len(in, p);
        return (n + MT - 1) / MT;
    }, in.replicas, tbase, s_w);
}

// ic = exclusive scan of tcnt[0..n) (ic[n] = total), then
// out.off[p] = l_off[p] + ic[tbase[p]].  More tiles than the n planned (R
// ranges summing past n_r): CRDT_DEV_RANGE, no offsets written.
// KV (tkv non-null): also ikv = exclusive scan of tkv, and the new Diff's
// closing kv offset kv_off[out_off[replicas]] = the kv total.
__global__ __launch_bounds__(SB) void k_rm_scan_small(const uint32_t *__restrict__ tcnt, uint32_t n,
                                                      uint64_t *__restrict__ ic, crdt_refmerge_in in,
                                                      const uint64_t *__restrict__ tbase,
                                                      uint64_t *__restrict__ out_off, const uint64_t *__restrict__ tkv,
                                                      uint64_t *__restrict__ ikv, uint64_t *__restrict__ kv_off,
                                                      uint32_t *__restrict__ err) {
    __shared__ uint64_t s_w[SB / 64];
    if (tbase[in.replicas] > n) {                        // (uniform: every thread reads the same word)
        if (threadIdx.x == 0) atomicOr(err, CRDT_DEV_RANGE);
        return;
    }
    small_scan([&](uint32_t i) -> uint64_t { return tcnt[i]; }, n, ic, s_w);
    if (tkv) small_scan([&](uint32_t i) -> uint64_t { return tkv[i]; }, n, ikv, s_w);
    __syncthreads();                                     // ic / ikv visible to the whole workgroup
    for (uint32_t p = threadIdx.x; p <= in.replicas; p += SB) out_off[p] = in.l_off[p] + ic[tbase[p]];
    if (tkv && threadIdx.x == 0) {                       // (and at the capacity end: a fixed place to read it)
        kv_off[in.l_off[in.replicas] + ic[tbase[in.replicas]]] = ikv[n];
        kv_off[in.n_l + in.n_r] = ikv[n];
    }
}

// Go Atoi over the string arena and the replay accumulators' reset, one launch.
__global__ void k_rm_prep(const uint8_t *__restrict__ bytes, const uint64_t *__restrict__ off, uint64_t nstr,
                          OkVal *__restrict__ okv, SlotAcc acc, uint32_t ns) {
    prep_items(bytes, off, nstr, okv, acc, ns, (uint64_t)blockIdx.x * 256 + threadIdx.x, (uint64_t)gridDim.x * 256);
}

// out.off[p] = l_off[p] + inserted R entries of replicas before p
// (KV: kv_off[out_off[replicas]] = kv total, ikv_total = &ikv[tiles])
__global__ void k_out_off(crdt_refmerge_in in, const uint64_t *__restrict__ tbase, const uint64_t *__restrict__ ic,
                          uint64_t *__restrict__ out_off, const uint64_t *__restrict__ ikv_total,
                          uint64_t *__restrict__ kv_off, uint64_t tmax, uint32_t *__restrict__ err) {
    if (tbase[in.replicas] > tmax) {                     // (see k_rm_scan_small)
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err, CRDT_DEV_RANGE);
        return;
    }
    for (uint32_t p = blockIdx.x * 256 + threadIdx.x; p <= in.replicas; p += gridDim.x * 256) {
        out_off[p] = in.l_off[p] + ic[tbase[p]];
        if (kv_off && p == in.replicas) {
            kv_off[out_off[p]] = *ikv_total;
            kv_off[in.n_l + in.n_r] = *ikv_total;
        }
    }
}

// Per-key closed form (main.go:82-96): verbatim base unless the base parses
// AND another holder's value parses; then Itoa(sum) with int64 wrap.
__global__ void k_slot_final(crdt_refmerge_out out, SlotAcc acc, const OkVal *__restrict__ okv, uint32_t n) {
    for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s < n; s += gridDim.x * 256) {
        const unsigned long long best = acc.best[s];
        if (!best) {                                     // no remote holder: absent from CurrentState
            out.st_kind[s] = 0;
            out.st_str[s] = 0;
            out.st_sum[s] = 0;
            continue;
        }
        const uint32_t str = (uint32_t)best;
        const bool sum_form = okv[str].ok && acc.npar[s] >= 2;
        out.st_kind[s] = sum_form ? 2 : 1;
        out.st_str[s] = str;
        out.st_sum[s] = sum_form ? (int64_t)acc.sum[s] : 0;
    }
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_atoi_batch(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *off, uint64_t n_str,
                               uint8_t *ok, int64_t *val) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (n_str == 0) return CRDT_OK;
    if (!bytes || !off || !ok || !val) return CRDT_E_INVAL;
    k_atoi<<<grid_for(n_str, 256, (unsigned)ctx->num_cus * 8), 256, 0, ctx->stream>>>(bytes, off, n_str, ok, val);
    return check_launch(ctx);
}

static int refmerge_run(crdt_ctx *ctx, const crdt_refmerge_in *inp, const crdt_refmerge_out *outp,
                        const int64_t *maxl_dev, const crdt_refmerge_acc *acc_out, const crdt_replay_state *delta,
                        const crdt_refmerge_kv_out *kv = nullptr, const crdt_refmerge_pull *pull = nullptr,
                        bool one_pair = false);

namespace crdt {
// crdt_refmerge_batch_pull for a caller that knows every entry of L and of
// the pulled ranges has exactly one kv pair (population.hip tracks it): the
// kv count pass takes each tile's pair count from its emitted count instead
// of reading every entry's kv range, and the tile pass runs as one-pair
// tiles only.
int refmerge_batch_pull_one_pair(crdt_ctx *ctx, const crdt_refmerge_in *inp, const crdt_refmerge_out *outp,
                                 const crdt_refmerge_pull *pull, const crdt_refmerge_kv_out *kv) {
    if (!pull || !pull->r_end || !kv) return CRDT_E_INVAL;
    return refmerge_run(ctx, inp, outp, nullptr, nullptr, nullptr, kv, pull, true);
}
}  // namespace crdt

extern "C" int crdt_refmerge_batch(crdt_ctx *ctx, const crdt_refmerge_in *inp, const crdt_refmerge_out *outp) {
    return refmerge_run(ctx, inp, outp, nullptr, nullptr, nullptr);
}

extern "C" int crdt_refmerge_batch_kv(crdt_ctx *ctx, const crdt_refmerge_in *inp, const crdt_refmerge_out *outp,
                                      const crdt_refmerge_kv_out *kv) {
    if (!kv) return CRDT_E_INVAL;
    return refmerge_run(ctx, inp, outp, nullptr, nullptr, nullptr, kv);
}

extern "C" int crdt_refmerge_batch_pull(crdt_ctx *ctx, const crdt_refmerge_in *inp, const crdt_refmerge_out *outp,
                                        const crdt_refmerge_pull *pull, const crdt_refmerge_kv_out *kv) {
    // re-based key slots need the fused kv output: a caller gathering the new
    // Diff's pairs by src afterwards cannot re-base them
    if (!pull || !pull->r_end || (pull->r_slot_delta && !kv)) return CRDT_E_INVAL;
    return refmerge_run(ctx, inp, outp, nullptr, nullptr, nullptr, kv, pull);
}

namespace crdt {
static int rp_delta_fold(crdt_ctx *ctx, const crdt_refmerge_in &in, const uint16_t *r_dk, const OkVal *okv,
                         const crdt_replay_state &st, const crdt_refmerge_out *out, bool phase1_done);
}

extern "C" int crdt_refmerge_batch_ex(crdt_ctx *ctx, const crdt_refmerge_in *inp, const crdt_refmerge_out *outp,
                                      const int64_t *maxl_dev, const crdt_refmerge_acc *acc_out) {
    return refmerge_run(ctx, inp, outp, maxl_dev, acc_out, nullptr);
}

extern "C" int crdt_refmerge_delta(crdt_ctx *ctx, const crdt_refmerge_in *inp, const crdt_refmerge_out *outp,
                                   const crdt_replay_state *st) {
    if (!st) return CRDT_E_INVAL;
    return refmerge_run(ctx, inp, outp, nullptr, nullptr, st);
}

static int refmerge_run(crdt_ctx *ctx, const crdt_refmerge_in *inp, const crdt_refmerge_out *outp,
                        const int64_t *maxl_dev, const crdt_refmerge_acc *acc_out, const crdt_replay_state *delta,
                        const crdt_refmerge_kv_out *kv, const crdt_refmerge_pull *pull, bool one_pair) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!inp || !outp) return CRDT_E_INVAL;
    if (take_fail_refmerge()) return CRDT_E_NOMEM;              // injected failure (diagnostic build)
    if (delta && inp->n_slots && (!delta->best_key || !delta->best_str || !delta->sum || !delta->npar ||
                                  !delta->nhold))
        return CRDT_E_INVAL;
    if (acc_out && inp->n_slots && (!acc_out->best || !acc_out->sum || !acc_out->npar)) return CRDT_E_INVAL;
    RmIn in;
    static_cast<crdt_refmerge_in &>(in) = *inp;
    if (pull) {                                                  // in-place pulls: R ranges by (r_off, r_end)
        if (delta || maxl_dev || acc_out) return CRDT_E_INVAL;
        in.r_end = pull->r_end;
        in.r_sd = pull->r_slot_delta;
    }
    const crdt_refmerge_out out = *outp;
    if (in.replicas == 0) return CRDT_OK;
    if (!in.l_off || !in.r_off || !out.off) return CRDT_E_INVAL;
    if (in.n_l && (!in.l_ts || !in.l_origin)) return CRDT_E_INVAL;
    if (!in.l_kv || !in.r_kv) return CRDT_E_INVAL;
    if (in.n_r && !in.r_ts) return CRDT_E_INVAL;
    if (in.n_kv && (!in.kv_key || !in.kv_val)) return CRDT_E_INVAL;
    if (in.n_l + in.n_r && (!out.ts || !out.origin || !out.src)) return CRDT_E_INVAL;
    if (!acc_out && in.n_slots && (!out.st_kind || !out.st_str || !out.st_sum)) return CRDT_E_INVAL;
    if (in.n_str && (!in.str_bytes || !in.str_off)) return CRDT_E_INVAL;
    if (in.n_kv && !in.n_str) return CRDT_E_INVAL;
    if (kv && (delta || !kv->kv_off || (in.n_kv && (!kv->kv_key || !kv->kv_val)))) return CRDT_E_INVAL;

    const size_t nr = in.n_r, ns = in.n_slots, nstr = in.n_str, np = in.replicas;
    // The replay keys a holder as best = rank << 32 | string id, rank = its
    // 1-based position in the replica's merge sequence (<= |L_p| + |R_p|), and
    // the ts-range-sharded form re-packs it as shard << 40 | rank: every
    // replica's sequence must stay below 2^32 entries and string ids must fit
    // 32 bits.  n_l + n_r bounds every replica's sequence.
    if (in.n_l + nr >= 0xffffffffULL || nstr > 0xffffffffULL) return CRDT_E_RANGE;
    const size_t tmax = (in.n_l + nr) / MT + np + 1;             // >= tiles over all replicas
    if (tmax > 0x7fffffffULL) return CRDT_E_RANGE;
    const size_t need = Carve::round(np * 4 + 4) + Carve::round((np + 1) * 8) + scan_tmp_bytes(std::max(np, tmax)) +
                        Carve::round((tmax + 1) * sizeof(TileDesc)) + Carve::round(tmax * 8 + 8) +
                        Carve::round(tmax * 4 + 4) + Carve::round(tmax * 2 * NW * 8) + Carve::round((nstr + 1) * sizeof(OkVal)) +
                        (delta ? Carve::round(nr * 2 + 2) : 0) +
                        Carve::round(ns * 8 + 8) * 2 + Carve::round(ns * 4 + 4) + 4096 +
                        (delta ? Carve::round(tmax * TT * sizeof(RpCand)) + Carve::round(tmax * 4 + 4) + 256 : 0) +
                        (kv ? 2 * Carve::round((tmax + 1) * 8) + Carve::round((tmax + 1) * 4) : 0);
    rc = ws_reserve(ctx, need);
    if (rc) return rc;
    Carve w(ctx->ws);
    uint32_t *nt = w.take<uint32_t>(np + 1);
    uint64_t *tbase = w.take<uint64_t>(np + 1);
    void *tmp = w.take<char>(scan_tmp_bytes(std::max(np, tmax)));

    TileDesc *desc = w.take<TileDesc>(tmax + 1);
    uint64_t *ic = w.take<uint64_t>(tmax + 1);
    uint32_t *tcnt = w.take<uint32_t>(tmax + 1);
    uint64_t *bits = w.take<uint64_t>(tmax * 2 * NW);             // per tile: merge-order isl / emit bitmaps
    uint16_t *r_dk = delta ? w.take<uint16_t>(nr + 1) : nullptr; // delta: inserted R ranks (holder overflow walk)
    RpCand *cand = delta ? w.take<RpCand>(tmax * TT) : nullptr;   // delta: per-tile max-holder candidates
    uint32_t *cand_n = delta ? w.take<uint32_t>(tmax + 1) : nullptr;
    uint32_t *ovf = delta ? w.take<uint32_t>(4) : nullptr;        // a tile's LDS table overflowed
    OkVal *okv = w.take<OkVal>(nstr + 1);
    uint64_t *tkv = kv ? w.take<uint64_t>(tmax + 1) : nullptr;   // KV: kv pairs per tile, then (ikv) their scan
    uint64_t *ikv = kv ? w.take<uint64_t>(tmax + 1) : nullptr;
    uint32_t *tone = kv ? w.take<uint32_t>(tmax + 1) : nullptr;   // KV: tile whose emitted entries have one pair each
    SlotAcc acc;
    acc.best = w.take<unsigned long long>(ns + 1);
    acc.sum = w.take<unsigned long long>(ns + 1);
    acc.npar = w.take<unsigned>(ns + 1);
    if (acc_out) {                                               // the caller keeps the unreduced accumulators
        acc.best = reinterpret_cast<unsigned long long *>(acc_out->best);
        acc.sum = reinterpret_cast<unsigned long long *>(acc_out->sum);
        acc.npar = acc_out->npar;
    }

    const hipStream_t s = ctx->stream;
    const unsigned cap = (unsigned)ctx->num_cus * 8;
    const uint32_t reps = in.replicas;
    if (np <= kSmallPlan) {
        k_rm_plan_small<<<1, SB, 0, s>>>(in, tbase, ctx->dev_status);
    } else {
        k_rm_ntiles<<<grid_for(np, 256, cap), 256, 0, s>>>(in, nt, ctx->dev_status);
        rc = check_launch(ctx);
        if (rc) return rc;
        rc = exclusive_scan_u32(ctx, nt, tbase, np, tmp);         // tbase[np] = tile count
        if (rc) return rc;
    }
    k_rm_split<<<(unsigned)((tmax + 4) / 4), 256, 0, s>>>(in, reps, tbase, maxl_dev, tmax, desc, okv, acc,
                                                           (uint32_t)ns, ctx->dev_status);
    // tile grids = the tile-count upper bound; empty descriptors exit at once
    // (count-pass shapes at 4096-item tiles: 256 x 16 51 us, 512 x 8 45 us, 1024 x 4 67 us)
    // LDS-DMA staging of the ts runs when both logs are 8-byte aligned (refmerge.count_dma)
    const int cdma = g_rm_count_dma && !((((uintptr_t)in.l_ts) | ((uintptr_t)in.r_ts)) & 7);
    if (kv) k_rm_count<MB, true><<<(unsigned)tmax, MB, 0, s>>>(in, desc, tcnt, bits, ovf, cdma, tkv, tone, ctx->dev_status,
                                                             one_pair ? 1 : 0);
    else k_rm_count<MB><<<(unsigned)tmax, MB, 0, s>>>(in, desc, tcnt, bits, ovf, cdma, nullptr, nullptr, nullptr);
    rc = check_launch(ctx);
    if (rc) return rc;
    // (a completion ticket letting the count pass's last block do this scan
    // measured 95 us against 56 + 11.5: same-address arrivals serialise at
    // ~11 ns each and the tail runs alone after the grid)
    if (tmax <= kSmallPlan) {
        k_rm_scan_small<<<1, SB, 0, s>>>(tcnt, (uint32_t)tmax, ic, in, tbase, out.off, tkv, ikv,
                                         kv ? kv->kv_off : nullptr, ctx->dev_status);
    } else {
        rc = exclusive_scan_u32(ctx, tcnt, ic, tmax, tmp);
        if (rc) return rc;
        if (kv) {                                                 // (in place: one workgroup, any tile count)
            hipError_t e = hipMemcpyAsync(ikv, tkv, tmax * 8, hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) return hip_fail(ctx, e);
            k_scan_tsums<<<1, 256, 0, s>>>(ikv, tmax, 0, ikv + tmax);
        }
        k_out_off<<<grid_for(np + 1, 256, cap), 256, 0, s>>>(in, tbase, ic, out.off, kv ? ikv + tmax : nullptr,
                                                              kv ? kv->kv_off : nullptr, tmax, ctx->dev_status);
    }
    if (take_fail_zero_bits()) {                                  // failpoint: the tile pass must flag, not fault
        hipError_t e = hipMemsetAsync(bits, 0, tmax * 2 * NW * 8, s);
        if (e != hipSuccess) return hip_fail(ctx, e);
    }
    // the tile pass: slice write and (with slots) the replay fold
    const unsigned tg = (unsigned)tmax;
    // (one_pair: the caller's population keeps one pair per entry in entry
    // order -- refmerge_batch_pull_one_pair; the tile pass then computes
    // each entry's pair index instead of loading its kv range)
    const KvOut kvo = kv ? KvOut{kv->kv_off, kv->kv_key, kv->kv_val, kv->kv_cap, ikv, tone,
                                 one_pair && g_rm_affine ? 1u : 0u}
                         : KvOut{};
    if (delta && ns) {                                            // incremental replay: fold only the inserted R
        k_rm_tile<RM_FOLD_DELTA><<<tg, FB, 0, s>>>(in, desc, bits, r_dk, okv, acc, 0, ic, out, *delta, cand, cand_n,
                                                   ovf, ctx->dev_status);
        rc = check_launch(ctx);
        if (rc) return rc;
        k_rp_holder<<<tg, 64, 0, s>>>(in, r_dk, *delta, cand, cand_n, ovf, tmax);   // the candidates' holders
        rc = check_launch(ctx);
        if (rc) return rc;
        return rp_delta_fold(ctx, in, r_dk, okv, *delta, &out, true);
    }
    // one workgroup per tile (1/P of a tile per workgroup measured slower: DESIGN.md §5.4)
#define RM_TILE(F, P, KV, DIAG)                                                                                \
    if (KV && one_pair) {                                   /* every tile a one-pair tile */                   \
        if (ctx->rm_nt) k_rm_tile_kv1<F, true><<<tg, FB, 0, s>>>(in, desc, bits, okv, acc, DIAG, ic, out, ctx->dev_status, kvo); \
        else k_rm_tile_kv1<F, false><<<tg, FB, 0, s>>>(in, desc, bits, okv, acc, DIAG, ic, out, ctx->dev_status, kvo); \
    } else if (KV && tg <= (unsigned)ctx->num_cus) {                                                           \
        if (ctx->rm_nt) k_rm_tile_kvx<F, true><<<tg, FB, 0, s>>>(in, desc, bits, okv, acc, DIAG, ic, out, ctx->dev_status, kvo); \
        else k_rm_tile_kvx<F, false><<<tg, FB, 0, s>>>(in, desc, bits, okv, acc, DIAG, ic, out, ctx->dev_status, kvo); \
    } else if (KV) {                                                                                           \
        if (ctx->rm_nt) {                                                                                      \
            k_rm_tile_kv1<F, true><<<tg, FB, 0, s>>>(in, desc, bits, okv, acc, DIAG, ic, out, ctx->dev_status, kvo); \
            k_rm_tile_kv<F, true><<<tg, FB, 0, s>>>(in, desc, bits, okv, acc, DIAG, ic, out, ctx->dev_status, kvo); \
        } else {                                                                                               \
            k_rm_tile_kv1<F, false><<<tg, FB, 0, s>>>(in, desc, bits, okv, acc, DIAG, ic, out, ctx->dev_status, kvo); \
            k_rm_tile_kv<F, false><<<tg, FB, 0, s>>>(in, desc, bits, okv, acc, DIAG, ic, out, ctx->dev_status, kvo); \
        }                                                                                                      \
    } else                                                                                                       \
        k_rm_tile<F, P><<<tg * P, FB / P, 0, s>>>(in, desc, bits, nullptr, okv, acc, DIAG, ic, out,            \
                                                  crdt_replay_state{}, nullptr, nullptr, nullptr, ctx->dev_status)
    if (!ns || g_rm_diag == 1) {                                  // (diag 1: timing without the replay fold)
        if (kv) RM_TILE(RM_FOLD_NONE, 1, true, 0);
        else RM_TILE(RM_FOLD_NONE, 1, false, 0);
        if (!ns || delta) return check_launch(ctx);
    } else {
        if (kv) RM_TILE(RM_FOLD_FULL, 1, true, g_rm_diag);
        else RM_TILE(RM_FOLD_FULL, 1, false, g_rm_diag);
    }
#undef RM_TILE
    if (ns && !acc_out) k_slot_final<<<grid_for(ns, 256, cap), 256, 0, s>>>(out, acc, okv, (uint32_t)ns);
    return check_launch(ctx);
}

// ---------------------------------------------------------------- ts-range-sharded merge (§8(e))
namespace crdt {
__global__ void k_rm_local_maxl(crdt_refmerge_in in, int64_t *__restrict__ out) {
    for (uint32_t p = blockIdx.x * 256 + threadIdx.x; p < in.replicas; p += gridDim.x * 256) {
        const uint64_t b = in.l_off[p], e = in.l_off[p + 1];
        out[p] = e > b ? in.l_ts[e - 1] : INT64_MIN;
    }
}

// mode 0: c = best ? shard << 40 | (best >> 32) : 0   (cross-shard rank of the max-ts holder)
// mode 1: v = (c != 0 && c == cmax) ? (uint32)best : 0  (only the owning shard contributes)
// mode 2: best = cmax ? 1 << 32 | (uint32)v : 0          (the reduced accumulator)
__global__ void k_rm_acc_xform(crdt_refmerge_acc acc, uint32_t n, int mode, uint32_t shard, int64_t *__restrict__ c,
                               const int64_t *__restrict__ cmax, int64_t *__restrict__ v) {
    for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s < n; s += gridDim.x * 256) {
        const uint64_t best = acc.best[s];
        if (mode == 0) c[s] = best ? (int64_t)(((uint64_t)shard << 40) | (best >> 32)) : 0;
        else if (mode == 1) v[s] = (c[s] != 0 && c[s] == cmax[s]) ? (int64_t)(uint32_t)best : 0;
        else acc.best[s] = cmax[s] ? ((1ull << 32) | (uint32_t)v[s]) : 0;
    }
}
}  // namespace crdt

extern "C" int crdt_refmerge_local_maxl(crdt_ctx *ctx, const crdt_refmerge_in *in, int64_t *maxl_dev) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!in || !maxl_dev) return CRDT_E_INVAL;
    if (in->replicas == 0) return CRDT_OK;
    if (!in->l_off || (in->n_l && !in->l_ts)) return CRDT_E_INVAL;
    k_rm_local_maxl<<<grid_for(in->replicas, 256, (unsigned)ctx->num_cus * 4), 256, 0, ctx->stream>>>(*in, maxl_dev);
    return check_launch(ctx);
}

static int acc_xform(crdt_ctx *ctx, const crdt_refmerge_acc *acc, size_t n, int mode, uint32_t shard, int64_t *c,
                     const int64_t *cmax, int64_t *v) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (n == 0) return CRDT_OK;
    if (!acc || !acc->best || n > 0xffffffffULL) return CRDT_E_INVAL;
    k_rm_acc_xform<<<grid_for(n, 256, (unsigned)ctx->num_cus * 4), 256, 0, ctx->stream>>>(*acc, (uint32_t)n, mode,
                                                                                        shard, c, cmax, v);
    return check_launch(ctx);
}

extern "C" int crdt_refmerge_acc_rank(crdt_ctx *ctx, const crdt_refmerge_acc *acc, size_t n_slots, uint32_t shard,
                                      int64_t *c_dev) {
    if (!c_dev) return CRDT_E_INVAL;
    if (shard >= (1u << 23)) return CRDT_E_RANGE;      // shard << 40 | rank must stay a positive int64
    return acc_xform(ctx, acc, n_slots, 0, shard, c_dev, nullptr, nullptr);
}

extern "C" int crdt_refmerge_acc_owner_str(crdt_ctx *ctx, const crdt_refmerge_acc *acc, size_t n_slots,
                                           const int64_t *c_dev, const int64_t *cmax_dev, int64_t *v_dev) {
    if (!c_dev || !cmax_dev || !v_dev) return CRDT_E_INVAL;
    return acc_xform(ctx, acc, n_slots, 1, 0, const_cast<int64_t *>(c_dev), cmax_dev, v_dev);
}

extern "C" int crdt_refmerge_acc_set_best(crdt_ctx *ctx, const crdt_refmerge_acc *acc, size_t n_slots,
                                          const int64_t *cmax_dev, const int64_t *v_dev) {
    if (!cmax_dev || !v_dev) return CRDT_E_INVAL;
    return acc_xform(ctx, acc, n_slots, 2, 0, nullptr, cmax_dev, const_cast<int64_t *>(v_dev));
}

extern "C" int crdt_refmerge_finalize(crdt_ctx *ctx, const crdt_refmerge_acc *accp, size_t n_slots,
                                      const uint8_t *str_bytes, const uint64_t *str_off, uint64_t n_str,
                                      const crdt_refmerge_out *outp) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (n_slots == 0) return CRDT_OK;
    if (!accp || !outp || !accp->best || !accp->sum || !accp->npar || n_slots > 0xffffffffULL) return CRDT_E_INVAL;
    if (!outp->st_kind || !outp->st_str || !outp->st_sum) return CRDT_E_INVAL;
    if (n_str && (!str_bytes || !str_off)) return CRDT_E_INVAL;
    rc = ws_reserve(ctx, Carve::round((n_str + 1) * sizeof(OkVal)) + 4096);
    if (rc) return rc;
    Carve w(ctx->ws);
    OkVal *okv = w.take<OkVal>(n_str + 1);
    const unsigned cap = (unsigned)ctx->num_cus * 8;
    if (n_str) k_rm_prep<<<grid_for(n_str, 256, cap), 256, 0, ctx->stream>>>(str_bytes, str_off, n_str, okv, SlotAcc{}, 0);
    SlotAcc acc;
    acc.best = reinterpret_cast<unsigned long long *>(accp->best);
    acc.sum = reinterpret_cast<unsigned long long *>(accp->sum);
    acc.npar = accp->npar;
    // a best string id >= n_str cannot occur (pairs with v >= n_str are never folded)
    k_slot_final<<<grid_for(n_slots, 256, cap), 256, 0, ctx->stream>>>(*outp, acc, okv, (uint32_t)n_slots);
    return check_launch(ctx);
}

// ---------------------------------------------------------------- incremental replay (§8(f) row 3)
// The reference re-folds the whole Diff on every merge (main.go:76).  A
// merge only ever ADDS remote entries to Diff (inserted R; an equal ts keeps
// the local entry), so the replay over Diff' = the replay over Diff plus the
// inserted entries -- provided the per-key state is keyed by ts, not by a
// merge-order rank: best_key = max over holders of ts ^ 2^63 (order-
// preserving), best_str = the string of that holder (ts are unique within a
// Diff, so exactly one holder matches), the wrapped sum and the parsable and
// holder counts.  Two passes per fold: max/sum/counts through a per-block
// LDS table flushed with global atomics, then the unique max holder writes
// its string.  (A local write that overwrites a remote entry at the same ms,
// main.go:187, removes a holder: the caller rebuilds the state then.)
namespace crdt {
constexpr int RPB = 256;                  // threads per block
constexpr int RPE = 4;                    // entries per thread per round

__device__ __forceinline__ uint64_t ord_ts(int64_t ts) { return (uint64_t)ts ^ 0x8000000000000000ull; }

// PHASE 1: max / sum / counts; PHASE 2: the max holder writes its string.
// RSIDE: the R entries marked inserted in r_dk (delta); else the L entries
// of remote origin (state init).
template <bool RSIDE, int PHASE>
__global__ __launch_bounds__(RPB) void k_rp_fold(crdt_refmerge_in in, const uint16_t *__restrict__ r_dk,
                                                 const OkVal *__restrict__ okv, crdt_replay_state st) {
    __shared__ uint32_t t_slot[TT];
    __shared__ unsigned long long t_max[TT];
    __shared__ unsigned long long t_sum[TT];
    __shared__ uint32_t t_npar[TT], t_nh[TT];
    __shared__ int64_t s_okval[OKC];
    __shared__ uint8_t s_okok[OKC];
    const uint64_t n = RSIDE ? in.n_r : in.n_l;
    const uint64_t *kvo = RSIDE ? in.r_kv : in.l_kv;
    const int64_t *tsv = RSIDE ? in.r_ts : in.l_ts;
    const bool okc = PHASE == 1 && in.n_str <= OKC;      // small string table: Atoi records in LDS
    if (okc)
        for (uint32_t i = threadIdx.x; i < in.n_str; i += RPB) {
            const OkVal o = okv[i];
            s_okval[i] = o.val;
            s_okok[i] = (uint8_t)(o.ok != 0);
        }
    // (the first round's table-init barrier publishes the staged records)
    for (uint64_t base = (uint64_t)blockIdx.x * RPB * RPE; base < n; base += (uint64_t)gridDim.x * RPB * RPE) {
        if (PHASE == 1) {
            for (int h = threadIdx.x; h < TT; h += RPB) {
                t_slot[h] = kEmpty;
                t_max[h] = 0;
                t_sum[h] = 0;
                t_npar[h] = 0;
                t_nh[h] = 0;
            }
            __syncthreads();
        }
        // every load of the round issued before the first atomic
        uint64_t e_kb[RPE], e_key[RPE];
        uint32_t e_cnt[RPE], e_slot[RPE], e_v[RPE];
#pragma unroll
        for (int f = 0; f < RPE; ++f) {
            const uint64_t e = base + threadIdx.x + (uint64_t)f * RPB;
            e_cnt[f] = 0;
            e_kb[f] = 0;
            e_key[f] = 0;
            if (e < n) {
                const bool take = RSIDE ? r_dk[e] != 0 : in.l_origin[e] == 0;   // *Command skipped (main.go:80)
                const uint64_t kb = kvo[e], ke = kvo[e + 1] < in.n_kv ? kvo[e + 1] : in.n_kv;
                e_kb[f] = kb;
                e_key[f] = ord_ts(tsv[e]);
                e_cnt[f] = take && kb < ke ? (uint32_t)(ke - kb < 0xFFFFFFFFull ? ke - kb : 0xFFFFFFFFull) : 0;
            }
        }
#pragma unroll
        for (int f = 0; f < RPE; ++f) {
            e_slot[f] = e_cnt[f] ? in.kv_key[e_kb[f]] : 0xFFFFFFFFu;
            e_v[f] = e_cnt[f] ? in.kv_val[e_kb[f]] : 0xFFFFFFFFu;
        }
        OkVal e_o[RPE];
#pragma unroll
        for (int f = 0; f < RPE; ++f) {
            e_o[f] = OkVal{0, 0};
            if (PHASE == 1 && e_slot[f] < in.n_slots && e_v[f] < in.n_str)
                e_o[f] = okc ? OkVal{s_okval[e_v[f]], s_okok[e_v[f]]} : okv[e_v[f]];
        }
#pragma unroll
        for (int f = 0; f < RPE; ++f) {
            for (uint32_t j = 0; j < e_cnt[f]; ++j) {
                uint32_t slot = e_slot[f], v = e_v[f];
                OkVal o = e_o[f];
                if (j) {                                     // further kvs of the entry (rare)
                    slot = in.kv_key[e_kb[f] + j];
                    v = in.kv_val[e_kb[f] + j];
                    if (PHASE == 1 && slot < in.n_slots && v < in.n_str) o = okv[v];
                }
                if (slot >= in.n_slots || v >= in.n_str) continue;
                const uint64_t key = e_key[f];
                if (PHASE == 2) {
                    if (st.best_key[slot] == key) st.best_str[slot] = v;   // the unique max holder
                    continue;
                }
                const uint32_t idx = table_find(t_slot, slot);
                if (idx != kEmpty) {
                    atomicMax(&t_max[idx], key);
                    atomicAdd(&t_nh[idx], 1u);
                    if (o.ok) {
                        atomicAdd(&t_sum[idx], (unsigned long long)o.val);   // mod 2^64 (main.go:95)
                        atomicAdd(&t_npar[idx], 1u);
                    }
                } else {
                    atomicMax(reinterpret_cast<unsigned long long *>(&st.best_key[slot]), key);
                    atomicAdd(&st.nhold[slot], 1u);
                    if (o.ok) {
                        atomicAdd(reinterpret_cast<unsigned long long *>(&st.sum[slot]), (unsigned long long)o.val);
                        atomicAdd(&st.npar[slot], 1u);
                    }
                }
            }
        }
        if (PHASE == 1) {
            __syncthreads();
            for (int h = threadIdx.x; h < TT; h += RPB) {
                const uint32_t slot = t_slot[h];
                if (slot == kEmpty) continue;
                atomicMax(reinterpret_cast<unsigned long long *>(&st.best_key[slot]), t_max[h]);
                atomicAdd(&st.nhold[slot], t_nh[h]);
                if (t_npar[h]) {
                    atomicAdd(reinterpret_cast<unsigned long long *>(&st.sum[slot]), t_sum[h]);
                    atomicAdd(&st.npar[slot], t_npar[h]);
                }
            }
            __syncthreads();                                 // table reused by the next round
        }
    }
}

__global__ void k_rp_clear(crdt_replay_state st, uint32_t n) {
    for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s < n; s += gridDim.x * 256) {
        st.best_key[s] = 0;
        st.best_str[s] = 0;
        st.sum[s] = 0;
        st.npar[s] = 0;
        st.nhold[s] = 0;
    }
}

// CurrentState from the state (closed form as k_slot_final)
__global__ void k_rp_final(crdt_refmerge_out out, crdt_replay_state st, const OkVal *__restrict__ okv, uint32_t n) {
    for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s < n; s += gridDim.x * 256) {
        if (!st.nhold[s]) {
            out.st_kind[s] = 0;
            out.st_str[s] = 0;
            out.st_sum[s] = 0;
            continue;
        }
        const uint32_t str = st.best_str[s];
        const bool sum_form = okv[str].ok && st.npar[s] >= 2;
        out.st_kind[s] = sum_form ? 2 : 1;
        out.st_str[s] = str;
        out.st_sum[s] = sum_form ? st.sum[s] : 0;
    }
}

static int rp_delta_fold(crdt_ctx *ctx, const crdt_refmerge_in &in, const uint16_t *r_dk, const OkVal *okv,
                         const crdt_replay_state &st, const crdt_refmerge_out *out, bool phase1_done) {
    const hipStream_t s = ctx->stream;
    const unsigned g = grid_for((in.n_r + RPE - 1) / RPE, RPB, (unsigned)ctx->num_cus * 8);
    if (in.n_r) {
        if (!phase1_done) {
            k_rp_fold<true, 1><<<g, RPB, 0, s>>>(in, r_dk, okv, st);
            k_rp_fold<true, 2><<<g, RPB, 0, s>>>(in, r_dk, okv, st);
        }
    }
    k_rp_final<<<grid_for(in.n_slots, 256, (unsigned)ctx->num_cus * 8), 256, 0, s>>>(*out, st, okv, in.n_slots);
    return check_launch(ctx);
}
}  // namespace crdt

// Replay state of the L logs alone (their remote-origin entries): the
// starting point of crdt_refmerge_delta.  R is ignored.
extern "C" int crdt_replay_state_init(crdt_ctx *ctx, const crdt_refmerge_in *inp, const crdt_replay_state *st) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!inp || !st) return CRDT_E_INVAL;
    const crdt_refmerge_in in = *inp;
    if (in.n_slots == 0) return CRDT_OK;
    if (!st->best_key || !st->best_str || !st->sum || !st->npar || !st->nhold) return CRDT_E_INVAL;
    if (in.n_l && (!in.l_ts || !in.l_origin || !in.l_kv)) return CRDT_E_INVAL;
    if (in.n_kv && (!in.kv_key || !in.kv_val || !in.n_str)) return CRDT_E_INVAL;
    if (in.n_str && (!in.str_bytes || !in.str_off)) return CRDT_E_INVAL;
    rc = ws_reserve(ctx, Carve::round((in.n_str + 1) * sizeof(OkVal)) + 4096);
    if (rc) return rc;
    Carve w(ctx->ws);
    OkVal *okv = w.take<OkVal>(in.n_str + 1);
    const hipStream_t s = ctx->stream;
    const unsigned cap = (unsigned)ctx->num_cus * 8;
    if (in.n_str)
        k_rm_prep<<<grid_for(in.n_str, 256, cap), 256, 0, s>>>(in.str_bytes, in.str_off, in.n_str, okv, SlotAcc{}, 0);
    k_rp_clear<<<grid_for(in.n_slots, 256, cap), 256, 0, s>>>(*st, in.n_slots);
    if (in.n_l) {
        const unsigned g = grid_for((in.n_l + RPE - 1) / RPE, RPB, cap);
        k_rp_fold<false, 1><<<g, RPB, 0, s>>>(in, nullptr, okv, *st);
        k_rp_fold<false, 2><<<g, RPB, 0, s>>>(in, nullptr, okv, *st);
    }
    return check_launch(ctx);
}

