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
// GPU structure: two passes over merge-order bitmaps, no cross-workgroup
// waiting:
//   split  : merge-path splits of every tile (16-ary searches, four tile
//            diagonals per wave);
//   count  : per tile the merge in LDS -> two bitmaps in merge order (`isa`:
//            the item is an A element; `emit`: the item is an output) and the
//            tile's output count;
//   scan   : one workgroup turns the counts into output offsets;
//   write  : per part of a tile, the runs staged in LDS by LDS-DMA, every
//            index a prefix popcount of the bitmaps, outputs stored at their
//            rank.
// The tiles run in chunks of at most 16384 (one scan workgroup each): chunk
// c's count, scan and write pass in turn on the context's stream.  (Smaller
// chunks, so that the keys the count pass read were still in the Infinity
// Cache for the write pass, and a second stream running chunk c+1's count
// beside chunk c's write, measured slower: DESIGN.md §5.4.1.  So did one
// pass with a decoupled look-back, §5.4.4.)
#include <algorithm>
#include <atomic>

#include "scan.hpp"

namespace crdt {

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
// Field-wise select (a ternary on Tag objects lowers to a scratch alloca).
__device__ __forceinline__ Tag tag_sel(bool c, const Tag &x, const Tag &y) {
    return Tag{c ? x.k : y.k, c ? x.t : y.t, c ? x.r : y.r};
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

// A write pass derives every staged run and index from its tile's bitmaps
// (lane w < nw holds word w of each): they must set no bit at or past the
// tile's n items and hold exactly na A items.  Wave-uniform.
__device__ __forceinline__ bool bitmaps_consistent(uint64_t word_a, uint64_t word_e, uint32_t pre_a, int nw,
                                                   uint32_t na, uint32_t n, int lane) {
    const uint32_t lo = 64u * (uint32_t)lane;
    const uint64_t valid = lane >= nw || lo >= n ? 0ull : (n - lo >= 64u ? ~0ull : (1ull << (n - lo)) - 1);
    const bool bad = ((word_a | word_e) & ~valid) != 0;
    // (readlane: scalar, no LDS round trip in front of the staging loads)
    const uint32_t tot_a = (uint32_t)__builtin_amdgcn_readlane((int)(pre_a + (uint32_t)__popcll(word_a)), 63);
    return __ballot(bad) == 0 && tot_a == na;
}

// ---------------------------------------------------------------- LWW by key runs
// LWW needs no tag-ordered merge: its output is one tuple per distinct key,
// in key order, and a key's winner depends only on the END of the key's run
// on each side -- A's run ends at its max (ts, rep) tag, B's likewise; the
// larger tag wins, A on an equal tag (left / local wins, main.go:54-65), and
// the winner's tomb is that of the FIRST copy of its tag on its side (the
// first element in the stable merged order carrying the key's max tag).  So
// the merge runs over KEYS only (A first on an equal key), and only the run
// ends' ts / rep / tomb are ever read:
//   k_lww_split : merge-path splits of 4096-item tiles over the keys;
//   k_lww_count : per tile, the keys staged in LDS by LDS-DMA and merged
//                 (512 threads x 8 items): bitmap `isa` (merge item is an A
//                 element) and `emit` (its key differs from the next merged
//                 key: the last element of the key's merged run -- B's run
//                 end when B holds the key, else A's), 512 B per tile, and
//                 the tile's emit count;
//   k_chunk_scan: the counts of a chunk of tiles -> output offsets;
//   k_lww_write : per quarter tile the runs staged in LDS; an emitting
//                 item's A / B index and output rank are prefix popcounts
//                 of the bitmaps; a B run end looks at A's element just
//                 before it in merged order, picks the winner, steps back
//                 over equal-tag copies for the first one's tomb, and stores
//                 at its rank (consecutive across the emitting lanes).
constexpr int LT = 4096;                 // merge items per LWW tile
constexpr int LCB = 512;                 // count pass threads (8 items each)
constexpr int LNW = LT / 64;             // bitmap words per tile and bitmap
constexpr uint32_t kScanMax = 16384;     // tiles per chunk (one scan workgroup)

template <int TT = LT>
__global__ __launch_bounds__(256) void k_lww_split(const uint64_t *__restrict__ ka, const uint64_t *__restrict__ kb,
                                                   size_t na, size_t nb, size_t ntiles, uint64_t *__restrict__ split) {
    const int lane = threadIdx.x & 63, grp = lane >> 4, gl = lane & 15;
    const size_t t = ((((size_t)blockIdx.x * 256 + threadIdx.x) >> 6) << 2) + (size_t)grp;
    const size_t n = na + nb;
    const size_t d = t * TT < n ? t * TT : n;
    size_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
    bool done = t > ntiles || hi <= lo;
    // P(i) = A.key[i] <= B.key[d-1-i]: true below the split, false from it
    while (__ballot(!done)) {
        const size_t span = hi - lo;
        const bool small = span <= 16;
        const size_t c = small ? lo + (size_t)gl : lo + ((size_t)gl * span) / 16;
        const bool valid = !done && (small ? (size_t)gl < span : true);
        const bool p = valid && ka[c] <= kb[d - 1 - c];
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

struct LwwTile {
    size_t i0, i1, j0, j1;
    uint32_t na, nb, n;
};
template <int TT = LT>
__device__ __forceinline__ LwwTile lww_tile(const uint64_t *__restrict__ split, uint64_t t, size_t n) {
    LwwTile b;
    const size_t d0 = (size_t)t * TT, d1 = d0 + TT < n ? d0 + TT : n;
    b.i0 = split[t];
    b.i1 = split[t + 1];
    b.j0 = d0 - b.i0;
    b.j1 = d1 - b.i1;
    b.na = (uint32_t)(b.i1 - b.i0);
    b.nb = (uint32_t)(b.j1 - b.j0);
    b.n = b.na + b.nb;
    return b;
}

__global__ __launch_bounds__(LCB) void k_lww_count(const uint64_t *__restrict__ ka, const uint64_t *__restrict__ kb,
                                                   size_t na, size_t nb, const uint64_t *__restrict__ split,
                                                   uint32_t *__restrict__ tcnt, uint64_t *__restrict__ bits,
                                                   uint64_t t0) {
    constexpr int NI = LT / LCB, LPW = 64 / NI;
    __shared__ alignas(16) uint64_t sk[LT + 8];          // A's run, then B's, each from its 16-byte aligned-down start
    __shared__ uint32_t s_w[LCB / 64];
    const uint64_t t = t0 + blockIdx.x;
    const LwwTile b = lww_tile(split, t, na + nb);
    const int lane0 = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t at = 0;
    const int oa = dma_run<uint64_t, LCB / 64>(ka, b.i0, b.na, sk, &at, wv, lane0);
    const int ob = dma_run<uint64_t, LCB / 64>(kb, b.j0, b.nb, sk, &at, wv, lane0);
    // the keys after the tile: the next merged key past its last item
    const bool ha_next = b.i1 < na, hb_next = b.j1 < nb;
    const uint64_t ka_next = ha_next ? ka[b.i1] : 0, kb_next = hb_next ? kb[b.j1] : 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA has landed in LDS
    __syncthreads();
    const uint64_t *SA = sk + oa, *SB = sk + ob;
    const uint32_t k0 = threadIdx.x * NI < b.n ? threadIdx.x * NI : b.n;
    const uint32_t k1 = k0 + NI < b.n ? k0 + NI : b.n;
    uint32_t isa = 0, emit = 0;
    if (k0 < k1) {
        uint32_t lo = k0 > b.nb ? k0 - b.nb : 0, hi = k0 < b.na ? k0 : b.na;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (SA[mid] <= SB[k0 - 1 - mid]) lo = mid + 1;
            else hi = mid;
        }
        uint32_t ia = lo, ib = k0 - lo;
        uint64_t ha = ia < b.na ? SA[ia] : 0, hb = ib < b.nb ? SB[ib] : 0;
        uint64_t prev = 0;
        for (uint32_t i = 0; i < k1 - k0; ++i) {
            const bool take_a = ia < b.na && (ib >= b.nb || ha <= hb);
            const uint64_t key = take_a ? ha : hb;
            if (i > 0 && key != prev) emit |= 1u << (i - 1);
            prev = key;
            if (take_a) {
                isa |= 1u << i;
                ++ia;
                if (ia < b.na) ha = SA[ia];
            } else {
                ++ib;
                if (ib < b.nb) hb = SB[ib];
            }
        }
        // the item after the thread's last one: the merge's next head, or
        // past the tile the first of A[i1] / B[j1] (A first on an equal key)
        bool has_next;
        uint64_t nk;
        if (ia < b.na || ib < b.nb) {
            has_next = true;
            nk = (ia < b.na && (ib >= b.nb || ha <= hb)) ? ha : hb;
        } else {
            has_next = ha_next || hb_next;
            nk = (ha_next && (!hb_next || ka_next <= kb_next)) ? ka_next : kb_next;
        }
        if (!has_next || nk != prev) emit |= 1u << (k1 - k0 - 1);
    }
    const int lane = threadIdx.x & 63, sh = (lane % LPW) * NI;
    uint64_t wl = (uint64_t)isa << sh, we = (uint64_t)emit << sh;
#pragma unroll
    for (int o = 1; o < LPW; o <<= 1) {
        wl |= (uint64_t)__shfl_xor((unsigned long long)wl, o);
        we |= (uint64_t)__shfl_xor((unsigned long long)we, o);
    }
    if (lane % LPW == 0) {
        const uint32_t w = threadIdx.x / LPW;
        bits[t * 2 * LNW + w] = wl;
        bits[t * 2 * LNW + LNW + w] = we;
    }
    uint32_t x = (uint32_t)__popc(emit);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) s_w[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
#pragma unroll
        for (int k = 0; k < LCB / 64; ++k) tot += s_w[k];
        tcnt[t] = tot;
    }
}

// Exclusive scan of the n <= kScanMax tile counts of one chunk (tiles t0 ..
// t0 + n) by one workgroup, on top of the offset the previous chunk's scan
// left at ic[t0] (0 for t0 == 0); ic[t0 + n] = the running total, also
// written to *count when count != nullptr.  Over 8k counts, striped rows
// (scan.hpp wg_scan_rows, every access coalesced): 11.7 -> 8.4 us at 9.8k
// tiles; up to 8k a contiguous run per thread in registers is quicker (4.7
// us at 4.9k; striped ~7-10 us at that size).  (16 coalesced rows per wave
// with a serial carry: 11.9 / 12.0 us.)
__global__ __launch_bounds__(1024) void k_chunk_scan(const uint32_t *__restrict__ tcnt, uint64_t t0, uint32_t n,
                                                     uint64_t *__restrict__ ic, uint64_t *__restrict__ count) {
    __shared__ uint64_t s_pre[16 * 16 + 1];
    __shared__ uint64_t s_w[16];
    static_assert(kScanMax <= 16 * 1024, "striped rows: 16 per thread");
    const uint64_t base = t0 ? ic[t0] : 0;               // (read before any thread rewrites ic[t0]: the
    const uint32_t *tc = tcnt + t0;                      //  scan's first barrier lies between)
    uint64_t *o = ic + t0;
    uint64_t tot = 0;
    if (n > 8u * 1024) {                                 // (uniform) striped rows
        tot = wg_scan_rows<1024, 16, uint32_t>([&](uint32_t i) { return tc[i]; }, n,
                                               [&](uint32_t i, uint64_t x) { o[i] = base + x; }, s_pre);
    } else {                                             // <= 8 counts per thread: a contiguous run each
        const uint32_t per = (n + 1023) / 1024;
        const uint32_t b = threadIdx.x * per < n ? threadIdx.x * per : n;
        const uint32_t e = b + per < n ? b + per : n;
        uint32_t v[8];
        uint64_t sum = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            v[k] = b + k < e ? tc[b + k] : 0u;
            sum += v[k];
        }
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        uint64_t x = sum;
#pragma unroll
        for (int o2 = 1; o2 < 64; o2 <<= 1) {
            const uint64_t y = __shfl_up(x, o2);
            if (lane >= o2) x += y;
        }
        if (lane == 63) s_w[w] = x;
        __syncthreads();
        uint64_t run = base + x - sum;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            run += k < w ? s_w[k] : 0;
            tot += s_w[k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (b + k < e) o[b + k] = run;
            run += v[k];
        }
    }
    if (threadIdx.x == 0) {
        o[n] = base + tot;
        if (count) *count = base + tot;
    }
}

// the first element of a side's run of equal tags ending at index w
__device__ __forceinline__ size_t first_copy(const uint64_t *sk, const uint64_t *st, const uint32_t *sr, size_t w,
                                             uint64_t k, uint64_t ts, uint32_t r) {
    while (w > 0 && sk[w - 1] == k && st[w - 1] == ts && sr[w - 1] == r) --w;
    return w;
}

// k_lww_write: one workgroup per part of a tile (1/P of its 4096 merge
// items, sets.lww_parts).  The part's A run and B run (plus the two A
// elements and the one B element before them) are staged in LDS by LDS-DMA
// -- every field of every input element is read once, in order; per-lane
// gathers of the run ends kept the vector-memory address pipe saturated
// (185 us, 52 % of wave time in issue stalls; a shuffle-window variant
// 216-224 us).  Then, per emitting item, X / Y / their predecessors come
// from LDS.
constexpr int LWH = 2048;                // merge items per write workgroup (template default)
constexpr int LWT = 512;                 // its threads (4 items each)

// WH merge items per workgroup (a 1/P of a tile, P = LT / WH), WT threads
template <int WH = LWH, int WT = LWT>
__global__ __launch_bounds__(WT) void k_lww_write(crdt_tuples A, crdt_tuples B, size_t na, size_t nb,
                                                  const uint64_t *__restrict__ split,
                                                  const uint64_t *__restrict__ bits, const uint64_t *__restrict__ ic,
                                                  crdt_tuples out, uint64_t t0, uint32_t *__restrict__ err) {
    constexpr int NWV = WT / 64, FI = (WH / 64) / NWV, CAP = WH + 3, P = LT / WH, WPP = LNW / P;
    static_assert(LNW == 64 && WH * P == LT && FI * NWV * 64 == WH && WH == 4 * WT, "shape");
    // (each field holds A's run then B's, each from its 16-byte aligned-down
    // start by LDS-DMA: up to 64 bytes more than the elements)
    __shared__ alignas(16) uint64_t s_key[CAP + 8];
    __shared__ alignas(16) uint64_t s_ts[CAP + 8];
    __shared__ alignas(16) uint32_t s_rep[CAP + 16];
    __shared__ alignas(16) uint8_t s_tomb[CAP + 64];
    const uint64_t t = t0 + blockIdx.x / P;
    const uint32_t h = blockIdx.x % P;
    const LwwTile b = lww_tile(split, t, na + nb);
    const int lane = threadIdx.x & 63;
    const uint64_t word_a = bits[t * 2 * LNW + lane], word_e = bits[t * 2 * LNW + LNW + lane];
    const uint64_t ob = ic[t];                           // (with the split and bitmaps: no load after the barrier)
    uint32_t pre_a = (uint32_t)__popcll(word_a), pre_e = (uint32_t)__popcll(word_e);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t ya = __shfl_up(pre_a, o), ye = __shfl_up(pre_e, o);
        if (lane >= o) {
            pre_a += ya;
            pre_e += ye;
        }
    }
    pre_a -= (uint32_t)__popcll(word_a);
    pre_e -= (uint32_t)__popcll(word_e);
    // every index below derives from the bitmaps: a tile whose bitmaps do not
    // describe its counts raises CRDT_DEV_RANGE instead of reading out of range
    if (!bitmaps_consistent(word_a, word_e, pre_a, LNW, b.na, b.n, lane)) {
        if (threadIdx.x == 0 && blockIdx.x % P == 0) atomicOr(err, CRDT_DEV_RANGE);
        return;
    }
    // the half's runs: A [ra, ra + ca), B [rb, rb + cb); staged from ra - 2 / rb - 1
    const uint32_t ha = (uint32_t)__builtin_amdgcn_readlane(pre_a, WPP * h);       // A items before the part
    const uint32_t ha1 = h + 1 == P ? b.na : (uint32_t)__builtin_amdgcn_readlane(pre_a, WPP * (h + 1));  // ... before its end
    const uint32_t d0 = WH * h;
    const uint32_t hn = b.n > d0 ? (b.n - d0 < (uint32_t)WH ? b.n - d0 : (uint32_t)WH) : 0;   // items in the part
    if (hn == 0) return;
    const size_t ra = b.i0 + ha, rb = b.j0 + (d0 - ha);
    const uint32_t ca = ha1 - ha, cb = hn - ca;
    const uint32_t na2 = ca + 2;                         // staged A: ra-2 .. ra+ca-1 (slots 0 .. ca+1)
    // slot x of field f sits at LDS element x + (x < na2 ? oa[f] : ob[f])
    int oa_k, ob_k, oa_t, ob_t, oa_r, ob_r, oa_m, ob_m;
    {
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const size_t ga = ra >= 2 ? ra - 2 : 0, gb = rb >= 1 ? rb - 1 : 0;   // first staged element of each side
        const uint32_t ka = (uint32_t)(ra + ca - ga), kb = (uint32_t)(rb + cb - gb);
        const int sa = (int)(ga - (ra - 2)), sb = (int)(gb - (rb - 1)) + (int)na2;   // their slots
        uint32_t at = 0;
        oa_k = dma_run<uint64_t, NWV>(A.key, ga, ka, s_key, &at, wv, lane) - sa;
        ob_k = dma_run<uint64_t, NWV>(B.key, gb, kb, s_key, &at, wv, lane) - sb;
        at = 0;
        // (ts / rep / tomb read once, nontemporal: they do not evict the keys
        // the count pass left in the Infinity Cache)
        oa_t = dma_run<uint64_t, NWV, 2>(A.ts, ga, ka, s_ts, &at, wv, lane) - sa;
        ob_t = dma_run<uint64_t, NWV, 2>(B.ts, gb, kb, s_ts, &at, wv, lane) - sb;
        at = 0;
        oa_r = dma_run<uint32_t, NWV, 2>(A.rep, ga, ka, s_rep, &at, wv, lane) - sa;
        ob_r = dma_run<uint32_t, NWV, 2>(B.rep, gb, kb, s_rep, &at, wv, lane) - sb;
        at = 0;
        oa_m = dma_run<uint8_t, NWV, 2>(A.tomb, ga, ka, s_tomb, &at, wv, lane) - sa;
        ob_m = dma_run<uint8_t, NWV, 2>(B.tomb, gb, kb, s_tomb, &at, wv, lane) - sb;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA has landed in LDS
    }
    __syncthreads();
    const int wvu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    auto below = [&](uint64_t msk) -> uint32_t {        // set bits of msk below this lane
        return __builtin_amdgcn_mbcnt_hi((uint32_t)(msk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)msk, 0u));
    };
    // staged fields of slot sl
    auto tag_at = [&](uint32_t sl, uint64_t &k, uint64_t &ts, uint32_t &r) {
        const bool sa = sl < na2;
        k = s_key[(int)sl + (sa ? oa_k : ob_k)];
        ts = s_ts[(int)sl + (sa ? oa_t : ob_t)];
        r = s_rep[(int)sl + (sa ? oa_r : ob_r)];
    };
    auto tomb_at = [&](uint32_t sl) -> uint8_t { return s_tomb[(int)sl + (sl < na2 ? oa_m : ob_m)]; };
#pragma unroll
    for (int f = 0; f < FI; ++f) {
        const int w = WPP * (int)h + wvu + NWV * f;      // the tile's word
        const uint64_t wa = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(word_a >> 32), w) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((uint32_t)word_a, w);
        const uint64_t we = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(word_e >> 32), w) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((uint32_t)word_e, w);
        if (!((we >> lane) & 1)) continue;
        const uint32_t pa = (uint32_t)__builtin_amdgcn_readlane(pre_a, w) + below(wa);   // A items before (tile)
        const uint32_t rk = (uint32_t)__builtin_amdgcn_readlane(pre_e, w) + below(we);   // output rank
        const uint32_t k = 64u * (uint32_t)w + (uint32_t)lane;                          // tile merge item
        const uint32_t la = pa - ha, lb = (k - d0) - la; // A / B items of the half before this one
        const bool is_a = (wa >> lane) & 1;
        const size_t ai = ra + la;                       // A elements merged before this item
        uint64_t key, ts;
        uint32_t rep, xs;                                // the winner's staging slot
        bool on_a;
        size_t wi;
        if (is_a) {                                      // an A run end whose key B does not hold
            xs = la + 2;
            tag_at(xs, key, ts, rep);
            on_a = true;
            wi = ai;
        } else {                                         // B's run end; A's run end of the key just before it
            const uint32_t bs = na2 + 1 + lb;
            uint64_t kb_, tb, ka_ = 0, ta = 0;
            uint32_t rb_, ra_ = 0;
            tag_at(bs, kb_, tb, rb_);
            const bool a_has = ai > 0 && (tag_at(la + 1, ka_, ta, ra_), ka_ == kb_);
            const bool ya = a_has && (ta > tb || (ta == tb && ra_ >= rb_));   // A wins an equal tag
            key = kb_;
            on_a = ya;
            xs = ya ? la + 1 : bs;
            ts = ya ? ta : tb;
            rep = ya ? ra_ : rb_;
            wi = ya ? ai - 1 : rb + lb;
        }
        // the first copy of the winner's tag on its side: its staged
        // predecessor, then (rare) global memory before the staging
        uint8_t tomb = tomb_at(xs);
        const uint32_t lo = on_a ? 0u : na2;             // first staged slot of the side
        bool more = wi > 0;
        uint32_t sl = xs;
        while (more && sl > lo) {
            uint64_t pk, pt;
            uint32_t pr;
            tag_at(sl - 1, pk, pt, pr);
            if (pk != key || pt != ts || pr != rep) {
                more = false;
                break;
            }
            --sl;
            --wi;
            tomb = tomb_at(sl);
            more = wi > 0;
        }
        if (more && sl == lo) {                          // the run of copies reaches past the staging
            const size_t fc = first_copy(on_a ? A.key : B.key, on_a ? A.ts : B.ts, on_a ? A.rep : B.rep, wi, key, ts,
                                         rep);
            tomb = (on_a ? A.tomb : B.tomb)[fc];
        }
        const uint64_t o = ob + rk;
        if (o >= na + nb) {                              // (consistent bitmaps never get here)
            atomicOr(err, CRDT_DEV_RANGE);
            continue;
        }
        out.key[o] = key;
        out.ts[o] = ts;
        out.rep[o] = rep;
        out.tomb[o] = tomb;
    }
}

// ---------------------------------------------------------------- OR-Set, two passes
// The same structure for the OR-Set, over TAGS: one output per distinct tag
// (key, ts, rep) in tag order, its tomb the OR over every copy; in the
// stable merge (A first on an equal tag) a tag's copies are consecutive --
// A's, then B's -- so the first copy emits:
//   k_or_split : merge-path splits of 2048-item tiles over the tags;
//   k_or_count : per tile the tags merged in LDS (512 threads x 4 items):
//                bitmaps `isa` and `emit` (the item's tag differs from the
//                previous merged tag), 512 B per tile, the emit count;
//   k_chunk_scan;
//   k_or_write : per part of a tile (sets.or_parts), the part's A and B runs
//                staged in LDS by LDS-DMA (every field once); an emitting
//                item ORs the tombs of its tag's copies -- forward over A's,
//                then B's from the B position of the item -- and stores at
//                its rank.
constexpr int OT = 2048;                 // merge items per OR tile
constexpr int OCB = 512;                 // count pass threads (4 items each; 256 x 8: 120 us, 1024 x 2: 153 us, against 111)
constexpr int OWT = 512;                 // write pass threads (4 items each)
constexpr int ONW = OT / 64;             // bitmap words per tile and bitmap

// The merge-path split of diagonal t * OT (one 16-lane group per diagonal,
// four per wave; every lane of the wave calls it: the ballots are wave-wide).
__device__ __forceinline__ void or_split_diag(const crdt_tuples &A, const crdt_tuples &B, size_t na, size_t nb,
                                              size_t ntiles, size_t t, uint64_t *__restrict__ split) {
    const int lane = threadIdx.x & 63, grp = lane >> 4, gl = lane & 15;
    const size_t n = na + nb;
    const size_t d = t * OT < n ? t * OT : n;
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

__global__ __launch_bounds__(256) void k_or_split(crdt_tuples A, crdt_tuples B, size_t na, size_t nb, size_t ntiles,
                                                  uint64_t *__restrict__ split) {
    const size_t t = ((((size_t)blockIdx.x * 256 + threadIdx.x) >> 6) << 2) + (size_t)((threadIdx.x & 63) >> 4);
    or_split_diag(A, B, na, nb, ntiles, t, split);
}

__device__ __forceinline__ LwwTile or_tile(const uint64_t *__restrict__ split, uint64_t t, size_t n) {
    LwwTile b;
    const size_t d0 = (size_t)t * OT, d1 = d0 + OT < n ? d0 + OT : n;
    b.i0 = split[t];
    b.i1 = split[t + 1];
    b.j0 = d0 - b.i0;
    b.j1 = d1 - b.i1;
    b.na = (uint32_t)(b.i1 - b.i0);
    b.nb = (uint32_t)(b.j1 - b.j0);
    b.n = b.na + b.nb;
    return b;
}

template <int NT>
__global__ __launch_bounds__(NT) void k_or_count(crdt_tuples A, crdt_tuples B, size_t na, size_t nb,
                                                 const uint64_t *__restrict__ split, uint32_t *__restrict__ tcnt,
                                                 uint64_t *__restrict__ bits, uint64_t t0) {
    constexpr int NI = OT / NT, LPW = 64 / NI, CAP = OT + 2;
    // staged: A[i0-1], A part, B[j0-1], B part (slot 0 of each side: the
    // element before the tile, the first item's merged predecessor candidate)
    __shared__ uint64_t sk[CAP], st[CAP];
    __shared__ uint32_t sr[CAP];
    __shared__ uint32_t s_w[NT / 64];
    const uint64_t t = t0 + blockIdx.x;
    const LwwTile b = or_tile(split, t, na + nb);
    const uint32_t nsa = b.na + 1, nst = nsa + b.nb + 1;
    {
        uint64_t k[NI + 1], ts[NI + 1];
        uint32_t r[NI + 1];
#pragma unroll
        for (int j = 0; j <= NI; ++j) {                  // every staging load issued before the first store
            const uint32_t x = threadIdx.x + (uint32_t)j * NT;
            const bool on_a = x < nsa;
            const size_t g = on_a ? b.i0 - 1 + x : b.j0 - 1 + (x - nsa);
            const bool v = x < nst && (on_a ? b.i0 + x >= 1 : b.j0 + (x - nsa) >= 1);
            k[j] = v ? (on_a ? A.key : B.key)[g] : 0;
            ts[j] = v ? (on_a ? A.ts : B.ts)[g] : 0;
            r[j] = v ? (on_a ? A.rep : B.rep)[g] : 0;
        }
#pragma unroll
        for (int j = 0; j <= NI; ++j) {
            const uint32_t x = threadIdx.x + (uint32_t)j * NT;
            if (x < nst) {
                sk[x] = k[j];
                st[x] = ts[j];
                sr[x] = r[j];
            }
        }
    }
    __syncthreads();
    // side views: A element a of the tile at slot 1 + a, B element j at nsa + 1 + j
#define OA(x) Tag{sk[1 + (x)], st[1 + (x)], sr[1 + (x)]}
#define OB(x) Tag{sk[nsa + 1 + (x)], st[nsa + 1 + (x)], sr[nsa + 1 + (x)]}
    const uint32_t k0 = threadIdx.x * NI < b.n ? threadIdx.x * NI : b.n;
    const uint32_t k1 = k0 + NI < b.n ? k0 + NI : b.n;
    uint32_t isa = 0, emit = 0;
    if (k0 < k1) {
        uint32_t lo = k0 > b.nb ? k0 - b.nb : 0, hi = k0 < b.na ? k0 : b.na;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            const uint64_t ka = sk[1 + mid], kb = sk[nsa + 1 + (k0 - 1 - mid)];
            const bool le = ka != kb ? ka < kb : tag_le(OA(mid), OB(k0 - 1 - mid));
            if (le) lo = mid + 1;
            else hi = mid;
        }
        uint32_t ia = lo, ib = k0 - lo;
        // the merged predecessor of item k0: the later of A[ia-1], B[ib-1]
        // (A first on an equal tag), each possibly the element before the tile
        const bool hpa = b.i0 + ia > 0, hpb = b.j0 + ib > 0;
        const Tag pa{sk[ia], st[ia], sr[ia]}, pb{sk[nsa + ib], st[nsa + ib], sr[nsa + ib]};
        bool has_prev = hpa || hpb;
        Tag prev = tag_sel(hpa && hpb ? tag_le(pa, pb) : !hpa, pb, pa);
        Tag ha = ia < b.na ? OA(ia) : Tag{0, 0, 0}, hb = ib < b.nb ? OB(ib) : Tag{0, 0, 0};
        for (uint32_t i = 0; i < k1 - k0; ++i) {
            const bool take_a = ia < b.na && (ib >= b.nb || tag_le(ha, hb));
            const Tag cur = tag_sel(take_a, ha, hb);
            if (!has_prev || !tag_eq(prev, cur)) emit |= 1u << i;
            prev = cur;
            has_prev = true;
            if (take_a) {
                isa |= 1u << i;
                ++ia;
                if (ia < b.na) ha = OA(ia);
            } else {
                ++ib;
                if (ib < b.nb) hb = OB(ib);
            }
        }
    }
#undef OA
#undef OB
    const int lane = threadIdx.x & 63, sh = (lane % LPW) * NI;
    uint64_t wl = (uint64_t)isa << sh, we = (uint64_t)emit << sh;
#pragma unroll
    for (int o = 1; o < LPW; o <<= 1) {
        wl |= (uint64_t)__shfl_xor((unsigned long long)wl, o);
        we |= (uint64_t)__shfl_xor((unsigned long long)we, o);
    }
    if (lane % LPW == 0) {
        const uint32_t w = threadIdx.x / LPW;
        bits[t * 2 * ONW + w] = wl;
        bits[t * 2 * ONW + ONW + w] = we;
    }
    uint32_t x = (uint32_t)__popc(emit);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) s_w[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
#pragma unroll
        for (int k = 0; k < NT / 64; ++k) tot += s_w[k];
        tcnt[t] = tot;
    }
}

// k_or_count with the tile's key / ts / rep staged by LDS-DMA (each side's
// run from the element before the tile, from its 16-byte aligned-down start:
// no VGPR round trip; sets.or_count_dma).  Same merge, same bitmaps.
template <int NT>
__global__ __launch_bounds__(NT) void k_or_count_dma(crdt_tuples A, crdt_tuples B, size_t na, size_t nb,
                                                     const uint64_t *__restrict__ split, uint32_t *__restrict__ tcnt,
                                                     uint64_t *__restrict__ bits, uint64_t t0) {
    constexpr int NI = OT / NT, LPW = 64 / NI, CAP = OT + 2;
    __shared__ alignas(16) uint64_t sk[CAP + 8], st[CAP + 8];
    __shared__ alignas(16) uint32_t sr[CAP + 16];
    __shared__ uint32_t s_w[NT / 64];
    const uint64_t t = t0 + blockIdx.x;
    const LwwTile b = or_tile(split, t, na + nb);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), ln = threadIdx.x & 63;
    // each side from the element before the tile (when there is one): element
    // x of the tile's A run (x >= -1) is at field index oa_f + x
    const uint32_t pa = b.i0 > 0 ? 1u : 0u, pb = b.j0 > 0 ? 1u : 0u;
    uint32_t at = 0;
    const int oa_k = dma_run<uint64_t, NT / 64>(A.key, b.i0 - pa, b.na + pa, sk, &at, wv, ln) + (int)pa;
    const int ob_k = dma_run<uint64_t, NT / 64>(B.key, b.j0 - pb, b.nb + pb, sk, &at, wv, ln) + (int)pb;
    at = 0;
    const int oa_t = dma_run<uint64_t, NT / 64>(A.ts, b.i0 - pa, b.na + pa, st, &at, wv, ln) + (int)pa;
    const int ob_t = dma_run<uint64_t, NT / 64>(B.ts, b.j0 - pb, b.nb + pb, st, &at, wv, ln) + (int)pb;
    at = 0;
    const int oa_r = dma_run<uint32_t, NT / 64>(A.rep, b.i0 - pa, b.na + pa, sr, &at, wv, ln) + (int)pa;
    const int ob_r = dma_run<uint32_t, NT / 64>(B.rep, b.j0 - pb, b.nb + pb, sr, &at, wv, ln) + (int)pb;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA has landed in LDS
    __syncthreads();
#define OA(x) Tag{sk[oa_k + (int)(x)], st[oa_t + (int)(x)], sr[oa_r + (int)(x)]}
#define OB(x) Tag{sk[ob_k + (int)(x)], st[ob_t + (int)(x)], sr[ob_r + (int)(x)]}
    const uint32_t k0 = threadIdx.x * NI < b.n ? threadIdx.x * NI : b.n;
    const uint32_t k1 = k0 + NI < b.n ? k0 + NI : b.n;
    uint32_t isa = 0, emit = 0;
    if (k0 < k1) {
        uint32_t lo = k0 > b.nb ? k0 - b.nb : 0, hi = k0 < b.na ? k0 : b.na;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            const uint64_t ka = sk[oa_k + (int)mid], kb = sk[ob_k + (int)(k0 - 1 - mid)];
            const bool le = ka != kb ? ka < kb : tag_le(OA(mid), OB(k0 - 1 - mid));
            if (le) lo = mid + 1;
            else hi = mid;
        }
        uint32_t ia = lo, ib = k0 - lo;
        // the merged predecessor of item k0: the later of A[ia-1], B[ib-1]
        // (A first on an equal tag), each possibly the element before the tile
        const bool hpa = b.i0 + ia > 0, hpb = b.j0 + ib > 0;
        const Tag qa = hpa ? OA((int)ia - 1) : Tag{0, 0, 0}, qb = hpb ? OB((int)ib - 1) : Tag{0, 0, 0};
        bool has_prev = hpa || hpb;
        Tag prev = tag_sel(hpa && hpb ? tag_le(qa, qb) : !hpa, qb, qa);
        Tag ha = ia < b.na ? OA(ia) : Tag{0, 0, 0}, hb = ib < b.nb ? OB(ib) : Tag{0, 0, 0};
        for (uint32_t i = 0; i < k1 - k0; ++i) {
            const bool take_a = ia < b.na && (ib >= b.nb || tag_le(ha, hb));
            const Tag cur = tag_sel(take_a, ha, hb);
            if (!has_prev || !tag_eq(prev, cur)) emit |= 1u << i;
            prev = cur;
            has_prev = true;
            if (take_a) {
                isa |= 1u << i;
                ++ia;
                if (ia < b.na) ha = OA(ia);
            } else {
                ++ib;
                if (ib < b.nb) hb = OB(ib);
            }
        }
    }
#undef OA
#undef OB
    const int lane = threadIdx.x & 63, sh = (lane % LPW) * NI;
    uint64_t wl = (uint64_t)isa << sh, we = (uint64_t)emit << sh;
#pragma unroll
    for (int o = 1; o < LPW; o <<= 1) {
        wl |= (uint64_t)__shfl_xor((unsigned long long)wl, o);
        we |= (uint64_t)__shfl_xor((unsigned long long)we, o);
    }
    if (lane % LPW == 0) {
        const uint32_t w = threadIdx.x / LPW;
        bits[t * 2 * ONW + w] = wl;
        bits[t * 2 * ONW + ONW + w] = we;
    }
    uint32_t x = (uint32_t)__popc(emit);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) s_w[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
#pragma unroll
        for (int k = 0; k < NT / 64; ++k) tot += s_w[k];
        tcnt[t] = tot;
    }
}

// WH merge items per workgroup (a 1/P of a tile, P = OT / WH), WT threads
template <int WH = OT, int WT = OWT>
__global__ __launch_bounds__(WT) void k_or_write(crdt_tuples A, crdt_tuples B, size_t na, size_t nb,
                                                 const uint64_t *__restrict__ split,
                                                 const uint64_t *__restrict__ bits, const uint64_t *__restrict__ ic,
                                                 crdt_tuples out, uint64_t t0, uint32_t *__restrict__ err) {
    constexpr int NWV = WT / 64, P = OT / WH, WPP = ONW / P, FI = WPP / NWV, CAP = WH + 2;
    static_assert(FI * NWV == WPP && WH * P == OT && ONW <= 64 && WH == 4 * WT, "shape");
    __shared__ alignas(16) uint64_t s_key[CAP + 8];
    __shared__ alignas(16) uint64_t s_ts[CAP + 8];
    __shared__ alignas(16) uint32_t s_rep[CAP + 16];
    __shared__ alignas(16) uint8_t s_tomb[CAP + 64];
    const uint64_t t = t0 + blockIdx.x / P;
    const uint32_t h = blockIdx.x % P;
    const LwwTile b = or_tile(split, t, na + nb);
    const int lane = threadIdx.x & 63;
    const bool wl_ok = lane < ONW;
    // split, bitmap words and offset loads issued together (none after the barrier)
    const uint64_t word_a = wl_ok ? bits[t * 2 * ONW + lane] : 0, word_e = wl_ok ? bits[t * 2 * ONW + ONW + lane] : 0;
    const uint64_t ob = ic[t];
    uint32_t pre_a = (uint32_t)__popcll(word_a), pre_e = (uint32_t)__popcll(word_e);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t ya = __shfl_up(pre_a, o), ye = __shfl_up(pre_e, o);
        if (lane >= o) {
            pre_a += ya;
            pre_e += ye;
        }
    }
    pre_a -= (uint32_t)__popcll(word_a);
    pre_e -= (uint32_t)__popcll(word_e);
    if (!bitmaps_consistent(word_a, word_e, pre_a, ONW, b.na, b.n, lane)) {   // (see k_lww_write)
        if (threadIdx.x == 0 && blockIdx.x % P == 0) atomicOr(err, CRDT_DEV_RANGE);
        return;
    }
    // the part's runs: A [pa0, pa0 + ca), B [pb0, pb0 + cb) (tile-relative)
    const uint32_t d0 = WH * h;
    const uint32_t hn = b.n > d0 ? (b.n - d0 < (uint32_t)WH ? b.n - d0 : (uint32_t)WH) : 0;   // items in the part
    if (hn == 0) return;
    const uint32_t pa0 = P == 1 ? 0u : (uint32_t)__builtin_amdgcn_readlane(pre_a, WPP * h);
    const uint32_t pa1 = h + 1 == P ? b.na : (uint32_t)__builtin_amdgcn_readlane(pre_a, WPP * (h + 1));
    const uint32_t ca = pa1 - pa0, cb = hn - ca, pb0 = d0 - pa0;
    const size_t ga = b.i0 + pa0, gb = b.j0 + pb0;       // global index of each run's first element
    // staged by LDS-DMA: A run (slots 0 .. ca-1), then B run (slots ca ..),
    // every field once; slot x of field f at LDS element x + (x < ca ? oa[f] : ob[f])
    int oa_k, ob_k, oa_t, ob_t, oa_r, ob_r, oa_m, ob_m;
    {
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const int sb = (int)ca;
        uint32_t at = 0;
        oa_k = dma_run<uint64_t, NWV>(A.key, ga, ca, s_key, &at, wv, lane);
        ob_k = dma_run<uint64_t, NWV>(B.key, gb, cb, s_key, &at, wv, lane) - sb;
        at = 0;
        oa_t = dma_run<uint64_t, NWV>(A.ts, ga, ca, s_ts, &at, wv, lane);
        ob_t = dma_run<uint64_t, NWV>(B.ts, gb, cb, s_ts, &at, wv, lane) - sb;
        at = 0;
        oa_r = dma_run<uint32_t, NWV>(A.rep, ga, ca, s_rep, &at, wv, lane);
        ob_r = dma_run<uint32_t, NWV>(B.rep, gb, cb, s_rep, &at, wv, lane) - sb;
        at = 0;
        oa_m = dma_run<uint8_t, NWV>(A.tomb, ga, ca, s_tomb, &at, wv, lane);
        ob_m = dma_run<uint8_t, NWV>(B.tomb, gb, cb, s_tomb, &at, wv, lane) - sb;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA has landed in LDS
    }
    __syncthreads();
    const int wvu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    auto below = [&](uint64_t msk) -> uint32_t {        // set bits of msk below this lane
        return __builtin_amdgcn_mbcnt_hi((uint32_t)(msk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)msk, 0u));
    };
#pragma unroll
    for (int f = 0; f < FI; ++f) {
        const int w = WPP * (int)h + wvu + NWV * f;      // the tile's word
        // (readlane returns int: widen through uint32_t, never sign-extend)
        const uint64_t wa = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(word_a >> 32), w) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((uint32_t)word_a, w);
        const uint64_t we = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(word_e >> 32), w) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((uint32_t)word_e, w);
        if (!((we >> lane) & 1)) continue;
        const uint32_t la = (uint32_t)__builtin_amdgcn_readlane(pre_a, w) + below(wa) - pa0;   // A items before (part)
        const uint32_t rk = (uint32_t)__builtin_amdgcn_readlane(pre_e, w) + below(we);         // output rank (tile)
        const uint32_t k = 64u * (uint32_t)w + (uint32_t)lane - d0;
        const uint32_t lb = k - la;                      // B items before (part)
        const bool is_a = (wa >> lane) & 1;
        const uint32_t xs = is_a ? la : ca + lb;         // the first copy's slot
        const int xo = is_a ? 0 : 1;
        const uint64_t key = s_key[(int)xs + (xo ? ob_k : oa_k)], ts = s_ts[(int)xs + (xo ? ob_t : oa_t)];
        const uint32_t rep = s_rep[(int)xs + (xo ? ob_r : oa_r)];
        uint32_t tomb = 0;
        // A's copies (an A first copy only), then B's from position lb:
        // in the staging, then past the part in global memory (rare)
        if (is_a) {
            uint32_t s = la;
            while (s < ca && s_key[(int)s + oa_k] == key && s_ts[(int)s + oa_t] == ts && s_rep[(int)s + oa_r] == rep)
                tomb |= s_tomb[(int)(s++) + oa_m];
            if (s == ca)
                for (size_t g = ga + ca; g < na && A.key[g] == key && A.ts[g] == ts && A.rep[g] == rep; ++g)
                    tomb |= A.tomb[g];
        }
        {
            uint32_t s = lb;
            while (s < cb && s_key[(int)(ca + s) + ob_k] == key && s_ts[(int)(ca + s) + ob_t] == ts &&
                   s_rep[(int)(ca + s) + ob_r] == rep)
                tomb |= s_tomb[(int)(ca + s++) + ob_m];
            if (s == cb)
                for (size_t g = gb + cb; g < nb && B.key[g] == key && B.ts[g] == ts && B.rep[g] == rep; ++g)
                    tomb |= B.tomb[g];
        }
        const uint64_t o = ob + rk;
        if (o >= na + nb) {                              // (consistent bitmaps never get here)
            atomicOr(err, CRDT_DEV_RANGE);
            continue;
        }
        out.key[o] = key;
        out.ts[o] = ts;
        out.rep[o] = rep;
        out.tomb[o] = (uint8_t)tomb;
    }
}

// The chunked two-pass schedule.  count(t0, n, s) / scan(t0, n, count_out,
// s) / write(t0, n, s) enqueue one chunk's pass on the context's stream; a
// chunk is at most kScanMax tiles (one scan workgroup), or `chunk` tiles
// (sets.lww_chunk / sets.or_chunk, diagnostic build: smaller chunks measured
// slower; so did a second stream for the counts).
template <class CountF, class ScanF, class WriteF>
static int two_pass(crdt_ctx *ctx, size_t ntiles, uint64_t *out_count, CountF count, ScanF scan, WriteF write,
                    size_t chunk, bool fail_bits, uint64_t *bits, size_t bits_bytes) {
    if (chunk == 0 || chunk > kScanMax) chunk = kScanMax;
    const hipStream_t s = ctx->stream;
    if (fail_bits) {                                     // failpoint: one chunk, bitmaps zeroed before the writes
        for (size_t t0 = 0; t0 < ntiles; t0 += chunk) {
            const uint32_t n = (uint32_t)std::min(chunk, ntiles - t0);
            count(t0, n, s);
            scan(t0, n, t0 + n == ntiles ? out_count : nullptr, s);
        }
        hipError_t e = hipMemsetAsync(bits, 0, bits_bytes, s);
        if (e != hipSuccess) return hip_fail(ctx, e);
        for (size_t t0 = 0; t0 < ntiles; t0 += chunk) write(t0, (uint32_t)std::min(chunk, ntiles - t0), s);
        return check_launch(ctx);
    }
    for (size_t t0 = 0; t0 < ntiles; t0 += chunk) {
        const uint32_t n = (uint32_t)std::min(chunk, ntiles - t0);
        count(t0, n, s);
        scan(t0, n, t0 + n == ntiles ? out_count : nullptr, s);
        write(t0, n, s);
    }
    return check_launch(ctx);
}

static int lww_merge_keyruns(crdt_ctx *ctx, const crdt_tuples &A, size_t na, const crdt_tuples &B, size_t nb,
                             const crdt_tuples &O, uint64_t *out_count) {
    const size_t n = na + nb;
    const size_t ntiles = (n + LT - 1) / LT;
    if (ntiles >= 0x7fffffffULL || n >= (1ULL << 62)) return CRDT_E_RANGE;
    const size_t need = Carve::round((ntiles + 1) * 8) + Carve::round(ntiles * 4 + 4) + Carve::round((ntiles + 1) * 8) +
                        Carve::round(ntiles * 2 * LNW * 8) + 1024;
    int rc = ws_reserve(ctx, need);
    if (rc) return rc;
    Carve w(ctx->ws);
    uint64_t *split = w.take<uint64_t>(ntiles + 1);
    uint32_t *tcnt = w.take<uint32_t>(ntiles + 1);
    uint64_t *ic = w.take<uint64_t>(ntiles + 1);
    uint64_t *bits = w.take<uint64_t>(ntiles * 2 * LNW);
    uint32_t *err = ctx->dev_status;
    const uint64_t *ka = A.key, *kb = B.key;             // (nullptr for an empty side: never dereferenced)
    k_lww_split<<<(unsigned)((ntiles + 1 + 15) / 16), 256, 0, ctx->stream>>>(ka, kb, na, nb, ntiles, split);
    // write-pass workgroups per tile (sets.lww_parts): 1/P of a tile's items, 4 per thread
    const unsigned P = (unsigned)g_lww_parts;
    auto cnt = [&](size_t t0, uint32_t nt, hipStream_t s) {
        k_lww_count<<<nt, LCB, 0, s>>>(ka, kb, na, nb, split, tcnt, bits, t0);
    };
    auto scn = [&](size_t t0, uint32_t nt, uint64_t *c, hipStream_t s) {
        k_chunk_scan<<<1, 1024, 0, s>>>(tcnt, t0, nt, ic, c);
    };
    auto wr = [&](size_t t0, uint32_t nt, hipStream_t s) {
        const unsigned g = P * nt;
        if (P == 2) k_lww_write<2048, 512><<<g, 512, 0, s>>>(A, B, na, nb, split, bits, ic, O, t0, err);
        else if (P == 8) k_lww_write<512, 128><<<g, 128, 0, s>>>(A, B, na, nb, split, bits, ic, O, t0, err);
        else if (P == 16) k_lww_write<256, 64><<<g, 64, 0, s>>>(A, B, na, nb, split, bits, ic, O, t0, err);
        else k_lww_write<1024, 256><<<g, 256, 0, s>>>(A, B, na, nb, split, bits, ic, O, t0, err);
    };
    return two_pass(ctx, ntiles, out_count, cnt, scn, wr, (size_t)g_lww_chunk, take_fail_zero_bits(), bits,
                    ntiles * 2 * LNW * 8);
}

static int orset_merge_twopass(crdt_ctx *ctx, const crdt_tuples &A, size_t na, const crdt_tuples &B, size_t nb,
                               const crdt_tuples &O, uint64_t *out_count) {
    const size_t n = na + nb;
    const size_t ntiles = (n + OT - 1) / OT;
    if (ntiles >= 0x7fffffffULL || n >= (1ULL << 62)) return CRDT_E_RANGE;
    const size_t need = Carve::round((ntiles + 1) * 8) + Carve::round(ntiles * 4 + 4) + Carve::round((ntiles + 1) * 8) +
                        Carve::round(ntiles * 2 * ONW * 8) + 1024;
    int rc = ws_reserve(ctx, need);
    if (rc) return rc;
    Carve w(ctx->ws);
    uint64_t *split = w.take<uint64_t>(ntiles + 1);
    uint32_t *tcnt = w.take<uint32_t>(ntiles + 1);
    uint64_t *ic = w.take<uint64_t>(ntiles + 1);
    uint64_t *bits = w.take<uint64_t>(ntiles * 2 * ONW);
    uint32_t *err = ctx->dev_status;
    k_or_split<<<(unsigned)((ntiles + 1 + 15) / 16), 256, 0, ctx->stream>>>(A, B, na, nb, ntiles, split);
    // write-pass workgroups per tile (sets.or_parts): 1/P of a tile's items, 4 per thread
    const unsigned P = (unsigned)g_or_parts;
    auto cnt = [&](size_t t0, uint32_t nt, hipStream_t s) {
        if (g_or_count_dma) k_or_count_dma<OCB><<<nt, OCB, 0, s>>>(A, B, na, nb, split, tcnt, bits, t0);
        else k_or_count<OCB><<<nt, OCB, 0, s>>>(A, B, na, nb, split, tcnt, bits, t0);
    };
    auto scn = [&](size_t t0, uint32_t nt, uint64_t *c, hipStream_t s) {
        k_chunk_scan<<<1, 1024, 0, s>>>(tcnt, t0, nt, ic, c);
    };
    auto wr = [&](size_t t0, uint32_t nt, hipStream_t s) {
        const unsigned g = P * nt;
        if (P == 2) k_or_write<1024, 256><<<g, 256, 0, s>>>(A, B, na, nb, split, bits, ic, O, t0, err);
        else if (P == 4) k_or_write<512, 128><<<g, 128, 0, s>>>(A, B, na, nb, split, bits, ic, O, t0, err);
        else k_or_write<2048, 512><<<g, 512, 0, s>>>(A, B, na, nb, split, bits, ic, O, t0, err);
    };
    return two_pass(ctx, ntiles, out_count, cnt, scn, wr, (size_t)g_or_chunk, take_fail_zero_bits(), bits,
                    ntiles * 2 * ONW * 8);
}

// ---------------------------------------------------------------- stable merge (no dedup)
// out = the stable merge of A and B (every tuple kept; on an equal tag A's
// copies first) -- the rank-order merge of the runs a key-range owner
// receives in crdt_shard_*_merge_local.  Its length is na + nb, known on the
// host, so a tree of these merges needs no read-back between levels.  Tiles
// of OT merge items from k_or_split; per tile both runs staged in LDS, every
// item's output position = its index in its run + its rank in the other run
// (B elements strictly below an A tag, A elements at or below a B tag).
template <int NT>
__device__ __forceinline__ void tmerge_tile(const crdt_tuples &A, const crdt_tuples &B, size_t na, size_t nb,
                                            const uint64_t *__restrict__ split, const crdt_tuples &out, uint64_t t,
                                            uint64_t *sk, uint64_t *st, uint32_t *sr, uint8_t *sm) {
    // both runs staged in LDS (A at slots [0, na), B at [na, n)); thread k
    // merges items [k NI, (k+1) NI) of the tile after a merge-path search
    // of its diagonal (A first on an equal tag), the merged tuples are put
    // back into LDS in merged order, then stored coalesced.  (Round 4's form
    // -- every item binary-searched its rank in the other run, ~11 dependent
    // 3-field LDS compares per item -- ran at ~1.6 TB/s.)
    constexpr int NI = OT / NT;
    const LwwTile b = or_tile(split, t, na + nb);
#pragma unroll
    for (int j = 0; j < NI; ++j) {
        const uint32_t x = threadIdx.x + (uint32_t)j * NT;
        if (x >= b.n) continue;
        const bool on_a = x < b.na;
        const size_t g = on_a ? b.i0 + x : b.j0 + (x - b.na);
        const crdt_tuples &S = on_a ? A : B;
        sk[x] = S.key[g];
        st[x] = S.ts[g];
        sr[x] = S.rep[g];
        sm[x] = S.tomb[g];
    }
    __syncthreads();
    auto tg = [&](uint32_t x) { return Tag{sk[x], st[x], sr[x]}; };
    const uint32_t k0 = threadIdx.x * NI < b.n ? threadIdx.x * NI : b.n;
    const uint32_t k1 = k0 + NI < b.n ? k0 + NI : b.n;
    uint64_t ok[NI], ot[NI];
    uint32_t orr[NI];
    uint8_t om[NI];
    {
        uint32_t lo = k0 > b.nb ? k0 - b.nb : 0, hi = k0 < b.na ? k0 : b.na;
        while (lo < hi) {                                // P(i) = A[i] <= B[k0-1-i]: true below the split
            const uint32_t mid = (lo + hi) >> 1;
            if (tag_le(tg(mid), tg(b.na + (k0 - 1 - mid)))) lo = mid + 1;
            else hi = mid;
        }
        uint32_t ia = lo, ib = k0 - lo;
#pragma unroll
        for (int j = 0; j < NI; ++j) {
            if ((uint32_t)j >= k1 - k0) break;
            const bool take_a = ia < b.na && (ib >= b.nb || tag_le(tg(ia), tg(b.na + ib)));
            const uint32_t x = take_a ? ia : b.na + ib;
            ok[j] = sk[x];
            ot[j] = st[x];
            orr[j] = sr[x];
            om[j] = sm[x];
            ia += take_a ? 1u : 0u;
            ib += take_a ? 0u : 1u;
        }
    }
    __syncthreads();                                     // every staged input read
#pragma unroll
    for (int j = 0; j < NI; ++j) {
        if ((uint32_t)j >= k1 - k0) break;
        const uint32_t x = k0 + (uint32_t)j;
        sk[x] = ok[j];
        st[x] = ot[j];
        sr[x] = orr[j];
        sm[x] = om[j];
    }
    __syncthreads();
    const size_t o0 = (size_t)t * OT;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
        const uint32_t x = threadIdx.x + (uint32_t)j * NT;
        if (x >= b.n) continue;
        out.key[o0 + x] = sk[x];
        out.ts[o0 + x] = st[x];
        out.rep[o0 + x] = sr[x];
        out.tomb[o0 + x] = sm[x];
    }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_tmerge(crdt_tuples A, crdt_tuples B, size_t na, size_t nb,
                                               const uint64_t *__restrict__ split, crdt_tuples out) {
    __shared__ uint64_t sk[OT], st[OT];
    __shared__ uint32_t sr[OT];
    __shared__ uint8_t sm[OT];
    tmerge_tile<NT>(A, B, na, nb, split, out, blockIdx.x, sk, st, sr, sm);
}

// Up to kMergeBatch independent stable merges in ONE split launch and ONE
// merge launch (a level of the key-range owner's rank-order merge tree, both
// sides: crdt_shard_*_merge_local).  Pair p's tiles are tile0[p] ..
// tile0[p+1]; its split entries (ntiles_p + 1 of them) start at tile0[p] + p.
// (One crdt_tuples_merge per pair paid ~27 us of fixed split + merge latency
// each: 112 of them per distributed set merge at R = 8.)
constexpr int kMergeBatch = 16;
struct MergeBatch {
    crdt_tuples A[kMergeBatch], B[kMergeBatch], O[kMergeBatch];
    uint64_t na[kMergeBatch], nb[kMergeBatch];
    uint32_t tile0[kMergeBatch + 1];
    uint32_t np;
};

__device__ __forceinline__ uint32_t batch_pair(const MergeBatch &mb, uint64_t x, uint32_t per_pair_extra) {
    uint32_t p = 0;                                      // the last p with tile0[p] + p * extra <= x
    for (uint32_t q = 1; q < mb.np; ++q)
        if ((uint64_t)mb.tile0[q] + (uint64_t)q * per_pair_extra <= x) p = q;
    return p;
}

__global__ __launch_bounds__(256) void k_or_split_batch(MergeBatch mb, uint64_t *__restrict__ split) {
    const uint64_t e = ((((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6) << 2) + (uint64_t)((threadIdx.x & 63) >> 4);
    const uint32_t p = batch_pair(mb, e, 1);
    const uint64_t s0 = (uint64_t)mb.tile0[p] + p, nt = mb.tile0[p + 1] - mb.tile0[p];
    // entries past the last pair's (nt + 1) compute nothing: t > ntiles
    const uint64_t t = e - s0;
    or_split_diag(mb.A[p], mb.B[p], mb.na[p], mb.nb[p], nt, t, split + s0);
}

template <int NT>
__global__ __launch_bounds__(NT) void k_tmerge_batch(MergeBatch mb, const uint64_t *__restrict__ split) {
    __shared__ uint64_t sk[OT], st[OT];
    __shared__ uint32_t sr[OT];
    __shared__ uint8_t sm[OT];
    const uint32_t p = batch_pair(mb, blockIdx.x, 0);
    tmerge_tile<NT>(mb.A[p], mb.B[p], mb.na[p], mb.nb[p], split + mb.tile0[p] + p, mb.O[p],
                    blockIdx.x - mb.tile0[p], sk, st, sr, sm);
}

// Every pair's stable merge (tuples_merge_stable of each), kMergeBatch pairs
// per pair of launches.
int tuples_merge_stable_batch(crdt_ctx *ctx, const std::vector<MergePairArg> &pairs) {
    for (size_t p0 = 0; p0 < pairs.size(); p0 += kMergeBatch) {
        MergeBatch mb{};
        uint64_t tiles = 0;
        const size_t np = std::min(pairs.size() - p0, (size_t)kMergeBatch);
        for (size_t q = 0; q < np; ++q) {
            const MergePairArg &x = pairs[p0 + q];
            const crdt_tuples empty{nullptr, nullptr, nullptr, nullptr};
            mb.A[q] = x.na ? x.A : empty;
            mb.B[q] = x.nb ? x.B : empty;
            mb.O[q] = x.O;
            mb.na[q] = x.na;
            mb.nb[q] = x.nb;
            mb.tile0[q] = (uint32_t)tiles;
            tiles += (x.na + x.nb + OT - 1) / OT;
            if (tiles >= 0x7fffffffULL) return CRDT_E_RANGE;
        }
        mb.tile0[np] = (uint32_t)tiles;
        mb.np = (uint32_t)np;
        if (tiles == 0) continue;
        const uint64_t entries = tiles + np;
        int rc = ws_reserve(ctx, Carve::round(entries * 8) + 1024);
        if (rc) return rc;
        uint64_t *split = (uint64_t *)ctx->ws;
        k_or_split_batch<<<(unsigned)((entries + 15) / 16), 256, 0, ctx->stream>>>(mb, split);
        k_tmerge_batch<512><<<(unsigned)tiles, 512, 0, ctx->stream>>>(mb, split);
        rc = check_launch(ctx);
        if (rc) return rc;
    }
    return CRDT_OK;
}

int tuples_merge_stable(crdt_ctx *ctx, const crdt_tuples &A, size_t na, const crdt_tuples &B, size_t nb,
                        const crdt_tuples &O) {
    const size_t n = na + nb;
    if (n == 0) return CRDT_OK;
    const size_t ntiles = (n + OT - 1) / OT;
    if (ntiles >= 0x7fffffffULL || n >= (1ULL << 62)) return CRDT_E_RANGE;
    int rc = ws_reserve(ctx, Carve::round((ntiles + 1) * 8) + 1024);
    if (rc) return rc;
    Carve w(ctx->ws);
    uint64_t *split = w.take<uint64_t>(ntiles + 1);
    const crdt_tuples empty{nullptr, nullptr, nullptr, nullptr};
    const crdt_tuples &a = na ? A : empty, &b = nb ? B : empty;
    k_or_split<<<(unsigned)((ntiles + 1 + 15) / 16), 256, 0, ctx->stream>>>(a, b, na, nb, ntiles, split);
    k_tmerge<512><<<(unsigned)ntiles, 512, 0, ctx->stream>>>(a, b, na, nb, split, O);
    return check_launch(ctx);
}

// Adjacent pairs out of (key, ts, rep) order.
__global__ void k_count_unsorted(crdt_tuples T, size_t n, unsigned long long *bad) {
    unsigned long long c = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i + 1 < n; i += (size_t)gridDim.x * 256)
        c += tag_le(gtag(T, i), gtag(T, i + 1)) ? 0 : 1;
    if (c) atomicAdd(bad, c);
}

static bool tuples_ok(const crdt_tuples *t) { return t && t->key && t->ts && t->rep && t->tomb; }

// The write passes stage every field by LDS-DMA from element offsets: key /
// ts / rep must be naturally aligned (any element offset of an allocation is).
static bool dma_aligned(const crdt_tuples &t) {
    return !((((uintptr_t)t.key | (uintptr_t)t.ts) & 7) | ((uintptr_t)t.rep & 3));
}

template <bool LWW>
static int set_merge(crdt_ctx *ctx, const crdt_tuples *a, size_t na, const crdt_tuples *b, size_t nb,
                     crdt_tuples *out, uint64_t *out_count) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!out_count || !tuples_ok(out)) return CRDT_E_INVAL;
    if ((na && !tuples_ok(a)) || (nb && !tuples_ok(b))) return CRDT_E_INVAL;
    if ((na && !dma_aligned(*a)) || (nb && !dma_aligned(*b))) return CRDT_E_INVAL;
    if (na + nb == 0) {
        hipError_t e = hipMemsetAsync(out_count, 0, sizeof(uint64_t), ctx->stream);
        return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
    }
    crdt_tuples empty{nullptr, nullptr, nullptr, nullptr};
    const crdt_tuples &A = na ? *a : empty;
    const crdt_tuples &B = nb ? *b : empty;
    return LWW ? lww_merge_keyruns(ctx, A, na, B, nb, *out, out_count)
               : orset_merge_twopass(ctx, A, na, B, nb, *out, out_count);
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_lww_merge(crdt_ctx *ctx, const crdt_tuples *a, size_t na, const crdt_tuples *b, size_t nb,
                              crdt_tuples *out, uint64_t *out_count_dev) {
    return set_merge<true>(ctx, a, na, b, nb, out, out_count_dev);
}

extern "C" int crdt_orset_merge(crdt_ctx *ctx, const crdt_tuples *a, size_t na, const crdt_tuples *b, size_t nb,
                                crdt_tuples *out, uint64_t *out_count_dev) {
    return set_merge<false>(ctx, a, na, b, nb, out, out_count_dev);
}

extern "C" int crdt_tuples_merge(crdt_ctx *ctx, const crdt_tuples *a, size_t na, const crdt_tuples *b, size_t nb,
                                 const crdt_tuples *out) {
    int rc = bind(ctx);
    if (rc) return rc;
    if ((na + nb && !tuples_ok(out)) || (na && !tuples_ok(a)) || (nb && !tuples_ok(b))) return CRDT_E_INVAL;
    const crdt_tuples empty{nullptr, nullptr, nullptr, nullptr};
    return tuples_merge_stable(ctx, na ? *a : empty, na, nb ? *b : empty, nb, na + nb ? *out : empty);
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
