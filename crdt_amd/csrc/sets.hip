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
//   2. k_set_merge: a persistent grid of ND data waves + 1 control wave.
//      The control wave claims tiles one iteration ahead (one atomic), loads
//      their splits, warms the cache with the next tile's lines, publishes each tile's count and runs the
//      decoupled look-back (256 predecessors per round trip; {flag, count}
//      8-byte agent-scope atomics: the data is the flag) with an iteration
//      of slack: the data waves hold a tile's staged output in registers and
//      write it out after the NEXT tile's loads.  Per tile the data waves
//      find each lane's merge-path split in LDS and merge ITEMS elements
//      keeping the merged tags in registers, derive emit flags / LWW winners /
//      OR-Set tomb-ORs from registers (runs that cross a lane or tile edge
//      continue through the merged-order index in LDS and then global
//      memory: rare), stage in LDS and read back in coalesced copy-out order.
#include <algorithm>

#include "lookback.hpp"
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

// ---------------------------------------------------------------- partition
// split[t] = number of A elements among the first min(t*TILE, n) merged
// elements.  P(i) = A[i] <= B[d-1-i] is true for i < answer, false after.
// (One diagonal per wave with 64 probes per round was 2x slower: four times
// the waves, and a key tie in any lane stalls the whole wave's round.)
// It also zeroes the merge's look-back status words and tile counter
// (zero_words of them): one launch instead of a memset plus a launch.
__global__ __launch_bounds__(256) void k_partition(crdt_tuples A, crdt_tuples B, size_t na, size_t nb,
                                                   size_t tile, size_t ntiles, uint64_t *__restrict__ split,
                                                   uint64_t *__restrict__ zero, size_t zero_words) {
    for (size_t z = (size_t)blockIdx.x * 256 + threadIdx.x; z < zero_words; z += (size_t)gridDim.x * 256) zero[z] = 0;
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

// look-back helpers (wave_look_back, status flags): lookback.hpp

// ---------------------------------------------------------------- tile merge
// Workgroup of k_set_merge: warp-specialised, 8 waves.
//   waves 0..ND-1 : data waves -- merge a tile that is already in LDS
//   wave  ND      : loader    -- claims tiles, loads their split and edge
//                               candidates, DMAs the tile into the free LDS
//                               buffer (global_load_lds, no registers)
//   wave  ND+1    : look-back -- turns each tile's count into its offset
// 8 waves of <= 128 VGPRs pack exactly two workgroups per CU (2 waves per
// SIMD each); two double-buffered tiles per workgroup fill the 160 KB LDS.
constexpr int ND = 6;                  // data waves
constexpr int NDL = ND * 64;           // data lanes
constexpr int SET_BLOCK = NDL + 128;
constexpr int SET_ITEMS = 4;           // merged elements per data lane
constexpr int TILE = NDL * SET_ITEMS;  // 1536 merged elements per tile

// A wave-uniform 64-bit LDS value in scalar registers.
__device__ __forceinline__ uint64_t uread64(const uint64_t &v) {
    const uint64_t x = v;
    return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
           __builtin_amdgcn_readfirstlane((uint32_t)x);
}

// One tile's bounds in A and B, from the partition.
struct TileBounds {
    size_t d0, i0, i1, j0, j1;
    int len, na_t, nb_t;
};
__device__ __forceinline__ TileBounds tile_bounds(uint32_t t, uint64_t i0, uint64_t i1, size_t n) {
    TileBounds b;
    b.d0 = (size_t)t * TILE;
    const size_t d1 = b.d0 + TILE < n ? b.d0 + TILE : n;
    b.i0 = i0;
    b.i1 = i1;
    b.j0 = b.d0 - i0;
    b.j1 = d1 - i1;
    b.len = (int)(d1 - b.d0);
    b.na_t = (int)(i1 - i0);
    b.nb_t = b.len - b.na_t;
    return b;
}

// One LDS tile buffer.  Each array holds A's part of the tile, then B's,
// each DMA'd in 16-byte chunks from its 16-byte aligned-down start, so a
// part's element 0 sits at byte offset o[A|B] of its array (its global
// misalignment past a 16-byte boundary); the chunks never overlap.  After
// the merge the arrays are reused, from 0, as the output staging area.
struct TileBuf {
    alignas(16) uint64_t key[TILE + 8];
    alignas(16) uint64_t ts[TILE + 8];
    alignas(16) uint32_t rep[TILE + 16];
    alignas(16) uint8_t tomb[TILE + 64];
    uint64_t ek[4], et[4];             // edge candidates A[i0-1], B[j0-1], A[i1], B[j1]
    uint32_t er[4], ev[4];
    uint32_t tile;
    uint32_t ok[2], ot[2], orr[2], om[2];   // byte offsets of A's / B's element 0
    uint64_t i0, i1;                   // the tile's split
};

// LDS hand-off between waves of one workgroup: payload stores, then the
// tag (LDS accesses of one wave complete in order); the reader polls the tag
// and reads the payload after it.
__device__ __forceinline__ void lds_publish(uint32_t *tag, uint32_t v) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __hip_atomic_store(tag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_wait(const uint32_t *tag, uint32_t v) {
    while (__hip_atomic_load(tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != v) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}

// Barrier among the ND data waves only (the loader and look-back waves run
// on): an LDS arrival counter; gen advances by ND per use.
__device__ __forceinline__ void data_barrier(uint32_t *cnt, uint32_t &gen, int spin = 0) {
    gen += ND;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // this wave's LDS accesses are done
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (spin) {
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < gen) {}
    } else {
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < gen) __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");
}

// Loader wave: DMA elements src[0, cnt) into the LDS array `dst` at the
// 16-byte aligned byte offset `at`, in 16-byte chunks from src's aligned-down
// address (1 KB per wave instruction, no registers held; the last chunk reads
// at most 15 bytes past the part, inside the same 16-byte block, never past a
// page).  Returns the byte offset of element 0; *at advances past the chunks.
template <typename E>
__device__ __forceinline__ uint32_t dma_part(const E *src, uint32_t cnt, void *dst, uint32_t *at, int lane) {
    const uint32_t sh = (uint32_t)((uintptr_t)src & 15);
    const uint32_t o = *at + sh;
    if (cnt == 0) return o;
    const uint32_t bytes = (sh + cnt * (uint32_t)sizeof(E) + 15) & ~15u;
    const char *g = (const char *)src - sh;
    char *d = (char *)dst + *at;
    for (uint32_t off = 0; off < bytes; off += 1024) {
        if (off + 16u * (uint32_t)lane < bytes)
            __builtin_amdgcn_global_load_lds((const void *)(g + off + 16 * lane),
                                             (__attribute__((address_space(3))) void *)(d + off), 16, 0, 0);
    }
    *at += bytes;
    return o;
}

// Persistent, warp-specialised merge.  For iteration k of a workgroup
// (tile t_k, LDS buffer k & 1):
//   loader     : claim t_k (one atomic), load its split, wait until the data
//                waves are done with buffer k & 1 (iteration k-2), hand t_k to
//                the look-back wave, DMA the tile and its edge candidates in,
//                publish it
//   look-back  : look back for t_k's offset as soon as it is claimed (only
//                the predecessors' counts are needed), then wait for t_k's
//                count and publish its inclusive prefix and its offset
//   data waves : merge t_k from LDS | publish its count (globally: the
//                look-back's aggregate; and to the look-back wave) | write
//                t_{k-2}'s output, held in registers, at its offset | resolve
//                tombs, stage in LDS, read back into the hold registers |
//                release the buffer
// Only the data waves synchronise with each other (LDS counter); the other
// two roles communicate by tagged LDS words.  Loads of t_{k+1} overlap the
// merge of t_k, and a late look-back delays only this workgroup's copy-out,
// two iterations later, never the next tile's count, so look-back latency
// does not chain across the grid.  Tiles are claimed at the loader's pace,
// which tracks the data waves' (two buffers), so claim order tracks
// processing order; a workgroup that is not resident owns no tile, so every
// look-back makes progress.
template <int MODE>
__global__ __launch_bounds__(SET_BLOCK, 2 * SET_BLOCK / 256) void k_set_merge(
    crdt_tuples A, crdt_tuples B, size_t na, size_t nb, const uint64_t *__restrict__ split, uint64_t *status,
    uint32_t *tile_ctr, uint32_t *err, uint32_t ntiles, crdt_tuples out, uint64_t *__restrict__ out_count,
    uint64_t *stamps, int diag, int knobs) {
    __shared__ TileBuf buf[2];
    __shared__ uint16_t smi[TILE];
    __shared__ uint32_t s_wsum[ND];
    __shared__ uint64_t s_wf_k[ND], s_wf_t[ND], s_wl_k[ND], s_wl_t[ND];   // first / last item of each
    __shared__ uint32_t s_wf_r[ND], s_wl_r[ND];                            //   data wave
    __shared__ uint32_t s_dbar;                      // data-wave soft barrier counter
    __shared__ uint32_t s_load_tag[2];               // loader -> data: buffer holds iteration k (k+1)
    __shared__ uint32_t s_free_tag[2];               // data -> loader: iteration k done with it (k+1)
    // rings of 4 (slot k & 3): data waves lag the look-back by up to two
    // iterations (they write tile k-2 out in iteration k)
    __shared__ uint32_t s_lb_tile[4], s_lb_tag[4];   // loader -> look-back: tile of iteration k
    __shared__ uint32_t s_tot[4], s_tot_tag[4];      // data -> look-back: count of iteration k
    __shared__ uint64_t s_off[4];                    // look-back -> data: offset of iteration k
    __shared__ uint32_t s_off_tag[4];

    const int tid = threadIdx.x, lane = tid & 63;
    const size_t n = na + nb;
    const int role = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: separate loops
    // Diagnostic build only (stamps != nullptr): s_memtime at phase
    // boundaries of each tile, written to a buffer nothing else reads.
#define STAMP(t, i) \
    do { if (stamps && tid == 0) stamps[(size_t)(t) * 16 + (i)] = __builtin_amdgcn_s_memtime(); } while (0)
#define WSTAMP(t, i, v) \
    do { if (stamps && lane == 0) stamps[(size_t)(t) * 16 + (i)] = (v); } while (0)

    if (tid < 2) {
        s_load_tag[tid] = 0;
        s_free_tag[tid] = 0;
    }
    if (tid < 4) {
        s_lb_tag[tid] = 0;
        s_tot_tag[tid] = 0;
        s_off_tag[tid] = 0;
    }
    if (tid == 0) s_dbar = 0;
    __syncthreads();                          // the only workgroup-wide barrier

    if (role >= ND && (knobs & 1)) __builtin_amdgcn_s_setprio(2);   // control waves issue first
    if (role == ND) {
        // ============================================================ loader wave
        for (uint32_t k = 0;; ++k) {
            const int bi = k & 1;
            uint32_t a = 0;
            if (lane == 0) a = atomicAdd(tile_ctr, 1u);
            const uint32_t t = __shfl(a, 0);
            uint64_t sp = 0;
            if (lane < 2 && t < ntiles) sp = split[t + lane];
            const uint64_t i0 = __shfl(sp, 0), i1 = __shfl(sp, 1);
            if (k >= 2) lds_wait(&s_free_tag[bi], k - 1);     // iteration k-2 released the buffer
            if (lane == 0) {                  // the look-back can start now (its slot's last
                s_lb_tile[k & 3] = t;         // reader, iteration k-4, is done: the data waves
                lds_publish(&s_lb_tag[k & 3], k + 1);   // wrote k-4 out in iteration k-2)
            }
            TileBuf &tb = buf[bi];
            if (t < ntiles) {
                WSTAMP(t, 12, __builtin_amdgcn_s_memtime());
                const TileBounds b = tile_bounds(t, i0, i1, n);
                uint32_t ak = 0, at = 0, ar = 0, am = 0;
                const uint32_t okA = dma_part(A.key + b.i0, b.na_t, tb.key, &ak, lane);
                const uint32_t okB = dma_part(B.key + b.j0, b.nb_t, tb.key, &ak, lane);
                const uint32_t otA = dma_part(A.ts + b.i0, b.na_t, tb.ts, &at, lane);
                const uint32_t otB = dma_part(B.ts + b.j0, b.nb_t, tb.ts, &at, lane);
                const uint32_t orA = dma_part(A.rep + b.i0, b.na_t, tb.rep, &ar, lane);
                const uint32_t orB = dma_part(B.rep + b.j0, b.nb_t, tb.rep, &ar, lane);
                const uint32_t omA = dma_part(A.tomb + b.i0, b.na_t, tb.tomb, &am, lane);
                const uint32_t omB = dma_part(B.tomb + b.j0, b.nb_t, tb.tomb, &am, lane);
                if (lane < 4) {               // merged neighbours' candidates
                    const bool isA = (lane & 1) == 0;
                    const size_t g = lane == 0 ? b.i0 - 1 : lane == 1 ? b.j0 - 1 : lane == 2 ? b.i1 : b.j1;
                    const uint32_t ev = lane == 0 ? b.i0 > 0 : lane == 1 ? b.j0 > 0 : lane == 2 ? b.i1 < na : b.j1 < nb;
                    uint64_t ek = 0, et = 0;
                    uint32_t er = 0;
                    if (ev) {
                        ek = (isA ? A.key : B.key)[g];
                        et = (isA ? A.ts : B.ts)[g];
                        er = (isA ? A.rep : B.rep)[g];
                    }
                    tb.ek[lane] = ek;
                    tb.et[lane] = et;
                    tb.er[lane] = er;
                    tb.ev[lane] = ev;
                }
                if (lane == 0) {
                    tb.ok[0] = okA;
                    tb.ok[1] = okB;
                    tb.ot[0] = otA;
                    tb.ot[1] = otB;
                    tb.orr[0] = orA;
                    tb.orr[1] = orB;
                    tb.om[0] = omA;
                    tb.om[1] = omB;
                    tb.i0 = i0;
                    tb.i1 = i1;
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the DMA has landed in LDS
                WSTAMP(t, 13, __builtin_amdgcn_s_memtime());
            }
            if (lane == 0) {
                tb.tile = t;
                lds_publish(&s_load_tag[bi], k + 1);
            }
            if (t >= ntiles) break;
        }
        return;
    }

    if (role == ND + 1) {
        // ============================================================ look-back wave
        // Looks back as soon as the loader has claimed the tile (it needs
        // only the predecessors' counts), then waits for the tile's own count
        // to publish its inclusive prefix.
        for (uint32_t k = 0;; ++k) {
            const int si = k & 3;
            lds_wait(&s_lb_tag[si], k + 1);
            const uint32_t t = __builtin_amdgcn_readfirstlane(s_lb_tile[si]);
            if (t >= ntiles) break;
            uint64_t P = 0;
            uint32_t nsp = 0, nrd = 0;
            WSTAMP(t, 8, __builtin_amdgcn_s_memtime());
            if (diag) P = (uint64_t)t * TILE;  // timing diagnostic only: no look-back, scrambled output
            else if (t > 0) P = wave_look_back(status, t, err, &nsp, &nrd);
            WSTAMP(t, 9, __builtin_amdgcn_s_memtime());
            WSTAMP(t, 10, nsp);
            WSTAMP(t, 11, nrd);
            lds_wait(&s_tot_tag[si], k + 1);
            const uint32_t total = s_tot[si];
            if (lane == 0) {
                if (t > 0 && !diag) st_status(status + t, kFlagInc | (P + total));
                if (t == ntiles - 1) *out_count = P + total;
                s_off[si] = P;
                lds_publish(&s_off_tag[si], k + 1);
            }
        }
        return;
    }

    // ================================================================ data waves
    // the output of t_{k-1} (h1) and t_{k-2} (h2), held in registers in
    // copy-out order until its offset is known; t_{k-2}'s is written out in
    // iteration k, so a look-back has two iterations of slack
    uint64_t h1k[SET_ITEMS], h1t[SET_ITEMS], h2k[SET_ITEMS], h2t[SET_ITEMS];
    uint32_t h1r[SET_ITEMS], h2r[SET_ITEMS];
    uint8_t h1b[SET_ITEMS], h2b[SET_ITEMS];
    uint32_t held1 = 0, held2 = 0;            // their counts (0: nothing held)
    uint32_t dgen = 0;                        // data-wave soft-barrier generation
    uint32_t k = 0;
    for (;; ++k) {
        // Opaque per-iteration copy of the lane id: keeps LICM from hoisting
        // lane-dependent address arithmetic out of the loop.
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int lane = tid & 63;
        const int bi = k & 1;
        TileBuf &T = buf[bi];
        lds_wait(&s_load_tag[bi], k + 1);
        const uint32_t cur = __builtin_amdgcn_readfirstlane(T.tile);
        if (cur >= ntiles) break;
        STAMP(cur, 0);
        const TileBounds b = tile_bounds(cur, uread64(T.i0), uread64(T.i1), n);
        // tile element x: A part (x < na_t) through *A, B part through *B
        const uint64_t *KA = (const uint64_t *)((const char *)T.key + __builtin_amdgcn_readfirstlane(T.ok[0]));
        const uint64_t *KB = (const uint64_t *)((const char *)T.key + __builtin_amdgcn_readfirstlane(T.ok[1])) - b.na_t;
        const uint64_t *TA = (const uint64_t *)((const char *)T.ts + __builtin_amdgcn_readfirstlane(T.ot[0]));
        const uint64_t *TB = (const uint64_t *)((const char *)T.ts + __builtin_amdgcn_readfirstlane(T.ot[1])) - b.na_t;
        const uint32_t *RA = (const uint32_t *)((const char *)T.rep + __builtin_amdgcn_readfirstlane(T.orr[0]));
        const uint32_t *RB = (const uint32_t *)((const char *)T.rep + __builtin_amdgcn_readfirstlane(T.orr[1])) - b.na_t;
        const uint8_t *tombA = T.tomb + __builtin_amdgcn_readfirstlane(T.om[0]);
        const uint8_t *tombB = T.tomb + __builtin_amdgcn_readfirstlane(T.om[1]) - b.na_t;
#define LTAG_A(x) Tag{KA[(x)], TA[(x)], RA[(x)]}
#define LTAG_B(x) Tag{KB[(x)], TB[(x)], RB[(x)]}
#define LTAG(x) ((x) < b.na_t ? LTAG_A(x) : LTAG_B(x))
#define LTOMB(x) ((x) < b.na_t ? tombA[(x)] : tombB[(x)])

        // ---- merge path.  This lane owns merged positions [dd, dd + nv); the
        // merged tags stay in registers, the two heads are the only LDS reads
        // per serial step.  (The phase is bound by LDS throughput, not by
        // latency: an 8-ary search with 7 parallel probes per step was 1.5x
        // slower than this binary search.  Writing the output straight from
        // these registers, without the LDS staging below, was 1.2x slower:
        // per-lane runs make each store instruction touch many lines.)
        Tag it[SET_ITEMS];
        uint8_t tbm[SET_ITEMS];
        const int dd = tid * SET_ITEMS < b.len ? tid * SET_ITEMS : b.len;
        const int nv = b.len - dd < SET_ITEMS ? b.len - dd : SET_ITEMS;
        if (diag == 2) {
            // timing diagnostic only (the loader pipeline's ceiling): the data
            // waves release each tile unmerged and write nothing
            data_barrier(&s_dbar, dgen, knobs & 2);
            if (tid == 0) {
                st_status(status + cur, cur == 0 ? kFlagInc : kFlagAgg);
                s_tot[k & 3] = 0;
                lds_publish(&s_tot_tag[k & 3], k + 1);
                lds_publish(&s_free_tag[bi], k + 1);
            }
            continue;
        }
        {
            int lo = dd > b.nb_t ? dd - b.nb_t : 0, hi = dd < b.na_t ? dd : b.na_t;
            const int jb = b.na_t + dd - 1;   // B index paired with A index i: jb - i
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                const uint64_t ka = KA[mid], kb = KB[jb - mid];
                const bool le = ka != kb ? ka < kb : tag_le(LTAG_A(mid), LTAG_B(jb - mid));
                if (le) lo = mid + 1;
                else hi = mid;
            }
            int ia = lo, ib = b.na_t + dd - lo;               // tile indices of the heads
            const int ie = b.na_t, je = b.len;
            Tag ha = ia < ie ? LTAG_A(ia) : Tag{0, 0, 0};
            Tag hb_ = ib < je ? LTAG_B(ib) : Tag{0, 0, 0};
#pragma unroll
            for (int u = 0; u < SET_ITEMS; ++u) {
                if (u < nv) {
                    const bool takeA = ib >= je || (ia < ie && tag_le(ha, hb_));
                    const int src = takeA ? ia : ib;
                    it[u] = tag_sel(takeA, ha, hb_);
                    smi[dd + u] = (uint16_t)src;
                    tbm[u] = takeA ? tombA[src] : tombB[src];
                    if (takeA) {
                        ++ia;
                        if (ia < ie) ha = LTAG_A(ia);
                    } else {
                        ++ib;
                        if (ib < je) hb_ = LTAG_B(ib);
                    }
                } else {
                    it[u] = Tag{0, 0, 0};
                    tbm[u] = 0;
                }
            }
        }
        // wave-edge items for the neighbour exchange (lane 63's last item is
        // real whenever a next wave has items)
        const int w = tid >> 6;
        if (lane == 0) {
            s_wf_k[w] = it[0].k;
            s_wf_t[w] = it[0].t;
            s_wf_r[w] = it[0].r;
        }
        if (lane == 63) {
            s_wl_k[w] = it[SET_ITEMS - 1].k;
            s_wl_t[w] = it[SET_ITEMS - 1].t;
            s_wl_r[w] = it[SET_ITEMS - 1].r;
        }
        data_barrier(&s_dbar, dgen, knobs & 2);                                       // smi, wave edges
        STAMP(cur, 1);

        // ---- merged neighbours of this lane's run (lane +-1 by shuffles),
        // emit flags, block count
        const Tag up{(uint64_t)__shfl_up((unsigned long long)it[SET_ITEMS - 1].k, 1, 64),
                     (uint64_t)__shfl_up((unsigned long long)it[SET_ITEMS - 1].t, 1, 64),
                     (uint32_t)__shfl_up((int)it[SET_ITEMS - 1].r, 1, 64)};
        const Tag dn{(uint64_t)__shfl_down((unsigned long long)it[0].k, 1, 64),
                     (uint64_t)__shfl_down((unsigned long long)it[0].t, 1, 64),
                     (uint32_t)__shfl_down((int)it[0].r, 1, 64)};
        bool hp = false, hn = false;
        Tag pv{0, 0, 0}, nx{0, 0, 0};
        if (nv > 0) {
            if (dd > 0) {
                pv = lane > 0 ? up : Tag{s_wl_k[w - 1], s_wl_t[w - 1], s_wl_r[w - 1]};
                hp = true;
            } else {                          // d0-1 = the later of A[i0-1], B[j0-1] (A first on equal)
                const Tag a{T.ek[0], T.et[0], T.er[0]}, bb{T.ek[1], T.et[1], T.er[1]};
                const bool va = T.ev[0] != 0, vb = T.ev[1] != 0;
                hp = va || vb;
                pv = tag_sel(va && vb ? tag_le(a, bb) : !va, bb, a);
            }
            if (dd + nv < b.len) {
                nx = lane < 63 ? dn : Tag{s_wf_k[w + 1], s_wf_t[w + 1], s_wf_r[w + 1]};
                hn = true;
            } else {                          // d1 = the earlier of A[i1], B[j1]
                const Tag a{T.ek[2], T.et[2], T.er[2]}, bb{T.ek[3], T.et[3], T.er[3]};
                const bool va = T.ev[2] != 0, vb = T.ev[3] != 0;
                hn = va || vb;
                nx = tag_sel(va && vb ? !tag_le(a, bb) : !va, bb, a);
            }
        }
        // OR: first of a tag run; LWW: last of a key run
        uint32_t emask = 0;
#pragma unroll
        for (int u = 0; u < SET_ITEMS; ++u) {
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
        uint32_t woff;
        {
            uint32_t x = (uint32_t)__popc(emask);
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d, 64);
                if (lane >= d) x += y;
            }
            woff = x - (uint32_t)__popc(emask);
            if (lane == 63) s_wsum[w] = x;
        }
        data_barrier(&s_dbar, dgen, knobs & 2);                                       // wave sums
        STAMP(cur, 2);
        uint32_t total = 0, local_off = woff;
#pragma unroll
        for (int q = 0; q < ND; ++q) {
            const uint32_t ws = s_wsum[q];
            total += ws;
            local_off += (q < w) ? ws : 0;
        }
        // publish t_k's count (the look-back's aggregate) right away, and
        // hand it to the look-back wave for t_k's own offset
        if (tid == 0) {
            st_status(status + cur, (cur == 0 ? kFlagInc : kFlagAgg) | total);
            s_tot[k & 3] = total;
            lds_publish(&s_tot_tag[k & 3], k + 1);
        }
        // ---- t_{k-2} out at its offset (coalesced rows)
        if (held2) {
            lds_wait(&s_off_tag[(k - 2) & 3], k - 1);
            const uint64_t P = uread64(s_off[(k - 2) & 3]);
#pragma unroll
            for (int u = 0; u < SET_ITEMS; ++u) {
                const int x = u * NDL + tid;
                if (x < (int)held2) {
                    out.key[P + x] = h2k[u];
                    out.ts[P + x] = h2t[u];
                    out.rep[P + x] = h2r[u];
                    out.tomb[P + x] = h2b[u];
                }
            }
        }
        STAMP(cur, 3);

        // ---- output tombs (runs crossing this lane's edge are rare)
        uint8_t ot[SET_ITEMS];
        if constexpr (MODE == SET_OR) {
            // tomb-OR over the run that starts at each emitter (backward sweep)
            uint8_t carry = 0;
            Tag last = it[0];                                       // it[nv-1] without a runtime index
#pragma unroll
            for (int u = 1; u < SET_ITEMS; ++u)
                if (u < nv) last = it[u];
            if (nv > 0 && hn && tag_eq(nx, last)) {                 // run continues past this lane
                const Tag tg = last;
                int m = dd + nv;
                while (m < b.len && tag_eq(LTAG(smi[m]), tg)) {
                    carry |= LTOMB(smi[m]);
                    ++m;
                }
                if (m == b.len) {
                    for (size_t x = b.i1; x < na && tag_eq(gtag(A, x), tg); ++x) carry |= A.tomb[x];
                    for (size_t y = b.j1; y < nb && tag_eq(gtag(B, y), tg); ++y) carry |= B.tomb[y];
                }
            }
#pragma unroll
            for (int u = SET_ITEMS - 1; u >= 0; --u) {
                if (u < nv) {
                    const bool cont = (u + 1 < nv) ? tag_eq(it[u + 1], it[u]) : true;
                    const uint8_t c = (u + 1 < nv) ? (cont ? ot[u + 1] : (uint8_t)0) : carry;
                    ot[u] = (uint8_t)(tbm[u] | c);
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
                first = (dd > 0) ? LTOMB(smi[m]) : 0;
                if (dd == 0 || m == 0) {                             // ... or before the tile
                    if (b.i0 > 0 && tag_eq(gtag(A, b.i0 - 1), tg)) {
                        size_t x = b.i0 - 1;
                        while (x > 0 && tag_eq(gtag(A, x - 1), tg)) --x;
                        first = A.tomb[x];
                    } else if (b.j0 > 0 && tag_eq(gtag(B, b.j0 - 1), tg)) {
                        size_t y = b.j0 - 1;
                        while (y > 0 && tag_eq(gtag(B, y - 1), tg)) --y;
                        first = B.tomb[y];
                    }
                }
            } else {
                first = tbm[0];
            }
#pragma unroll
            for (int u = 0; u < SET_ITEMS; ++u) {
                if (u == 0) ot[0] = first;
                else ot[u] = (u < nv && tag_eq(it[u - 1], it[u])) ? ot[u - 1] : tbm[u];
            }
        }
#undef LTAG
#undef LTAG_A
#undef LTAG_B
#undef LTOMB
        data_barrier(&s_dbar, dgen, knobs & 2);                                       // inputs dead

        // ---- stage t_k's output in this buffer at its local offsets
        {
            uint32_t o = local_off;
#pragma unroll
            for (int u = 0; u < SET_ITEMS; ++u) {
                if (emask & (1u << u)) {
                    T.key[o] = it[u].k;
                    T.ts[o] = it[u].t;
                    T.rep[o] = it[u].r;
                    T.tomb[o] = ot[u];
                    ++o;
                }
            }
        }
        data_barrier(&s_dbar, dgen, knobs & 2);                                       // staged
        STAMP(cur, 4);
        // ---- hold it in registers in copy-out order (written out next iteration)
#pragma unroll
        for (int u = 0; u < SET_ITEMS; ++u) {
            h2k[u] = h1k[u];
            h2t[u] = h1t[u];
            h2r[u] = h1r[u];
            h2b[u] = h1b[u];
            const int x = u * NDL + tid;
            if (x < (int)total) {
                h1k[u] = T.key[x];
                h1t[u] = T.ts[x];
                h1r[u] = T.rep[x];
                h1b[u] = T.tomb[x];
            }
        }
        held2 = held1;
        held1 = total;
        data_barrier(&s_dbar, dgen, knobs & 2);                                       // staged copy read
        if (tid == 0) lds_publish(&s_free_tag[bi], k + 1);                 // the loader may refill it
        STAMP(cur, 5);
    }
    // the last two tiles' output (iterations k-2 and k-1)
    if (held2) {
        lds_wait(&s_off_tag[(k - 2) & 3], k - 1);
        const uint64_t P = uread64(s_off[(k - 2) & 3]);
#pragma unroll
        for (int u = 0; u < SET_ITEMS; ++u) {
            const int x = u * NDL + tid;
            if (x < (int)held2) {
                out.key[P + x] = h2k[u];
                out.ts[P + x] = h2t[u];
                out.rep[P + x] = h2r[u];
                out.tomb[P + x] = h2b[u];
            }
        }
    }
    if (held1) {
        lds_wait(&s_off_tag[(k - 1) & 3], k);
        const uint64_t P = uread64(s_off[(k - 1) & 3]);
#pragma unroll
        for (int u = 0; u < SET_ITEMS; ++u) {
            const int x = u * NDL + tid;
            if (x < (int)held1) {
                out.key[P + x] = h1k[u];
                out.ts[P + x] = h1t[u];
                out.rep[P + x] = h1r[u];
                out.tomb[P + x] = h1b[u];
            }
        }
    }
#undef STAMP
#undef WSTAMP
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
//   k_lww_split : merge-path splits of 4096-item tiles over the keys
//                 (16-lane 16-ary searches, four diagonals per wave);
//   k_lww_count : per tile, the keys merged in LDS (512 threads x 8 items):
//                 bitmap `isa` (merge item is an A element) and `emit` (its
//                 key differs from the next merged key: the last element of
//                 the key's merged run -- B's run end when B holds the key,
//                 else A's), 512 B per tile, and the tile's emit count;
//   scan of the counts -> each tile's output offset, *out_count;
//   k_lww_write : per tile, 1024 threads in merge order (wave w: items
//                 64 (w + 16 f) + lane); an item's A / B index and output
//                 rank are prefix popcounts of the bitmaps (mbcnt over
//                 wave-uniform words); each emitting lane loads its run end
//                 and -- for a B run end -- A's element just before it in
//                 merged order (A's run end when it holds the same key),
//                 picks the winner, steps back over equal-tag copies for the
//                 first one's tomb, and stores at its rank (consecutive
//                 across the emitting lanes).
// No cross-workgroup waiting; the key reads are the only full pass.
constexpr int LT = 4096;                 // merge items per LWW tile
constexpr int LCB = 512;                 // count pass threads (8 items each)
constexpr int LNW = LT / 64;             // bitmap words per tile and bitmap

__global__ __launch_bounds__(256) void k_lww_split(const uint64_t *__restrict__ ka, const uint64_t *__restrict__ kb,
                                                   size_t na, size_t nb, size_t ntiles, uint64_t *__restrict__ split) {
    const int lane = threadIdx.x & 63, grp = lane >> 4, gl = lane & 15;
    const size_t t = ((((size_t)blockIdx.x * 256 + threadIdx.x) >> 6) << 2) + (size_t)grp;
    const size_t n = na + nb;
    const size_t d = t * LT < n ? t * LT : n;
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
__device__ __forceinline__ LwwTile lww_tile(const uint64_t *__restrict__ split, uint64_t t, size_t n) {
    LwwTile b;
    const size_t d0 = (size_t)t * LT, d1 = d0 + LT < n ? d0 + LT : n;
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
                                                   uint32_t *__restrict__ tcnt, uint64_t *__restrict__ bits) {
    constexpr int NI = LT / LCB, LPW = 64 / NI;
    __shared__ uint64_t sk[LT];                          // A part, then B part
    __shared__ uint32_t s_w[LCB / 64];
    const uint64_t t = blockIdx.x;
    const LwwTile b = lww_tile(split, t, na + nb);
    uint64_t v[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) {                       // every load issued before the first store
        const uint32_t k = threadIdx.x + (uint32_t)j * LCB;
        v[j] = k < b.na ? ka[b.i0 + k] : k < b.n ? kb[b.j0 + (k - b.na)] : 0;
    }
    // the keys after the tile: the next merged key past its last item
    const bool ha_next = b.i1 < na, hb_next = b.j1 < nb;
    const uint64_t ka_next = ha_next ? ka[b.i1] : 0, kb_next = hb_next ? kb[b.j1] : 0;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
        const uint32_t k = threadIdx.x + (uint32_t)j * LCB;
        if (k < b.n) sk[k] = v[j];
    }
    __syncthreads();
    const uint64_t *SA = sk, *SB = sk + b.na;
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

// exclusive scan of n <= 16k tile counts by one workgroup (a contiguous
// chunk per thread); out[n] = total, also written to *count.  (Chunks held
// in registers: 6.9 / 11.5 µs at 4.9k / 9.8k tiles; 16 coalesced rows per
// wave: 11.9 / 12.0; this loop 5.5 / 11.9.)
__global__ __launch_bounds__(1024) void k_lww_scan(const uint32_t *__restrict__ tcnt, uint32_t n,
                                                   uint64_t *__restrict__ out, uint64_t *__restrict__ count) {
    __shared__ uint64_t s_w[16];
    const uint32_t per = (n + 1023) / 1024;
    const uint32_t b = threadIdx.x * per < n ? threadIdx.x * per : n;
    const uint32_t e = b + per < n ? b + per : n;
    uint64_t sum = 0;
    for (uint32_t i = b; i < e; ++i) sum += tcnt[i];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint64_t base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        base += k < w ? s_w[k] : 0;
        tot += s_w[k];
    }
    uint64_t run = base + x - sum;
    for (uint32_t i = b; i < e; ++i) {
        out[i] = run;
        run += tcnt[i];
    }
    if (threadIdx.x == 0) {
        out[n] = tot;
        *count = tot;
    }
}

__global__ void k_lww_total(const uint64_t *__restrict__ ic, uint64_t n, uint64_t *__restrict__ count) { *count = ic[n]; }

// the first element of a side's run of equal tags ending at index w
__device__ __forceinline__ size_t first_copy(const uint64_t *sk, const uint64_t *st, const uint32_t *sr, size_t w,
                                             uint64_t k, uint64_t ts, uint32_t r) {
    while (w > 0 && sk[w - 1] == k && st[w - 1] == ts && sr[w - 1] == r) --w;
    return w;
}

// k_lww_write: one workgroup per HALF tile (2048 merge items, words
// 32 h .. 32 h + 31 of the tile's bitmaps).  The half's A run and B run
// (plus the two A elements and the one B element before them) are staged in
// LDS with coalesced loads -- every field of every input element is read
// once, in order; per-lane gathers of the run ends kept the vector-memory
// address pipe saturated (185 µs, 52 % of wave time in issue stalls; a
// shuffle-window variant 216-224 µs).  Then, per emitting item, X / Y / their
// predecessors come from LDS.
constexpr int LWH = 2048;                // merge items per write workgroup
constexpr int LWT = 512;                 // its threads (4 items each)

// The DMA staging indexes elements from a byte offset: fields naturally aligned.
static inline bool dma_aligned(const crdt_tuples &t) {
    return !((((uintptr_t)t.key | (uintptr_t)t.ts) & 7) | ((uintptr_t)t.rep & 3));
}

// k_lww_count with its keys staged by LDS-DMA (the default; sets.knobs bit 3: register staging)
__global__ __launch_bounds__(LCB) void k_lww_count_dma(const uint64_t *__restrict__ ka, const uint64_t *__restrict__ kb,
                                                   size_t na, size_t nb, const uint64_t *__restrict__ split,
                                                   uint32_t *__restrict__ tcnt, uint64_t *__restrict__ bits) {
    constexpr int NI = LT / LCB, LPW = 64 / NI;
    __shared__ alignas(16) uint64_t sk[LT + 8];          // A's run, then B's, each from its 16-byte aligned-down start
    __shared__ uint32_t s_w[LCB / 64];
    const uint64_t t = blockIdx.x;
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

// WH merge items per workgroup (a 1/P of a tile, P = LT / WH), WT threads
template <bool DMA, int WH = LWH, int WT = LWT>
__global__ __launch_bounds__(WT) void k_lww_write(crdt_tuples A, crdt_tuples B, size_t na, size_t nb,
                                                  const uint64_t *__restrict__ split,
                                                  const uint64_t *__restrict__ bits, const uint64_t *__restrict__ ic,
                                                  crdt_tuples out) {
    constexpr int NWV = WT / 64, FI = (WH / 64) / NWV, CAP = WH + 3, P = LT / WH, WPP = LNW / P;
    static_assert(LNW == 64 && WH * P == LT && FI * NWV * 64 == WH && WH == 4 * WT, "shape");
    // (DMA: each field holds A's run then B's, each from its 16-byte aligned-down
    // start: up to 64 bytes more than the elements)
    __shared__ alignas(16) uint64_t s_key[CAP + 8];
    __shared__ alignas(16) uint64_t s_ts[CAP + 8];
    __shared__ alignas(16) uint32_t s_rep[CAP + 16];
    __shared__ alignas(16) uint8_t s_tomb[CAP + 64];
    const uint64_t t = blockIdx.x / P;
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
    // the half's runs: A [ra, ra + ca), B [rb, rb + cb); staged from ra - 2 / rb - 1
    const uint32_t ha = (uint32_t)__builtin_amdgcn_readlane(pre_a, WPP * h);       // A items before the part
    const uint32_t ha1 = h + 1 == P ? b.na : (uint32_t)__builtin_amdgcn_readlane(pre_a, WPP * (h + 1));  // ... before its end
    const uint32_t d0 = WH * h;
    const uint32_t hn = b.n > d0 ? (b.n - d0 < (uint32_t)WH ? b.n - d0 : (uint32_t)WH) : 0;   // items in the part
    if (hn == 0) return;
    const size_t ra = b.i0 + ha, rb = b.j0 + (d0 - ha);
    const uint32_t ca = ha1 - ha, cb = hn - ca;
    const uint32_t na2 = ca + 2;                         // staged A: ra-2 .. ra+ca-1 (slots 0 .. ca+1)
    const uint32_t nst = na2 + cb + 1;                   // then B: rb-1 .. rb+cb-1
    // DMA: slot x of field f sits at LDS element x + (x < na2 ? oa[f] : ob[f])
    int oa_k = 0, ob_k = 0, oa_t = 0, ob_t = 0, oa_r = 0, ob_r = 0, oa_m = 0, ob_m = 0;
    if (DMA) {
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const size_t ga = ra >= 2 ? ra - 2 : 0, gb = rb >= 1 ? rb - 1 : 0;   // first staged element of each side
        const uint32_t ka = (uint32_t)(ra + ca - ga), kb = (uint32_t)(rb + cb - gb);
        const int sa = (int)(ga - (ra - 2)), sb = (int)(gb - (rb - 1)) + (int)na2;   // their slots
        uint32_t at = 0;
        oa_k = dma_run<uint64_t, NWV>(A.key, ga, ka, s_key, &at, wv, lane) - sa;
        ob_k = dma_run<uint64_t, NWV>(B.key, gb, kb, s_key, &at, wv, lane) - sb;
        at = 0;
        oa_t = dma_run<uint64_t, NWV>(A.ts, ga, ka, s_ts, &at, wv, lane) - sa;
        ob_t = dma_run<uint64_t, NWV>(B.ts, gb, kb, s_ts, &at, wv, lane) - sb;
        at = 0;
        oa_r = dma_run<uint32_t, NWV>(A.rep, ga, ka, s_rep, &at, wv, lane) - sa;
        ob_r = dma_run<uint32_t, NWV>(B.rep, gb, kb, s_rep, &at, wv, lane) - sb;
        at = 0;
        oa_m = dma_run<uint8_t, NWV>(A.tomb, ga, ka, s_tomb, &at, wv, lane) - sa;
        ob_m = dma_run<uint8_t, NWV>(B.tomb, gb, kb, s_tomb, &at, wv, lane) - sb;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA has landed in LDS
    } else {
        uint64_t k[5], ts[5];
        uint32_t r[5];
        uint8_t m[5];
        bool v[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) {                    // every staging load issued before the first store
            const uint32_t x = threadIdx.x + (uint32_t)j * WT;
            const bool on_a = x < na2;
            const size_t g = on_a ? ra - 2 + x : rb - 1 + (x - na2);
            v[j] = x < nst && (on_a ? (ra + x >= 2 && g < na) : (rb + (x - na2) >= 1 && g < nb));
            k[j] = v[j] ? (on_a ? A.key : B.key)[g] : 0;
            ts[j] = v[j] ? (on_a ? A.ts : B.ts)[g] : 0;
            r[j] = v[j] ? (on_a ? A.rep : B.rep)[g] : 0;
            m[j] = v[j] ? (on_a ? A.tomb : B.tomb)[g] : 0;
        }
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const uint32_t x = threadIdx.x + (uint32_t)j * WT;
            if (x < nst) {
                s_key[x] = k[j];
                s_ts[x] = ts[j];
                s_rep[x] = r[j];
                s_tomb[x] = m[j];
            }
        }
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
        out.key[o] = key;
        out.ts[o] = ts;
        out.rep[o] = rep;
        out.tomb[o] = tomb;
    }
}

static int lww_merge_keyruns(crdt_ctx *ctx, const crdt_tuples &A, size_t na, const crdt_tuples &B, size_t nb,
                             const crdt_tuples &O, uint64_t *out_count) {
    const size_t n = na + nb;
    const size_t ntiles = (n + LT - 1) / LT;
    if (ntiles >= 0x7fffffffULL || n >= (1ULL << 62)) return CRDT_E_RANGE;
    const size_t need = Carve::round((ntiles + 1) * 8) + Carve::round(ntiles * 4 + 4) + Carve::round((ntiles + 1) * 8) +
                        Carve::round(ntiles * 2 * LNW * 8) + scan_tmp_bytes(ntiles) + 1024;
    int rc = ws_reserve(ctx, need);
    if (rc) return rc;
    Carve w(ctx->ws);
    uint64_t *split = w.take<uint64_t>(ntiles + 1);
    uint32_t *tcnt = w.take<uint32_t>(ntiles + 1);
    uint64_t *ic = w.take<uint64_t>(ntiles + 1);
    uint64_t *bits = w.take<uint64_t>(ntiles * 2 * LNW);
    void *tmp = w.take<char>(scan_tmp_bytes(ntiles));
    const hipStream_t s = ctx->stream;
    const uint64_t *ka = A.key, *kb = B.key;             // (nullptr for an empty side: never dereferenced)
    k_lww_split<<<(unsigned)((ntiles + 1 + 15) / 16), 256, 0, s>>>(ka, kb, na, nb, ntiles, split);
    if (!(g_sets_knobs & 8) && dma_aligned(A) && dma_aligned(B))   // LDS-DMA staging: 40.0 -> 37.2 us
        k_lww_count_dma<<<(unsigned)ntiles, LCB, 0, s>>>(ka, kb, na, nb, split, tcnt, bits);
    else
        k_lww_count<<<(unsigned)ntiles, LCB, 0, s>>>(ka, kb, na, nb, split, tcnt, bits);
    rc = check_launch(ctx);
    if (rc) return rc;
    if (ntiles <= 16384) {
        k_lww_scan<<<1, 1024, 0, s>>>(tcnt, (uint32_t)ntiles, ic, out_count);
    } else {
        rc = exclusive_scan_u32(ctx, tcnt, ic, ntiles, tmp);
        if (rc) return rc;
        k_lww_total<<<1, 1, 0, s>>>(ic, ntiles, out_count);
    }
    const bool dma = !(g_sets_knobs & 8) && dma_aligned(A) && dma_aligned(B);   // LDS-DMA staging (LWW 181 -> 178 us)
    // workgroups per tile (sets.lww_parts): 1/P of a tile's items, 4 per thread
    const unsigned P = (unsigned)g_lww_parts, g = (unsigned)(P * ntiles);
#define LWW_WRITE(WH)                                                                                  \
    (dma ? k_lww_write<true, WH, WH / 4><<<g, WH / 4, 0, s>>>(A, B, na, nb, split, bits, ic, O)        \
         : k_lww_write<false, WH, WH / 4><<<g, WH / 4, 0, s>>>(A, B, na, nb, split, bits, ic, O))
    if (P == 2) LWW_WRITE(2048);
    else if (P == 8) LWW_WRITE(512);
    else if (P == 16) LWW_WRITE(256);
    else LWW_WRITE(1024);
#undef LWW_WRITE
    return check_launch(ctx);
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
//   scan;
//   k_or_write : per tile (512 threads, wave w: items 64 (w + 8 f) + lane),
//                the tile's A and B runs staged in LDS (coalesced, every
//                field once); an emitting item ORs the tombs of its tag's
//                copies -- forward over A's, then B's from the B position
//                of the item -- and stores at its rank.
constexpr int OT = 2048;                 // merge items per OR tile
constexpr int OCB = 512;                 // count pass threads (4 items each; 256 x 8: 120 us, 1024 x 2: 153 us, against 111)
constexpr int OWT = 512;                 // write pass threads (4 items each)
constexpr int ONW = OT / 64;             // bitmap words per tile and bitmap

__global__ __launch_bounds__(256) void k_or_split(crdt_tuples A, crdt_tuples B, size_t na, size_t nb, size_t ntiles,
                                                  uint64_t *__restrict__ split) {
    const int lane = threadIdx.x & 63, grp = lane >> 4, gl = lane & 15;
    const size_t t = ((((size_t)blockIdx.x * 256 + threadIdx.x) >> 6) << 2) + (size_t)grp;
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
                                                 uint64_t *__restrict__ bits) {
    constexpr int NI = OT / NT, LPW = 64 / NI, CAP = OT + 2;
    // staged: A[i0-1], A part, B[j0-1], B part (slot 0 of each side: the
    // element before the tile, the first item's merged predecessor candidate)
    __shared__ uint64_t sk[CAP], st[CAP];
    __shared__ uint32_t sr[CAP];
    __shared__ uint32_t s_w[NT / 64];
    const uint64_t t = blockIdx.x;
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

// WH merge items per workgroup (a 1/P of a tile, P = OT / WH), WT threads
template <bool DMA, int WH = OT, int WT = OWT>
__global__ __launch_bounds__(WT) void k_or_write(crdt_tuples A, crdt_tuples B, size_t na, size_t nb,
                                                 const uint64_t *__restrict__ split,
                                                 const uint64_t *__restrict__ bits, const uint64_t *__restrict__ ic,
                                                 crdt_tuples out) {
    constexpr int NWV = WT / 64, P = OT / WH, WPP = ONW / P, FI = WPP / NWV, CAP = WH + 2;
    static_assert(FI * NWV == WPP && WH * P == OT && ONW <= 64 && WH == 4 * WT, "shape");
    __shared__ alignas(16) uint64_t s_key[CAP + 8];
    __shared__ alignas(16) uint64_t s_ts[CAP + 8];
    __shared__ alignas(16) uint32_t s_rep[CAP + 16];
    __shared__ alignas(16) uint8_t s_tomb[CAP + 64];
    const uint64_t t = blockIdx.x / P;
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
    // the part's runs: A [pa0, pa0 + ca), B [pb0, pb0 + cb) (tile-relative)
    const uint32_t d0 = WH * h;
    const uint32_t hn = b.n > d0 ? (b.n - d0 < (uint32_t)WH ? b.n - d0 : (uint32_t)WH) : 0;   // items in the part
    if (hn == 0) return;
    const uint32_t pa0 = P == 1 ? 0u : (uint32_t)__builtin_amdgcn_readlane(pre_a, WPP * h);
    const uint32_t pa1 = h + 1 == P ? b.na : (uint32_t)__builtin_amdgcn_readlane(pre_a, WPP * (h + 1));
    const uint32_t ca = pa1 - pa0, cb = hn - ca, pb0 = d0 - pa0;
    const size_t ga = b.i0 + pa0, gb = b.j0 + pb0;       // global index of each run's first element
    // staged: A run (slots 0 .. ca-1), then B run (slots ca ..): every field once
    // (DMA: slot x of field f at LDS element x + (x < ca ? oa[f] : ob[f]))
    int oa_k = 0, ob_k = 0, oa_t = 0, ob_t = 0, oa_r = 0, ob_r = 0, oa_m = 0, ob_m = 0;
    if (DMA) {
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
    } else {
        constexpr int NJ = (WH + WT - 1) / WT;
        uint64_t k[NJ], ts[NJ];
        uint32_t r[NJ];
        uint8_t m[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {                   // every staging load issued before the first store
            const uint32_t x = threadIdx.x + (uint32_t)j * WT;
            const bool on_a = x < ca;
            const size_t g = on_a ? ga + x : gb + (x - ca);
            const bool v = x < hn;
            k[j] = v ? (on_a ? A.key : B.key)[g] : 0;
            ts[j] = v ? (on_a ? A.ts : B.ts)[g] : 0;
            r[j] = v ? (on_a ? A.rep : B.rep)[g] : 0;
            m[j] = v ? (on_a ? A.tomb : B.tomb)[g] : 0;
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const uint32_t x = threadIdx.x + (uint32_t)j * WT;
            if (x < hn) {
                s_key[x] = k[j];
                s_ts[x] = ts[j];
                s_rep[x] = r[j];
                s_tomb[x] = m[j];
            }
        }
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
        out.key[o] = key;
        out.ts[o] = ts;
        out.rep[o] = rep;
        out.tomb[o] = (uint8_t)tomb;
    }
}

static int orset_merge_twopass(crdt_ctx *ctx, const crdt_tuples &A, size_t na, const crdt_tuples &B, size_t nb,
                               const crdt_tuples &O, uint64_t *out_count) {
    const size_t n = na + nb;
    const size_t ntiles = (n + OT - 1) / OT;
    if (ntiles >= 0x7fffffffULL || n >= (1ULL << 62)) return CRDT_E_RANGE;
    const size_t need = Carve::round((ntiles + 1) * 8) + Carve::round(ntiles * 4 + 4) + Carve::round((ntiles + 1) * 8) +
                        Carve::round(ntiles * 2 * ONW * 8) + scan_tmp_bytes(ntiles) + 1024;
    int rc = ws_reserve(ctx, need);
    if (rc) return rc;
    Carve w(ctx->ws);
    uint64_t *split = w.take<uint64_t>(ntiles + 1);
    uint32_t *tcnt = w.take<uint32_t>(ntiles + 1);
    uint64_t *ic = w.take<uint64_t>(ntiles + 1);
    uint64_t *bits = w.take<uint64_t>(ntiles * 2 * ONW);
    void *tmp = w.take<char>(scan_tmp_bytes(ntiles));
    const hipStream_t s = ctx->stream;
    k_or_split<<<(unsigned)((ntiles + 1 + 15) / 16), 256, 0, s>>>(A, B, na, nb, ntiles, split);
    k_or_count<OCB><<<(unsigned)ntiles, OCB, 0, s>>>(A, B, na, nb, split, tcnt, bits);
    rc = check_launch(ctx);
    if (rc) return rc;
    if (ntiles <= 16384) {
        k_lww_scan<<<1, 1024, 0, s>>>(tcnt, (uint32_t)ntiles, ic, out_count);
    } else {
        rc = exclusive_scan_u32(ctx, tcnt, ic, ntiles, tmp);
        if (rc) return rc;
        k_lww_total<<<1, 1, 0, s>>>(ic, ntiles, out_count);
    }
    const bool dma = !(g_sets_knobs & 8) && dma_aligned(A) && dma_aligned(B);   // LDS-DMA staging
    // workgroups per tile (sets.or_parts): 1/P of a tile's items, 4 per thread
    const unsigned P = (unsigned)g_or_parts, g = (unsigned)(P * ntiles);
#define OR_WRITE(WH)                                                                                   \
    (dma ? k_or_write<true, WH, WH / 4><<<g, WH / 4, 0, s>>>(A, B, na, nb, split, bits, ic, O)         \
         : k_or_write<false, WH, WH / 4><<<g, WH / 4, 0, s>>>(A, B, na, nb, split, bits, ic, O))
    if (P == 2) OR_WRITE(1024);
    else if (P == 4) OR_WRITE(512);
    else OR_WRITE(2048);
#undef OR_WRITE
    return check_launch(ctx);
}

size_t g_last_grid = 0;              // diagnostic: persistent grid of the last set merge
int g_last_occ = 0;
uint64_t *g_last_stamps = nullptr;   // diagnostic: stamps of the last set merge (16 per tile)
size_t g_last_stamps_n = 0;

// Adjacent pairs out of (key, ts, rep) order.
__global__ void k_count_unsorted(crdt_tuples T, size_t n, unsigned long long *bad) {
    unsigned long long c = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i + 1 < n; i += (size_t)gridDim.x * 256)
        c += tag_le(gtag(T, i), gtag(T, i + 1)) ? 0 : 1;
    if (c) atomicAdd(bad, c);
}

template <int MODE>
static int set_merge_impl(crdt_ctx *ctx, const crdt_tuples &A, size_t na, const crdt_tuples &B, size_t nb,
                          const crdt_tuples &O, uint64_t *out_count) {
    const size_t n = na + nb;
    const size_t ntiles = (n + TILE - 1) / TILE;
    if (ntiles >= 0x7fffffffULL || n >= (1ULL << 62)) return CRDT_E_RANGE;
    // the LDS-DMA copies key/ts/rep in whole dwords: naturally aligned arrays
    const crdt_tuples *sides[2] = {&A, &B};
    for (const crdt_tuples *t : sides)
        if (((uintptr_t)t->key | (uintptr_t)t->ts) & 7 || (uintptr_t)t->rep & 3) return CRDT_E_INVAL;
    // status words + tile counter first (zeroed by k_partition), split after
    const size_t b_status = Carve::round((ntiles + 4) * sizeof(uint64_t));
    const size_t b_split = Carve::round((ntiles + 1) * sizeof(uint64_t));
    const size_t b_stamps = g_sets_stamps ? Carve::round(ntiles * 16 * sizeof(uint64_t)) : 0;
    int rc = ws_reserve(ctx, b_status + b_split + b_stamps + 768);
    if (rc) return rc;
    Carve w(ctx->ws);
    uint64_t *status = w.take<uint64_t>(ntiles + 4);
    uint32_t *ctr = (uint32_t *)(status + ntiles);        // status[ntiles]: tile counter
    uint32_t *err = ctx->dev_status;                      // CRDT_DEV_LOOKBACK (crdt_ctx_device_status)
    uint64_t *split = w.take<uint64_t>(ntiles + 1);
    uint64_t *stamps = g_sets_stamps ? w.take<uint64_t>(ntiles * 16) : nullptr;
    g_last_stamps = stamps;
    g_last_stamps_n = stamps ? ntiles * 16 : 0;
    const hipStream_t s = ctx->stream;
    hipError_t e = hipSuccess;
    const size_t diags = ntiles + 1;                      // 4 diagonals per wave, 16 per block
    k_partition<<<(unsigned)((diags + 15) / 16), 256, 0, s>>>(A, B, na, nb, TILE, ntiles, split, status,
                                                              b_status / sizeof(uint64_t));
    // persistent grid: CUs x the occupancy query (tiles are claimed
    // dynamically, so a workgroup that is not resident owns nothing and any
    // grid is correct; a spilling build is refused: its scratch traffic
    // would defeat the design)
    static int occ = 0;
    if (occ == 0) {
        hipFuncAttributes fa{};
        e = hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(&k_set_merge<MODE>));
        if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_set_merge<MODE>, SET_BLOCK, 0);
        if (e != hipSuccess) return hip_fail(ctx, e);
        if (fa.localSizeBytes != 0 || occ < 1) {
            occ = 0;
            return CRDT_E_RANGE;
        }
    }
    const int per_cu = g_sets_grid_per_cu > 0 ? g_sets_grid_per_cu : occ;
    const size_t grid = std::min(ntiles, (size_t)ctx->num_cus * (size_t)per_cu);
    g_last_grid = grid;
    g_last_occ = occ;
    k_set_merge<MODE><<<(unsigned)grid, SET_BLOCK, 0, s>>>(A, B, na, nb, split, status, ctr, err, (uint32_t)ntiles,
                                                           O, out_count, stamps, g_sets_diag, g_sets_knobs);
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
    // two-pass merges (sets.knobs bit 2: the persistent tag-merge kernel instead)
    if (!(g_sets_knobs & 4))
        return MODE == SET_LWW ? lww_merge_keyruns(ctx, A, na, B, nb, *out, out_count)
                               : orset_merge_twopass(ctx, A, na, B, nb, *out, out_count);
    return set_merge_impl<MODE>(ctx, A, na, B, nb, *out, out_count);
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

// Diagnostic: copy the phase stamps of the last set merge (16 values per
// tile: 8 data-wave phase stamps, then control-wave stamps / counters) to host memory.  Enabled by crdt_set_option("sets.stamps", 1).
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

// Diagnostic: grid size and occupancy-query answer of the last set merge.
extern "C" int crdt_debug_set_grid(size_t *grid, int *occ) {
    if (!grid || !occ) return CRDT_E_INVAL;
    *grid = g_last_grid;
    *occ = g_last_occ;
    return CRDT_OK;
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
