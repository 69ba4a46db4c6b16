// sort.hip -- device sort of SoA tuples into the set-merge input order
// (unsorted set state; BASELINE configs[3]).
//
// Order: ascending (key, ts, rep, tomb) -- the merge's (key, ts, rep) order,
// with tomb breaking exact tag ties so the result is canonical (independent
// of the input order).
//
// Every field is replaced by its offset from the field's minimum and the
// four offsets are packed into one composite integer of W = bk+bt+br+1 bits
// (tomb lowest, key highest): comparing composites IS comparing tuples.  W is
// usually far below 64 (the D config: 23+20+6+1 = 50 bits), so the sort is a
// plain 64-bit LSD radix sort of the composites; wider data use 2 or 3 words
// per composite (W <= 161).  The last pass decodes the composite straight
// into the SoA output: the sort moves no payload and gathers nothing.
//
// Passes (8-bit digits, P = ceil(W / 8)), reduce-then-scan per pass:
//   k_sort_minmax : field minima/maxima (one read of the input)
//   k_sort_up     : per tile of 4096 composites, its 256 digit counts,
//                   stored digit-major (cnt[d * ntiles + t])
//   k_sort_colscan: one workgroup per digit: exclusive scan of its column
//                   of tile counts, and the digit's total
//   k_sort_pass   : per tile: stable in-tile ranking by wave ballots (a few
//                   barriers per tile), LDS-staged scatter in digit order
//                   (runs of ~16 consecutive outputs per digit) from the
//                   scanned starts (each tile scans the 256 digit totals
//                   itself for the digit bases).
// No tile waits on another: a onesweep-style per-digit decoupled look-back
// (tiles ticketed in order, each digit's lane walking back over published
// counts) was replaced because on MI355X every status word and ticket is a
// memory-side round trip across the 8 XCDs' non-coherent L2s; the extra
// read of the upsweep costs less than those chains.
#include <algorithm>
#include <cstring>

#include "scan.hpp"

namespace crdt {

constexpr int SB = 256;          // threads per sort workgroup
constexpr int SR = 16;           // composites per thread
constexpr int ST = SB * SR;      // 4096 composites per tile
constexpr int SWAVES = SB / 64;

struct SortPlan {
    uint64_t kmin, tmin, rmin;
    uint32_t bk, bt, br;         // bit widths of the key / ts / rep offsets
    uint32_t W, P, words;        // composite bits, passes, 64-bit words
    uint32_t b0;                 // bit offset of the rep field: 1 (tomb) + side bits (0 or 1)
    uint32_t s0;                 // bit of the first digit (0: the whole composite is sorted)
    uint32_t tl, tw;             // LWW key-bucket tables: key bits per bucket table, entry bytes (4 / 8; 0: none)
    uint64_t n1;                 // composites [0, n1) come from in (side 0), [n1, n) from in2 (side 1)
    crdt_tuples in2;
};

// The launch shape a pass was sized for, by value: a
// pass launched from a host-known plan (cached, sampled, planned) compares
// the device plan with it first and, on any difference, raises the plan's
// check word and stores nothing -- its grids, tables, buckets and chunks
// are never indexed by a shape they were not sized for (the fault of commit
// 01a0e59).  The unplanned calls redo from the exact plan on a raised check;
// the planned ones raise CRDT_DEV_PLAN (k_d2_check).  viol == nullptr: an
// exact plan the host read back, nothing to check.
struct PlanGuard {
    uint32_t bk, bt, br, W, P, words, b0, s0, tl, tw;
    uint32_t *viol;
};
__device__ __forceinline__ bool plan_guard_ok(const SortPlan &p, const PlanGuard &g) {
    if (!g.viol) return true;
    if (p.bk == g.bk && p.bt == g.bt && p.br == g.br && p.W == g.W && p.P == g.P && p.words == g.words &&
        p.b0 == g.b0 && p.s0 == g.s0 && p.tl == g.tl && p.tw == g.tw)
        return true;
    if (threadIdx.x == 0) atomicOr(g.viol, 1u);
    return false;
}
// The guard of the D2 call this host thread is launching (GuardScope in
// d2_body); none outside one.
static thread_local PlanGuard t_guard{};
static PlanGuard cur_guard() { return t_guard; }
struct GuardScope {
    explicit GuardScope(const SortPlan &h, uint32_t *viol) { set(h, viol); }
    ~GuardScope() { t_guard = PlanGuard{}; }
    void set(const SortPlan &h, uint32_t *viol) {
        t_guard = viol ? PlanGuard{h.bk, h.bt, h.br, h.W, h.P, h.words, h.b0, h.s0, h.tl, h.tw, viol} : PlanGuard{};
    }
};

struct SortMinMax {              // one per minmax workgroup, reduced by k_sort_plan
    unsigned long long kmin, kmax, tmin, tmax, rmin, rmax;
};

__device__ __forceinline__ uint32_t bitwidth(uint64_t x) { return x ? 64u - (uint32_t)__clzll((long long)x) : 0u; }

// VEC: key / ts / rep 16-byte aligned -- two tuples per lane per unit in
// 16- / 8-byte loads, four units in flight.  One
// launch covers both inputs of the fused merge: workgroups [0, g_a) read
// `in`, the rest `in2`.
template <bool VEC>
__global__ __launch_bounds__(256) void k_sort_minmax(crdt_tuples in, size_t n, crdt_tuples in2, size_t n2,
                                                     unsigned g_a, SortMinMax *mm) {
    unsigned long long kmin = ~0ULL, kmax = 0, tmin = ~0ULL, tmax = 0, rmin = ~0ULL, rmax = 0;
    auto acc = [&](unsigned long long k, unsigned long long t, unsigned long long r) {
        kmin = k < kmin ? k : kmin;
        kmax = k > kmax ? k : kmax;
        tmin = t < tmin ? t : tmin;
        tmax = t > tmax ? t : tmax;
        rmin = r < rmin ? r : rmin;
        rmax = r > rmax ? r : rmax;
    };
    const bool second = blockIdx.x >= g_a;
    const crdt_tuples t_in = second ? in2 : in;
    const size_t m = second ? n2 : n;
    const size_t b0 = second ? blockIdx.x - g_a : blockIdx.x, gs = second ? gridDim.x - g_a : g_a;
    size_t i0 = 0;
    if constexpr (VEC) {
        // units of two tuples: a lane reads 16 B of keys, 16 B of ts, 8 B of
        // reps per unit, consecutive lanes consecutive units (every load
        // instruction one contiguous 1 KB / 512 B span), four units in flight
        // (a lane reading two adjacent 16-B halves of 32 B per array ran at
        // 4.1 TB/s)
        const size_t nu = m / 2;
        const ulonglong2 *K = (const ulonglong2 *)t_in.key, *T = (const ulonglong2 *)t_in.ts;
        const uint2 *R = (const uint2 *)t_in.rep;
        const size_t stride = gs * 256;
        size_t u = b0 * 256 + threadIdx.x;
        for (; u + 3 * stride < nu; u += 4 * stride) {
            ulonglong2 k[4], t[4];
            uint2 r[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                k[j] = K[u + j * stride];
                t[j] = T[u + j * stride];
                r[j] = R[u + j * stride];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc(k[j].x, t[j].x, r[j].x);
                acc(k[j].y, t[j].y, r[j].y);
            }
        }
        for (; u < nu; u += stride) {
            const ulonglong2 k = K[u], t = T[u];
            const uint2 r = R[u];
            acc(k.x, t.x, r.x);
            acc(k.y, t.y, r.y);
        }
        i0 = nu * 2;
    }
    for (size_t i = i0 + b0 * 256 + threadIdx.x; i < m; i += gs * 256) acc(t_in.key[i], t_in.ts[i], t_in.rep[i]);
    for (int w = 32; w >= 1; w >>= 1) {
        kmin = min(kmin, (unsigned long long)__shfl_xor(kmin, w, 64));
        kmax = max(kmax, (unsigned long long)__shfl_xor(kmax, w, 64));
        tmin = min(tmin, (unsigned long long)__shfl_xor(tmin, w, 64));
        tmax = max(tmax, (unsigned long long)__shfl_xor(tmax, w, 64));
        rmin = min(rmin, (unsigned long long)__shfl_xor(rmin, w, 64));
        rmax = max(rmax, (unsigned long long)__shfl_xor(rmax, w, 64));
    }
    // workgroup partials, reduced by k_sort_plan (atomics on six shared
    // addresses serialised: they took as long as the whole read)
    __shared__ unsigned long long sred[6][4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sred[0][w] = kmin;
        sred[1][w] = kmax;
        sred[2][w] = tmin;
        sred[3][w] = tmax;
        sred[4][w] = rmin;
        sred[5][w] = rmax;
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int f = threadIdx.x;
        unsigned long long v = sred[f][0];
        for (int k = 1; k < 4; ++k) v = (f & 1) ? max(v, sred[f][k]) : min(v, sred[f][k]);
        (&mm[blockIdx.x].kmin)[f] = v;
    }
}

constexpr unsigned MM_BLOCKS = 1024;   // minmax partials per input (at most)

// one launch over `in` (n) and `in2` (n2, may be 0); returns the number of
// partials written to mm[0, g)
static unsigned launch_minmax(crdt_ctx *ctx, const crdt_tuples &in, size_t n, const crdt_tuples &in2, size_t n2,
                              SortMinMax *mm) {
    auto aligned = [](const crdt_tuples &t) {
        return (((uintptr_t)t.key | (uintptr_t)t.ts | (uintptr_t)t.rep) & 15) == 0;
    };
    const bool vec = (!n || aligned(in)) && (!n2 || aligned(in2));
    auto blocks = [&](size_t m) {
        return m ? std::min(MM_BLOCKS, grid_for(vec ? m / 8 + 1 : m, 256, (unsigned)(ctx->num_cus * g_mm_bpc))) : 0u;
    };
    const unsigned ga = blocks(n), gb = blocks(n2);
    if (vec) k_sort_minmax<true><<<ga + gb, 256, 0, ctx->stream>>>(in, n, in2, n2, ga, mm);
    else k_sort_minmax<false><<<ga + gb, 256, 0, ctx->stream>>>(in, n, in2, n2, ga, mm);
    return ga + gb;
}

// A SAMPLE of both inputs' field ranges (sort.sample_plan): per side 256
// runs of 64 consecutive tuples (one wave each: coalesced 512-B loads),
// evenly spread from the first tuple to the last, partials in the minmax
// format.  The plan widens the sampled ranges (k_sort_plan's margin) and
// the composing upsweep checks every tuple against them (the violation
// word): the dense-key D2 paths then skip the full minmax read (400 MB at
// config D) and redo the call from an exact plan only when a tuple fell
// outside.  (32768 single tuples per side, strided: 12 us.)
constexpr unsigned SAMPLE_WG = 64;       // workgroups per side (4 runs each)
__global__ __launch_bounds__(256) void k_sample_minmax(crdt_tuples in, size_t n, crdt_tuples in2, size_t n2,
                                                       SortMinMax *mm) {
    const bool second = blockIdx.x >= SAMPLE_WG;
    const crdt_tuples t = second ? in2 : in;
    const size_t m = second ? n2 : n;
    constexpr size_t NR = (size_t)SAMPLE_WG * 4;      // runs per side
    unsigned long long kmin = ~0ULL, kmax = 0, tmin = ~0ULL, tmax = 0, rmin = ~0ULL, rmax = 0;
    const size_t run = (size_t)(blockIdx.x % SAMPLE_WG) * 4 + (threadIdx.x >> 6);
    const size_t i = (m > NR * 64 ? run * (m - 64) / (NR - 1) : run * 64) + (threadIdx.x & 63);
    if (i < m) {
        const unsigned long long k = t.key[i], ts = t.ts[i], r = t.rep[i];
        kmin = kmax = k;
        tmin = tmax = ts;
        rmin = rmax = r;
    }
    for (int w = 32; w >= 1; w >>= 1) {
        kmin = min(kmin, (unsigned long long)__shfl_xor(kmin, w, 64));
        kmax = max(kmax, (unsigned long long)__shfl_xor(kmax, w, 64));
        tmin = min(tmin, (unsigned long long)__shfl_xor(tmin, w, 64));
        tmax = max(tmax, (unsigned long long)__shfl_xor(tmax, w, 64));
        rmin = min(rmin, (unsigned long long)__shfl_xor(rmin, w, 64));
        rmax = max(rmax, (unsigned long long)__shfl_xor(rmax, w, 64));
    }
    __shared__ unsigned long long sred[6][4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sred[0][w] = kmin;
        sred[1][w] = kmax;
        sred[2][w] = tmin;
        sred[3][w] = tmax;
        sred[4][w] = rmin;
        sred[5][w] = rmax;
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int f = threadIdx.x;
        unsigned long long v = sred[f][0];
        for (int k = 1; k < 4; ++k) v = (f & 1) ? max(v, sred[f][k]) : min(v, sred[f][k]);
        (&mm[blockIdx.x].kmin)[f] = v;
    }
}

// reduces the nmm minmax partials, then thread 0 sizes the composite
__global__ __launch_bounds__(256) void k_sort_plan(const SortMinMax *mms, uint32_t nmm, SortPlan *plan,
                                                   uint32_t side_bits, crdt_tuples in2, uint64_t n1,
                                                   uint32_t key_only = 0, uint32_t lww_table = 0,
                                                   uint32_t or_table = 0, uint64_t n_all = 0,
                                                   uint32_t margin = 0, uint32_t *viol = nullptr) {
    __shared__ unsigned long long sr[6][256];
    const int tid = threadIdx.x;
    if (viol && tid == 0) *viol = 0;                  // the upsweep's range check starts clean
    unsigned long long v[6] = {~0ULL, 0, ~0ULL, 0, ~0ULL, 0};
    for (uint32_t i = tid; i < nmm; i += 256)
#pragma unroll
        for (int f = 0; f < 6; ++f) {
            const unsigned long long x = (&mms[i].kmin)[f];
            v[f] = (f & 1) ? (x > v[f] ? x : v[f]) : (x < v[f] ? x : v[f]);
        }
#pragma unroll
    for (int f = 0; f < 6; ++f) sr[f][tid] = v[f];
    for (int h = 128; h >= 1; h >>= 1) {      // tree over the 256 thread partials
        __syncthreads();
        if (tid < h)
#pragma unroll
            for (int f = 0; f < 6; ++f) {
                const unsigned long long x = sr[f][tid + h], y = sr[f][tid];
                sr[f][tid] = (f & 1) ? (x > y ? x : y) : (x < y ? x : y);
            }
    }
    __syncthreads();
    if (tid >= 6) return;
    const unsigned long long r = sr[tid][0];
    const SortMinMax m{__shfl(r, 0), __shfl(r, 1), __shfl(r, 2), __shfl(r, 3), __shfl(r, 4), __shfl(r, 5)};
    if (tid != 0) return;
    SortMinMax mw = m;
    if (margin) {                                     // sampled ranges, widened by 1/256 of their span
        auto widen = [](unsigned long long &lo, unsigned long long &hi, unsigned long long cap) {
            if (lo > hi) return;                      // (no sample)
            const unsigned long long pad = (hi - lo) >> 8;
            lo = lo > pad ? lo - pad : 0;
            hi = cap - hi > pad ? hi + pad : cap;
        };
        widen(mw.kmin, mw.kmax, ~0ULL);
        widen(mw.tmin, mw.tmax, ~0ULL);
        widen(mw.rmin, mw.rmax, 0xFFFFFFFFULL);
    }
    const SortMinMax *mm = &mw;
    SortPlan p;
    p.b0 = 1 + side_bits;
    p.n1 = n1;
    p.in2 = in2;
    p.kmin = mm->kmin;
    p.tmin = mm->tmin;
    p.rmin = mm->rmin;
    p.bk = bitwidth(mm->kmax - mm->kmin);
    p.bt = bitwidth(mm->tmax - mm->tmin);
    p.br = bitwidth(mm->rmax - mm->rmin);
    p.W = p.bk + p.bt + p.br + p.b0;
    p.words = (p.W + 63) / 64;
    // key_only (the fused LWW merge): sort on the key's bits alone -- the
    // passes are stable, so each key's tuples stay in input order (A's, then
    // B's) and the dedup finds the winning tag within the key's run.  Config
    // D: 23 key bits, 3 passes instead of 7.  Single-word composites (a
    // shifted digit never straddles a word there).
    // key_only == 2 (the fused OR-Set merge): the key and the next tag bits
    // that fill its last digit plus one more digit (config D: 23 + 1 + 8 =
    // 32 bits, 4 passes) -- a group of equal sorted bits then holds ~1 tuple
    // instead of a key's ~2.5, so the dedup's in-group marks are nearly free
    // (key bits alone: the marks cost 200 + 400 us, more than the pass)
    uint32_t keep = p.bk;
    if (key_only == 2) keep += (8u - p.bk % 8u) % 8u + 8u;
    p.s0 = (key_only && p.words == 1 && p.W > keep) ? p.W - keep : 0;
    p.P = p.W - p.s0 ? (p.W - p.s0 + 7) / 8 : 1;        // >= 1: the first pass composes
    // LWW key-bucket tables (k_lww_table): one pass on the key's top 8 bits,
    // then a table of the remaining bk - 8 key bits per bucket in LDS -- 2^15
    // u32 entries (tag + marker <= 32 bits) or 2^14 u64 entries in 128 KB;
    // keys of fewer than 12 bits keep the key-only sort (tiny tables would
    // serialise the LDS atomics on a few entries)
    p.tl = p.tw = 0;
    const uint32_t kb = p.b0 + p.br + p.bt;
    if (key_only == 1 && lww_table && p.words == 1 && p.bk >= 12) {
        if (p.bk <= 8 + 15 && kb + 1 <= 32) p.tw = 4;
        else if (p.bk <= 8 + 14 && kb + 1 <= 64) p.tw = 8;
        if (p.tw) {
            p.tl = p.bk - 8;
            p.s0 = p.W - 8;
            p.P = 1;
        }
    }
    // OR-Set key chunks (k_or_chunk): the key's top bits grouped, then
    // chunks of 2^9 keys sorted in LDS -- where the grouped prefix fixes the
    // chunk (bk <= 25) and chunks hold <= 1280 tuples on average (config D:
    // 1.2k; the LDS holds 1536 -- sized for four workgroups per CU)
    if (or_table && key_only != 1 && p.words == 1 && p.bk >= 16 && p.bk <= 16 + 9 &&
        n_all <= (1280ull << (p.bk - 9))) {
        p.tw = 4;
        p.tl = 9;
        p.s0 = p.W - 16;
        p.P = 2;
    }
    *plan = p;
}

// ---------------------------------------------------------------- composite
template <int WORDS>
struct CKey {
    uint64_t w[WORDS];
};

// OR v (b bits) into c at bit offset s
template <int WORDS>
__device__ __forceinline__ void put_bits(CKey<WORDS> &c, uint32_t s, uint64_t v, uint32_t b) {
    if (b == 0) return;
#pragma unroll
    for (int q = 0; q < WORDS; ++q) {
        const int lo = q * 64;
        if ((int)s >= lo + 64 || (int)(s + b) <= lo) continue;
        if ((int)s >= lo) c.w[q] |= v << (s - lo);
        else c.w[q] |= v >> (lo - s);
    }
}
template <int WORDS>
__device__ __forceinline__ uint64_t get_bits(const CKey<WORDS> &c, uint32_t s, uint32_t b) {
    if (b == 0) return 0;
    uint64_t v = 0;
#pragma unroll
    for (int q = 0; q < WORDS; ++q) {
        const int lo = q * 64;
        if ((int)s >= lo + 64 || (int)(s + b) <= lo) continue;
        if ((int)s >= lo) v |= c.w[q] >> (s - lo);
        else v |= c.w[q] << (lo - s);
    }
    return b == 64 ? v : (v & ((1ULL << b) - 1));
}
// (key, ts, rep[, side], tomb) from the highest bits down; the side bit (the
// fused two-input sort) puts A's copy of an equal tag before B's
template <int WORDS>
__device__ __forceinline__ CKey<WORDS> compose(const SortPlan &p, uint64_t k, uint64_t t, uint32_t r, uint8_t tomb,
                                               uint32_t side) {
    CKey<WORDS> c;
#pragma unroll
    for (int q = 0; q < WORDS; ++q) c.w[q] = 0;
    c.w[0] = (tomb ? 1u : 0u) | ((uint64_t)side << 1);
    put_bits(c, p.b0, (uint64_t)(r - p.rmin), p.br);
    put_bits(c, p.b0 + p.br, t - p.tmin, p.bt);
    put_bits(c, p.b0 + p.br + p.bt, k - p.kmin, p.bk);
    return c;
}
template <int WORDS>
__device__ __forceinline__ uint32_t digit_of(const CKey<WORDS> &c, uint32_t pass, uint32_t s0) {
    const uint32_t s = 8 * pass + s0;
    uint64_t x = c.w[0];                      // select, not a runtime index: keeps c in registers
#pragma unroll
    for (int q = 1; q < WORDS; ++q)
        if ((s >> 6) == (uint32_t)q) x = c.w[q];
    return (uint32_t)(x >> (s & 63)) & 255u;
}

// ---------------------------------------------------------------- upsweep
template <int WORDS, bool FIRST>
__device__ __forceinline__ void sort_load(const crdt_tuples &in, const uint64_t *__restrict__ src, size_t n,
                                          const SortPlan &p, size_t base, CKey<WORDS> *c) {
#pragma unroll
    for (int r = 0; r < SR; ++r) {
        const size_t e = base + (size_t)r * SB + threadIdx.x;
        if (e < n) {
            if constexpr (FIRST) {
                if (e < p.n1) {
                    c[r] = compose<WORDS>(p, in.key[e], in.ts[e], in.rep[e], in.tomb[e], 0);
                } else {
                    const size_t f = e - p.n1;
                    c[r] = compose<WORDS>(p, p.in2.key[f], p.in2.ts[f], p.in2.rep[f], p.in2.tomb[f], 1);
                }
            } else {
#pragma unroll
                for (int q = 0; q < WORDS; ++q) c[r].w[q] = src[(size_t)q * n + e];
            }
        }
    }
}

// cnt[d * ntiles + t] = composites of tile t with digit d in this pass
__device__ __forceinline__ bool outside(uint64_t off, uint32_t b) { return b < 64 && (off >> b) != 0; }

template <int WORDS, bool FIRST>
__global__ __launch_bounds__(SB) void k_sort_up(crdt_tuples in, const uint64_t *__restrict__ src, size_t n,
                                                const SortPlan *__restrict__ plan_, uint32_t pass, uint32_t ntiles,
                                                uint32_t *__restrict__ cnt, uint64_t *__restrict__ comp,
                                                uint32_t *__restrict__ viol = nullptr, PlanGuard pg = {}) {
    __shared__ uint32_t h[SWAVES * 256];          // one histogram per wave: fewer LDS atomic collisions
    const int tid = threadIdx.x, w = tid >> 6;
    for (int i = tid; i < SWAVES * 256; i += SB) h[i] = 0;
    const SortPlan p = *plan_;
    if (!plan_guard_ok(p, pg)) return;                 // (uniform: before any barrier)
    const size_t base = (size_t)blockIdx.x * ST;
    CKey<WORDS> c[SR];
    sort_load<WORDS, FIRST>(in, src, n, p, base, c);
    if (FIRST && viol) {                          // a planned call: every tuple inside the plan's ranges?
        bool bad = false;
#pragma unroll
        for (int r = 0; r < SR; ++r) {
            const size_t e = base + (size_t)r * SB + tid;
            if (e >= n) continue;
            const bool side = e >= p.n1;
            const crdt_tuples &T = side ? p.in2 : in;
            const size_t f = side ? e - p.n1 : e;
            bad = bad || outside(T.key[f] - p.kmin, p.bk) || outside(T.ts[f] - p.tmin, p.bt) ||
                  outside((uint64_t)T.rep[f] - p.rmin, p.br);
        }
        if (__ballot(bad) && (tid & 63) == 0) atomicOr(viol, 1u);
    }
    if constexpr (FIRST) {                        // the composites, so pass 0 reads 8 B instead of a tuple
#pragma unroll
        for (int r = 0; r < SR; ++r) {
            const size_t e = base + (size_t)r * SB + tid;
            if (e < n)
#pragma unroll
                for (int q = 0; q < WORDS; ++q) comp[(size_t)q * n + e] = c[r].w[q];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < SR; ++r)
        if (base + (size_t)r * SB + tid < n) atomicAdd(&h[w * 256 + digit_of(c[r], pass, p.s0)], 1u);
    __syncthreads();
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < SWAVES; ++k) v += h[k * 256 + tid];
    cnt[(size_t)tid * ntiles + blockIdx.x] = v;
}

// The composing upsweep (pass 0) with two tuples per lane per round: 16-B
// key / ts loads, 8-B reps, 2-B tombs (the scalar form issues four narrow
// loads per tuple).  Needs key / ts 16-byte, rep 8-byte, tomb 2-byte aligned
// sides and an even n1 (no pair straddles the two inputs); the histogram
// counts do not depend on which lane composes which tuple.
__global__ __launch_bounds__(SB) void k_sort_up_vec(crdt_tuples in, size_t n, const SortPlan *__restrict__ plan_,
                                                    uint32_t ntiles, uint32_t *__restrict__ cnt,
                                                    uint64_t *__restrict__ comp, uint32_t *__restrict__ viol, PlanGuard pg = {}) {
    __shared__ uint32_t h[SWAVES * 256];
    const int tid = threadIdx.x, w = tid >> 6;
    for (int i = tid; i < SWAVES * 256; i += SB) h[i] = 0;
    const SortPlan p = *plan_;
    if (!plan_guard_ok(p, pg)) return;                 // (uniform: before any barrier)
    const size_t base = (size_t)blockIdx.x * ST;
    uint64_t c[SR];
    bool bad = false;                                 // (viol) a field outside the plan's ranges
    auto out_of = [&](uint64_t k, uint64_t t, uint32_t r) {
        return outside(k - p.kmin, p.bk) || outside(t - p.tmin, p.bt) || outside((uint64_t)r - p.rmin, p.br);
    };
#pragma unroll
    for (int r = 0; r < SR / 2; ++r) {
        const size_t e = base + 2 * ((size_t)r * SB + tid);
        c[2 * r] = c[2 * r + 1] = 0;
        if (e >= n) continue;
        const bool side = e >= p.n1;
        const crdt_tuples &T = side ? p.in2 : in;
        const size_t f = side ? e - p.n1 : e;
        if (e + 1 < n) {
            typedef uint64_t v2u64 __attribute__((ext_vector_type(2)));   // (nontemporal loads: each tuple is read once)
            typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));
            const v2u64 kv = __builtin_nontemporal_load((const v2u64 *)(T.key + f)),
                        tv = __builtin_nontemporal_load((const v2u64 *)(T.ts + f));
            const v2u32 rv = __builtin_nontemporal_load((const v2u32 *)(T.rep + f));
            const ulonglong2 k{kv.x, kv.y}, t{tv.x, tv.y};
            const uint2 rp{rv.x, rv.y};
            const uint16_t tb = __builtin_nontemporal_load((const uint16_t *)(T.tomb + f));
            if (viol) bad = bad || out_of(k.x, t.x, rp.x) || out_of(k.y, t.y, rp.y);
            c[2 * r] = compose<1>(p, k.x, t.x, rp.x, (uint8_t)(tb & 0xFF), side).w[0];
            c[2 * r + 1] = compose<1>(p, k.y, t.y, rp.y, (uint8_t)(tb >> 8), side).w[0];
            *(ulonglong2 *)(comp + e) = ulonglong2{c[2 * r], c[2 * r + 1]};
        } else {
            if (viol) bad = bad || out_of(T.key[f], T.ts[f], T.rep[f]);
            c[2 * r] = compose<1>(p, T.key[f], T.ts[f], T.rep[f], T.tomb[f], side).w[0];
            comp[e] = c[2 * r];
        }
    }
    if (viol && __ballot(bad) && (tid & 63) == 0) atomicOr(viol, 1u);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < SR; ++r) {
        const size_t e = base + 2 * ((size_t)(r >> 1) * SB + tid) + (r & 1);
        CKey<1> v;
        v.w[0] = c[r];
        if (e < n) atomicAdd(&h[w * 256 + digit_of(v, 0, p.s0)], 1u);
    }
    __syncthreads();
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < SWAVES; ++k) v += h[k * 256 + tid];
    cnt[(size_t)tid * ntiles + blockIdx.x] = v;
}

// loc[d * ntiles + t] = tile t's start within digit d's bucket; tot[d] = bucket size.
// One 1024-thread workgroup per column: 8192 tile counts per block-scan round
// (one round up to 33M composites; a 256-thread, 2048-per-round form spent
// most of its 9.6 us in three serial rounds of barriers).
constexpr int CSB = 1024;
__global__ __launch_bounds__(CSB) void k_sort_colscan(const uint32_t *__restrict__ cnt, uint32_t ntiles,
                                                      uint32_t *__restrict__ loc, uint32_t *__restrict__ tot,
                                                      unsigned long long *__restrict__ zero = nullptr) {
    constexpr int K = 8;
    constexpr int NW = CSB / 64;
    __shared__ uint32_t s_w[NW];
    const uint32_t *c = cnt + (size_t)blockIdx.x * ntiles;
    uint32_t *o = loc + (size_t)blockIdx.x * ntiles;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t carry = 0;
    for (uint32_t t0 = 0; t0 < ntiles; t0 += CSB * K) {
        const uint32_t i0 = t0 + threadIdx.x * K;
        uint32_t v[K], sum = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            v[k] = i0 + k < ntiles ? c[i0 + k] : 0u;
            sum += v[k];
        }
        uint32_t x = sum;                       // wave inclusive scan
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        if (lane == 63) s_w[w] = x;
        __syncthreads();
        uint32_t off = 0, all = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const uint32_t ws = s_w[k];
            off += k < w ? ws : 0u;
            all += ws;
        }
        __syncthreads();                        // s_w is rewritten next round
        uint32_t run = carry + off + x - sum;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (i0 + k < ntiles) o[i0 + k] = run;
            run += v[k];
        }
        carry += all;
    }
    if (threadIdx.x == 0) tot[blockIdx.x] = carry;
    if (zero && threadIdx.x == 0) zero[blockIdx.x] = 0;   // the bucket tables' flags
    if (zero && threadIdx.x == 0 && blockIdx.x == 0) zero[256] = 0;   // k_or_chunk's fallback word
}

// ---------------------------------------------------------------- one pass
// output start of tile t's digit-d composites = (sum of tot[0..d)) + loc[d * ntiles + t]
template <int WORDS, bool FIRST, bool LAST>
__global__ __launch_bounds__(SB) void k_sort_pass(crdt_tuples in, const uint64_t *__restrict__ src, size_t n,
                                                  const SortPlan *__restrict__ plan_, uint32_t pass, uint32_t ntiles,
                                                  const uint32_t *__restrict__ loc, const uint32_t *__restrict__ tot,
                                                  uint64_t *__restrict__ dst, crdt_tuples out, int xcd, PlanGuard pg = {}) {
    // wc: per (round, wave, digit) counts, then their exclusive prefix;
    // reused (after the ranks are taken) as the staging area of the tile
    constexpr int WC_BYTES = SR * SWAVES * 256 * 2;
    constexpr int STAGE_BYTES = ST * 8 * WORDS;
    __shared__ __attribute__((aligned(16))) unsigned char lds[WC_BYTES > STAGE_BYTES ? WC_BYTES : STAGE_BYTES];
    __shared__ uint32_t s_lstart[256], s_excl[256];
    __shared__ uint32_t s_wsum[SWAVES];
    uint16_t *wc = (uint16_t *)lds;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const SortPlan p = *plan_;
    if (!plan_guard_ok(p, pg)) return;                 // (uniform: before any barrier)
    // each XCD's workgroups take one contiguous range of tiles: tile t's and
    // t + 1's runs of a digit are adjacent in the output, so their partial
    // lines meet in one L2 instead of two (sort.xcd_tiles; speed only)
    const uint32_t t = xcd ? xcd_contig(blockIdx.x, gridDim.x) : blockIdx.x;
    const size_t base = (size_t)t * ST;
    for (int i = tid; i < SR * SWAVES * 256 / 4; i += SB) ((uint64_t *)lds)[i] = 0;
    {
        const uint32_t lt = loc[(size_t)tid * ntiles + t];
        uint64_t all;
        s_excl[tid] = (uint32_t)block_exclusive_scan_u64(tot[tid], &all) + lt;   // barriers inside
    }

    // ---- load (and compose on the first pass) SR composites per thread, round-major
    CKey<WORDS> c[SR];
    sort_load<WORDS, FIRST>(in, src, n, p, base, c);

    // ---- stable in-tile rank: wave ballots per round, then one prefix per digit
    uint32_t rk[SR / 4];                      // rank within the wave, 8 bits each
#pragma unroll
    for (int r = 0; r < SR / 4; ++r) rk[r] = 0;
    uint32_t dg[SR / 4];                      // digits, 8 bits each (256: past the end)
#pragma unroll
    for (int r = 0; r < SR; ++r) {
        const size_t e = base + (size_t)r * SB + tid;
        const bool valid = e < n;
        const uint32_t d = valid ? digit_of(c[r], pass, p.s0) : 0u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const uint64_t m = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? m : ~m;
        }
        const uint32_t below = (uint32_t)__popcll(peers & ((1ULL << lane) - 1ULL));
        if (valid && below == 0) wc[(r * SWAVES + w) * 256 + d] = (uint16_t)__popcll(peers);
        rk[r >> 2] |= below << (8 * (r & 3));
        if ((r & 3) == 0) dg[r >> 2] = 0;
        dg[r >> 2] |= (valid ? d : 255u) << (8 * (r & 3));
    }
    __syncthreads();
    {   // thread d: exclusive prefix of digit d over (round, wave), in tile order
        const int d = tid;
        uint32_t run = 0;
        for (int i = 0; i < SR * SWAVES; ++i) {
            const uint32_t v = wc[i * 256 + d];
            wc[i * 256 + d] = (uint16_t)run;
            run += v;
        }
        // local start of digit d in the digit-sorted tile
        uint32_t x = run;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_wsum[w] = x;
        __syncthreads();
        uint32_t off = 0;
        for (int k = 0; k < w; ++k) off += s_wsum[k];
        s_lstart[d] = off + x - run;
    }
    __syncthreads();                          // s_lstart of every digit
    uint32_t pos[SR / 2];                     // local positions, 16 bits each
#pragma unroll
    for (int r = 0; r < SR; ++r) {
        const uint32_t d = (dg[r >> 2] >> (8 * (r & 3))) & 255u;
        const size_t e = base + (size_t)r * SB + tid;
        uint32_t lp = 0;
        if (e < n) lp = s_lstart[d] + wc[(r * SWAVES + w) * 256 + d] + ((rk[r >> 2] >> (8 * (r & 3))) & 255u);
        if ((r & 1) == 0) pos[r >> 1] = 0;
        pos[r >> 1] |= lp << (16 * (r & 1));
    }
    __syncthreads();                          // wc dead: the area becomes the stage
    {
        uint64_t *stage = (uint64_t *)lds;
#pragma unroll
        for (int r = 0; r < SR; ++r) {
            const size_t e = base + (size_t)r * SB + tid;
            if (e < n) {
                const uint32_t lp = (pos[r >> 1] >> (16 * (r & 1))) & 0xFFFFu;
#pragma unroll
                for (int q = 0; q < WORDS; ++q) stage[q * ST + lp] = c[r].w[q];
            }
        }
    }
    __syncthreads();
    // ---- scatter in digit order: consecutive j of one digit -> consecutive outputs
    const size_t cnt = n - base < (size_t)ST ? n - base : (size_t)ST;
    const uint64_t *stage = (const uint64_t *)lds;
    for (int j = tid; j < (int)cnt; j += SB) {
        CKey<WORDS> v;
#pragma unroll
        for (int q = 0; q < WORDS; ++q) v.w[q] = stage[q * ST + j];
        const uint32_t d = digit_of(v, pass, p.s0);
        const size_t o = (size_t)s_excl[d] + (uint32_t)(j - (int)s_lstart[d]);
        if constexpr (LAST) {
            out.key[o] = p.kmin + get_bits(v, p.b0 + p.br + p.bt, p.bk);
            out.ts[o] = p.tmin + get_bits(v, p.b0 + p.br, p.bt);
            out.rep[o] = (uint32_t)(p.rmin + get_bits(v, p.b0, p.br));
            out.tomb[o] = (uint8_t)(v.w[0] & 1u);
        } else {
#pragma unroll
            for (int q = 0; q < WORDS; ++q) dst[(size_t)q * n + o] = v.w[q];
        }
    }
}

template <int WORDS>
static void launch_pass(bool first, bool last, unsigned grid, hipStream_t st, const crdt_tuples &in,
                        const uint64_t *src, size_t n, const SortPlan *plan, uint32_t pass, const uint32_t *loc,
                        const uint32_t *tot, uint64_t *dst, const crdt_tuples &out) {
    const int x = g_sort_xcd;
    if (first && last)
        k_sort_pass<WORDS, true, true><<<grid, SB, 0, st>>>(in, src, n, plan, pass, grid, loc, tot, dst, out, x,
                                                             cur_guard());
    else if (first)
        k_sort_pass<WORDS, true, false><<<grid, SB, 0, st>>>(in, src, n, plan, pass, grid, loc, tot, dst, out, x,
                                                             cur_guard());
    else if (last)
        k_sort_pass<WORDS, false, true><<<grid, SB, 0, st>>>(in, src, n, plan, pass, grid, loc, tot, dst, out, x,
                                                             cur_guard());
    else
        k_sort_pass<WORDS, false, false><<<grid, SB, 0, st>>>(in, src, n, plan, pass, grid, loc, tot, dst, out, x,
                                                             cur_guard());
}

// P passes; the last decodes into `out`, or (decode = false) leaves the
// sorted composites in *result (word-major planes of n)
template <int WORDS>
static int sort_words(crdt_ctx *ctx, const crdt_tuples &in, size_t n, const crdt_tuples &out, const SortPlan *plan_d,
                      uint32_t P, uint64_t *bufs, uint32_t *cnt, uint32_t *loc, uint32_t *tot, bool decode = true,
                      uint64_t **result = nullptr, bool vec_first = false,
                      unsigned long long *zero = nullptr, uint32_t *viol = nullptr) {
    const hipStream_t st = ctx->stream;
    const unsigned ntiles = (unsigned)((n + ST - 1) / ST);
    uint64_t *a = bufs, *b = bufs + (size_t)WORDS * n;
    for (uint32_t q = 0; q < P; ++q) {
        // pass 0's upsweep composes from the tuples and stores the composites
        if (q == 0 && WORDS == 1 && vec_first)
            k_sort_up_vec<<<ntiles, SB, 0, st>>>(in, n, plan_d, ntiles, cnt, a, viol, cur_guard());
        else if (q == 0)
            k_sort_up<WORDS, true><<<ntiles, SB, 0, st>>>(in, nullptr, n, plan_d, q, ntiles, cnt, a, viol, cur_guard());
        else
            k_sort_up<WORDS, false><<<ntiles, SB, 0, st>>>(in, a, n, plan_d, q, ntiles, cnt, nullptr, nullptr,
                                                              cur_guard());
        k_sort_colscan<<<256, CSB, 0, st>>>(cnt, ntiles, loc, tot, q == 0 ? zero : nullptr);
        launch_pass<WORDS>(false, decode && q + 1 == P, ntiles, st, in, a, n, plan_d, q, loc, tot, b, out);
        std::swap(a, b);
    }
    if (result) *result = a;
    return check_launch(ctx);
}

}  // namespace crdt

namespace crdt {
// out[i] = lower_bound(v[0..n), probes[i]) in unsigned order: one thread per probe.
__global__ void k_lower_bound_u64(const uint64_t *__restrict__ v, uint64_t n, const uint64_t *__restrict__ probes,
                                  uint64_t m, uint64_t *__restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
        const uint64_t x = probes[i];
        uint64_t lo = 0, hi = n;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (v[mid] < x) lo = mid + 1;
            else hi = mid;
        }
        out[i] = lo;
    }
}
}  // namespace crdt

namespace crdt {
// ---------------------------------------------------------------- fused D2 merge
// Unsorted set merge as ONE sort: both sides' tuples go through the radix
// sort together with a side bit between rep and tomb, composite order
// (key, ts, rep, side, tomb).  That order IS the stable merge of the two
// sorted sides (A's copies of an equal tag first, each side's copies by
// tomb), so the LWW / OR-Set merge reduces to a dedup over neighbours of the
// sorted composites: no decode pass, no second sort, no merge path.
//   LWW: emit the last composite of each key run (the key's maximal tag);
//        its tomb is that of the FIRST composite of its tag run
//   OR : emit the first composite of each tag run; tomb = OR over the run
// Count pass (per 2048-composite tile) -> scan of the tile counts -> apply
// pass (ballot ranks, compacted stores straight to the SoA output).
enum { DD_LWW = 0, DD_OR = 1 };
constexpr int DB = 256;              // threads per dedup workgroup
constexpr int DI = 8;                // composites per thread (round-major)
constexpr int DT = DB * DI;          // 2048 composites per tile

template <int WORDS>
__device__ __forceinline__ CKey<WORDS> ck_load(const uint64_t *__restrict__ c, size_t n, size_t e) {
    CKey<WORDS> v;
#pragma unroll
    for (int q = 0; q < WORDS; ++q) v.w[q] = c[(size_t)q * n + e];
    return v;
}
// bits [s, 64*WORDS) of x and y equal
template <int WORDS>
__device__ __forceinline__ bool eq_from(const CKey<WORDS> &x, const CKey<WORDS> &y, uint32_t s) {
    bool eq = true;
#pragma unroll
    for (int q = 0; q < WORDS; ++q) {
        const uint32_t lo = 64u * q;
        if (s >= lo + 64) continue;
        const uint64_t m = s > lo ? ~0ULL << (s - lo) : ~0ULL;
        eq = eq && ((x.w[q] ^ y.w[q]) & m) == 0;
    }
    return eq;
}
// bits [s, 64*WORDS) of x against y's: -1 / 0 / +1
template <int WORDS>
__device__ __forceinline__ int cmp_from(const CKey<WORDS> &x, const CKey<WORDS> &y, uint32_t s) {
    int r = 0;
#pragma unroll
    for (int q = WORDS - 1; q >= 0; --q) {
        const uint32_t lo = 64u * q;
        if (s >= lo + 64) continue;
        const uint64_t m = s > lo ? ~0ULL << (s - lo) : ~0ULL;
        const uint64_t a = x.w[q] & m, b = y.w[q] & m;
        if (r == 0 && a != b) r = a > b ? 1 : -1;
    }
    return r;
}
// LWW winner of a key's run, whatever the run's order (a key-only sort
// leaves it in input order): the max (ts, rep) tag; its tomb that of the
// tag's first copy in (key, ts, rep, side, tomb) order -- the least tomb of
// A's copies, else of B's (side = bit 1 when b0 > 1)
template <int WORDS>
struct LwwWin {                                          // (scalars, not side-indexed arrays: no scratch)
    CKey<WORDS> win;
    uint32_t ta, tb, ha, hb;                             // least tomb and "holds the tag", side A / side B
    __device__ __forceinline__ void reset(const CKey<WORDS> &x, uint32_t b0) {
        const bool sb = b0 > 1 && ((x.w[0] >> 1) & 1u);
        const uint32_t xt = (uint32_t)x.w[0] & 1u;
        ta = sb ? 1u : xt;
        tb = sb ? xt : 1u;
        ha = sb ? 0u : 1u;
        hb = sb ? 1u : 0u;
    }
    __device__ __forceinline__ LwwWin(const CKey<WORDS> &x, uint32_t b0) : win(x) { reset(x, b0); }
    __device__ __forceinline__ void consider(const CKey<WORDS> &x, uint32_t b0) {
        const int o = cmp_from(x, win, b0);
        if (o > 0) {                                    // a larger tag
            win = x;
            reset(x, b0);
        } else if (o == 0) {
            const bool sb = b0 > 1 && ((x.w[0] >> 1) & 1u);
            const uint32_t xt = (uint32_t)x.w[0] & 1u;
            if (sb) {
                tb &= xt;
                hb = 1u;
            } else {
                ta &= xt;
                ha = 1u;
            }
        }
    }
    __device__ __forceinline__ uint32_t tomb() const { return ha ? ta : tb; }
};

// The neighbours in sorted order come from the adjacent lanes (shuffles);
// a wave's edge lanes take them from the next / previous wave's edge values
// exchanged through LDS, the tile's two outer neighbours are loaded once up
// front.  (A global load per round in the edge lanes put eight dependent HBM
// round trips in front of every tile's ballots.)
template <int WORDS>
struct DdEdges {
    uint64_t lo[DI][DB / 64][WORDS], hi[DI][DB / 64][WORDS];   // lane 0 / lane 63 composites per (round, wave)
    uint64_t prev[WORDS], next[WORDS];                         // c[base - 1], c[base + DT]
};
template <int WORDS>
__device__ __forceinline__ void dd_edges_put(DdEdges<WORDS> &x, const CKey<WORDS> *v, int lane, int w) {
    if (lane == 0 || lane == 63)
#pragma unroll
        for (int r = 0; r < DI; ++r)
#pragma unroll
            for (int q = 0; q < WORDS; ++q) (lane == 0 ? x.lo : x.hi)[r][w][q] = v[r].w[q];
}
template <int WORDS>
__device__ __forceinline__ CKey<WORDS> dd_next(const DdEdges<WORDS> &x, const CKey<WORDS> &v, int r, int lane, int w) {
    CKey<WORDS> nx;
#pragma unroll
    for (int q = 0; q < WORDS; ++q) {
        nx.w[q] = (uint64_t)__shfl_down((unsigned long long)v.w[q], 1, 64);
        if (lane == 63)
            nx.w[q] = w + 1 < DB / 64 ? x.lo[r][w + 1][q] : (r + 1 < DI ? x.lo[r + 1][0][q] : x.next[q]);
    }
    return nx;
}
template <int WORDS>
__device__ __forceinline__ CKey<WORDS> dd_prev(const DdEdges<WORDS> &x, const CKey<WORDS> &v, int r, int lane, int w) {
    CKey<WORDS> pv;
#pragma unroll
    for (int q = 0; q < WORDS; ++q) {
        pv.w[q] = (uint64_t)__shfl_up((unsigned long long)v.w[q], 1, 64);
        if (lane == 0) pv.w[q] = w > 0 ? x.hi[r][w - 1][q] : (r > 0 ? x.hi[r - 1][DB / 64 - 1][q] : x.prev[q]);
    }
    return pv;
}
// the tile's composites (round-major) and its outer neighbours into LDS
template <int WORDS>
__device__ __forceinline__ void dd_load(const uint64_t *__restrict__ c, size_t n, size_t base, CKey<WORDS> *v,
                                        DdEdges<WORDS> &x) {
    const int tid = threadIdx.x;
    CKey<WORDS> pe, ne;
#pragma unroll
    for (int q = 0; q < WORDS; ++q) pe.w[q] = ne.w[q] = 0;
    if (tid == 0 && base > 0) pe = ck_load<WORDS>(c, n, base - 1);
    if (tid == 0 && base + DT < n) ne = ck_load<WORDS>(c, n, base + DT);
#pragma unroll
    for (int r = 0; r < DI; ++r) {
        const size_t e = base + (size_t)r * DB + tid;
        if (e < n) v[r] = ck_load<WORDS>(c, n, e);
        else
#pragma unroll
            for (int q = 0; q < WORDS; ++q) v[r].w[q] = 0;
    }
    if (tid == 0)
#pragma unroll
        for (int q = 0; q < WORDS; ++q) {
            x.prev[q] = pe.w[q];
            x.next[q] = ne.w[q];
        }
    dd_edges_put<WORDS>(x, v, tid & 63, tid >> 6);
}

template <int MODE, int WORDS>
__global__ __launch_bounds__(DB) void k_dd_count(const uint64_t *__restrict__ c, size_t n,
                                                 const SortPlan *__restrict__ plan_, uint32_t *__restrict__ cnt, PlanGuard pg = {}) {
    __shared__ uint32_t s_w[DB / 64];
    __shared__ DdEdges<WORDS> s_x;
    const SortPlan p = *plan_;
    if (!plan_guard_ok(p, pg)) return;                 // (uniform: before any barrier)
    const size_t base = (size_t)blockIdx.x * DT;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t m = 0;
    CKey<WORDS> v[DI];
    dd_load<WORDS>(c, n, base, v, s_x);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < DI; ++r) {
        const size_t e = base + (size_t)r * DB + threadIdx.x;
        if constexpr (MODE == DD_LWW) {
            const CKey<WORDS> nb = dd_next<WORDS>(s_x, v[r], r, lane, w);
            m += (e < n && (e + 1 == n || !eq_from(v[r], nb, p.b0 + p.br + p.bt))) ? 1u : 0u;
        } else {
            const CKey<WORDS> nb = dd_prev<WORDS>(s_x, v[r], r, lane, w);
            m += (e < n && (e == 0 || !eq_from(v[r], nb, p.b0))) ? 1u : 0u;
        }
    }
    for (int o = 32; o >= 1; o >>= 1) m += __shfl_xor(m, o, 64);
    if (lane == 0) s_w[w] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int k = 0; k < DB / 64; ++k) t += s_w[k];
        cnt[blockIdx.x] = t;
    }
}

template <int MODE, int WORDS>
__global__ __launch_bounds__(DB) void k_dd_apply(const uint64_t *__restrict__ c, size_t n,
                                                 const SortPlan *__restrict__ plan_, const uint32_t *__restrict__ loc,
                                                 const uint32_t *__restrict__ tot, crdt_tuples out,
                                                 uint64_t *__restrict__ out_count, int diag_ = 0, PlanGuard pg = {}) {
    const int diag = kDiagBuild ? diag_ : 0;          // (the product build has no timing diagnostics)
    __shared__ uint32_t s_c[DI * (DB / 64)];      // emits per (round, wave), then their exclusive prefix
    __shared__ uint64_t s_v[MODE == DD_LWW ? DT * WORDS : 1];   // LWW: the tile's composites (run walks)
    __shared__ DdEdges<WORDS> s_x;
    const SortPlan p = *plan_;
    if (!plan_guard_ok(p, pg)) return;                 // (uniform: before any barrier)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const size_t base = (size_t)blockIdx.x * DT;
    if (blockIdx.x == 0 && tid == 0) *out_count = tot[0];
    const size_t t0 = loc[blockIdx.x];
    uint64_t em[DI];
    CKey<WORDS> v[DI];
    uint8_t tb[DI];                               // output tomb; bit 1: the tag run continues (rare walk)
    constexpr bool SEG = MODE == DD_LWW && WORDS == 1;
    uint64_t mxr[SEG ? DI : 1];                   // LWW, one word: max of c ^ 3 over the key run's part in the wave-round
    dd_load<WORDS>(c, n, base, v, s_x);
    if constexpr (MODE == DD_LWW)
#pragma unroll
        for (int r = 0; r < DI; ++r)
#pragma unroll
            for (int q = 0; q < WORDS; ++q) s_v[q * DT + r * DB + tid] = v[r].w[q];
    __syncthreads();
    if (diag == 1) return;                        // timing diagnostics (sort.rdd_diag): no stores
#pragma unroll
    for (int r = 0; r < DI; ++r) {
        const size_t e = base + (size_t)r * DB + tid;
        const CKey<WORDS> nx = dd_next<WORDS>(s_x, v[r], r, lane, w), pv = dd_prev<WORDS>(s_x, v[r], r, lane, w);
        const bool valid = e < n, has_next = e + 1 < n, has_prev = e > 0;
        const bool same_next = has_next && eq_from(nx, v[r], p.b0);
        bool f;
        if constexpr (MODE == DD_LWW) {
            // the last tuple of a key run emits; with a previous tuple of the
            // same key the run is walked for its winning tag (bit 1)
            const uint32_t kb = p.b0 + p.br + p.bt;
            f = valid && (!has_next || !eq_from(v[r], nx, kb));
            // bit 1: an earlier tuple of the same key -- the emit walks the run
            const bool cont = valid && has_prev && eq_from(pv, v[r], kb);
            tb[r] = (uint8_t)((v[r].w[0] & 1u) | (cont ? 2u : 0u));
            if constexpr (SEG) {
                // the run's max of c ^ 3 by a segmented max-scan over the
                // wave-round's 64 consecutive tuples (shuffles, no walk); bit
                // 2: the run began before the wave-round (its earlier part is
                // walked from LDS, at most one run per wave-round)
                const uint64_t S = __ballot(!cont);
                const uint64_t sm = S & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
                const int head = sm ? 63 - __clzll((long long)sm) : -1;
                uint64_t mx = v[r].w[0] ^ 3u;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint64_t y = __shfl_up((unsigned long long)mx, d, 64);
                    if (lane >= d && lane - d >= head) mx = y > mx ? y : mx;
                }
                mxr[r] = mx;
                if (head < 0 && cont) tb[r] |= 4u;
            }
        } else {
            f = valid && !(has_prev && eq_from(pv, v[r], p.b0));     // the first copy of its tag
            tb[r] = (uint8_t)((v[r].w[0] & 1u) | (same_next ? 2u : 0u));
        }
        em[r] = __ballot(f);
        if (lane == 0) s_c[r * (DB / 64) + w] = (uint32_t)__popcll(em[r]);
    }
    __syncthreads();
    if (w == 0) {                                 // exclusive prefix of the (round, wave) emit counts
        constexpr int NC = DI * (DB / 64);
        static_assert(NC <= 64, "one wave");
        const uint32_t c0 = lane < NC ? s_c[lane] : 0u;
        uint32_t x = c0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane < NC) s_c[lane] = x - c0;
    }
    __syncthreads();
    if (diag == 2) return;
    const uint32_t sk = p.b0 + p.br + p.bt;
#pragma unroll
    for (int r = 0; r < DI; ++r) {
        if (!((em[r] >> lane) & 1)) continue;
        const size_t e = base + (size_t)r * DB + tid;
        const size_t o = t0 + s_c[r * (DB / 64) + w] + (uint32_t)__popcll(em[r] & ((1ULL << lane) - 1ULL));
        uint8_t tomb = tb[r] & 1u;
        CKey<WORDS> win = v[r];
        if (tb[r] & 2u) {
            if constexpr (MODE == DD_LWW && WORDS == 1) {
                // one word (key-only sort, b0 = 2: side at bit 1, tomb at bit 0):
                // the LWW winner is the max over the key's run of c ^ 3 -- the
                // max (ts, rep), then side A (bit 1 inverted), then its least
                // tomb (bit 0 inverted) -- so the backward walk is a plain
                // 64-bit max; the tile's part from LDS, the rest from global memory
                const uint32_t kb = p.b0 + p.br + p.bt;
                const uint64_t key = v[r].w[0] >> kb;
                uint64_t mx = mxr[r];
                if (tb[r] & 4u)                           // the run's part before the wave-round
                    for (size_t j = e - (size_t)lane; j > 0;) {
                        --j;
                        const uint64_t x = j >= base ? s_v[j - base] : c[j];
                        if ((x >> kb) != key) break;
                        mx = (x ^ 3u) > mx ? x ^ 3u : mx;
                    }
                win.w[0] = mx ^ 3u;
                tomb = (uint8_t)(win.w[0] & 1u);
            } else if constexpr (MODE == DD_LWW) {
                // the key's run backwards: the tile's part from LDS, the rest
                // (a run reaching back past the tile) from global memory
                const uint32_t kb = p.b0 + p.br + p.bt;
                LwwWin<WORDS> lw(win, p.b0);
                for (size_t j = e; j > 0;) {
                    --j;
                    CKey<WORDS> x;
                    if (j >= base) {
#pragma unroll
                        for (int q = 0; q < WORDS; ++q) x.w[q] = s_v[q * DT + (j - base)];
                    } else {
                        x = ck_load<WORDS>(c, n, j);
                    }
                    if (!eq_from(x, v[r], kb)) break;
                    lw.consider(x, p.b0);
                }
                win = lw.win;
                tomb = lw.tomb();
            } else {                              // OR over the tag's copies
                for (size_t j = e + 1; j < n; ++j) {
                    const CKey<WORDS> x = ck_load<WORDS>(c, n, j);
                    if (!eq_from(x, v[r], p.b0)) break;
                    tomb |= (uint8_t)(x.w[0] & 1u);
                }
            }
        }
        out.key[o] = p.kmin + get_bits(win, sk, p.bk);
        out.ts[o] = p.tmin + get_bits(win, p.b0 + p.br, p.bt);
        out.rep[o] = (uint32_t)(p.rmin + get_bits(win, p.b0, p.br));
        out.tomb[o] = tomb;
    }
}

// ---------------------------------------------------------------- LWW D2: key-bucket tables
// sort.lww_table (default 1).  LWW keeps one tuple per key, and a key's
// winner is a MAX -- of the tag word c ^ 3 over the key's tuples (the max
// (ts, rep), then side A (bit 1 inverted), then the least tomb (bit 0
// inverted): the order the key-only sort's dedup takes its run maximum in)
// -- so it needs no order among the key's tuples.  When the key offsets span
// 12..23 bits (config D: 23) the sort is ONE radix pass on the key's top 8
// bits, which leaves each of 256 key buckets contiguous, and one 1024-thread
// workgroup per bucket keeps the max of each of its 2^(bk-8) keys in an LDS
// table (<= 128 KB: one workgroup per CU): an LDS atomicMax per tuple, then
// a walk of the table in key order that stores one tuple per present key at
// its rank -- round-major, so consecutive lanes take consecutive keys and the
// ballot-compacted stores are contiguous per wave.
// A bucket's output offset is the number of present keys in the buckets
// before it.  Each workgroup publishes its own count as soon as its table
// is walked once (an agent-scope store of count | ready) and sums its
// predecessors' (thread d polls bucket d's word): no chain, every count is
// published before its workgroup waits.  Workgroups are dispatched in index
// order, so every polled predecessor has been dispatched; the polls are
// bounded, and a timeout raises CRDT_DEV_LOOKBACK (output invalid) instead
// of hanging.
constexpr int LTB = 1024;                          // threads per bucket workgroup
constexpr int LT_WAVES = LTB / 64;
constexpr uint32_t kLtBytes = 128u * 1024u;        // the LDS table
constexpr unsigned long long kLtReady = 1ull << 32;

__device__ __forceinline__ uint64_t lt_field(uint64_t x, uint32_t s, uint32_t b) {
    return b == 0 ? 0 : (x >> s) & (b >= 64 ? ~0ull : ((1ull << b) - 1ull));
}

template <typename E>
__global__ __launch_bounds__(LTB) void k_lww_table(const uint64_t *__restrict__ c, const SortPlan *__restrict__ plan_,
                                                   const uint32_t *__restrict__ tot,
                                                   unsigned long long *__restrict__ flag, crdt_tuples out,
                                                   uint64_t *__restrict__ out_count, uint32_t *__restrict__ err, PlanGuard pg = {}) {
    constexpr uint32_t NE = kLtBytes / sizeof(E);  // 2^15 u32 / 2^14 u64 entries
    constexpr uint32_t NR = NE / LTB;              // table rounds at most
    static_assert(NR * LT_WAVES <= 64 * 8, "one wave scans the round counts");
    __shared__ E tab[NE];
    __shared__ uint32_t s_cnt[NR * LT_WAVES];      // present keys per (round, wave), then their prefix
    __shared__ unsigned long long s_sum[3];        // bucket start, predecessors' keys, own keys
    const SortPlan p = *plan_;
    if (!plan_guard_ok(p, pg)) return;                 // (uniform: before any barrier)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t b = blockIdx.x, L = p.tl, ne = 1u << L;
    const uint32_t kb = p.b0 + p.br + p.bt;        // tag bits under the key (< 8 * sizeof(E))
    const E marker = (E)1 << kb, tmask = marker - 1;
    if (tid < 3) s_sum[tid] = 0;
    for (uint32_t i = tid; i < ne; i += LTB) tab[i] = 0;
    unsigned long long part = (tid < 256 && (uint32_t)tid < b) ? tot[tid] : 0u;
    for (int o = 32; o >= 1; o >>= 1) part += __shfl_xor(part, o, 64);
    __syncthreads();
    if (lane == 0 && w < 4 && part) atomicAdd(&s_sum[0], part);
    __syncthreads();
    const uint64_t *src = c + s_sum[0];
    const uint32_t nb = tot[b];
    // every tuple of the bucket into its key's entry
    uint32_t j = tid;
    for (; j + 3 * LTB < nb; j += 4 * LTB) {
        uint64_t x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = src[j + k * LTB];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            atomicMax(&tab[(uint32_t)(x[k] >> kb) & (ne - 1)], ((E)(x[k] ^ 3u) & tmask) | marker);
    }
    for (; j < nb; j += LTB) {
        const uint64_t x = src[j];
        atomicMax(&tab[(uint32_t)(x >> kb) & (ne - 1)], ((E)(x ^ 3u) & tmask) | marker);
    }
    __syncthreads();
    // present keys per (round, wave), their exclusive prefix, and the total
    const uint32_t R = (ne + LTB - 1) / LTB, NC = R * LT_WAVES;
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t e = r * LTB + tid;
        const uint64_t m = __ballot(e < ne && tab[e] != 0);
        if (lane == 0) s_cnt[r * LT_WAVES + w] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (w == 0) {
        uint32_t v[8], sum = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t i = lane * 8 + k;
            v[k] = i < NC ? s_cnt[i] : 0u;
            sum += v[k];
        }
        uint32_t x = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        uint32_t run = x - sum;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t i = lane * 8 + k;
            if (i < NC) s_cnt[i] = run;
            run += v[k];
        }
        if (lane == 63) {
            s_sum[2] = x;
            __hip_atomic_store(&flag[b], kLtReady | x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // the predecessors' counts
    unsigned long long pre = 0;
    if ((uint32_t)tid < b) {
        unsigned long long f;
        uint32_t spins = 0;
        while (!((f = __hip_atomic_load(&flag[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) & kLtReady)) {
            if (++spins > (1u << 22)) {            // bounded: report, never hang
                atomicOr(err, CRDT_DEV_LOOKBACK);
                f = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        pre = f & 0xFFFFFFFFull;
    }
    for (int o = 32; o >= 1; o >>= 1) pre += __shfl_xor(pre, o, 64);
    if (lane == 0 && w < 4 && pre) atomicAdd(&s_sum[1], pre);
    __syncthreads();
    const uint64_t off = s_sum[1];
    if (b == gridDim.x - 1 && tid == 0) *out_count = off + s_sum[2];
    // one tuple per present key, in key order
    const uint64_t kbase = (uint64_t)b << L;
    const uint32_t sr = p.b0, st = p.b0 + p.br;
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t e = r * LTB + tid;
        const E v = e < ne ? tab[e] : (E)0;
        const uint64_t m = __ballot(v != 0);
        if (v == 0) continue;
        const size_t o = off + s_cnt[r * LT_WAVES + w] + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        const uint64_t win = (uint64_t)(v & tmask) ^ 3u;
        out.key[o] = p.kmin + (kbase | e);
        out.ts[o] = p.tmin + lt_field(win, st, p.bt);
        out.rep[o] = (uint32_t)(p.rmin + lt_field(win, sr, p.br));
        out.tomb[o] = (uint8_t)(win & 1u);
    }
}

// ---------------------------------------------------------------- LWW D2: bucket tables fed by gathers
// sort.lww_gather (default 1, vector-aligned inputs).  The table form above
// needs each key bucket's composites contiguous, which cost a radix scatter
// pass (composites read and written once more, 320 MB at config D) and its
// column scan.  A bucket's winner is a MAX, so its composites may arrive in
// any order: here the composing pass groups each 4096-tuple tile's
// composites by bucket in LDS (an unstable counting sort) and stores the
// tile in that order, with each (bucket, tile) count and start; the bucket's
// workgroup then gathers its ~16-composite run from every tile -- 16 lanes
// per run, four runs per wave-instruction, so every load is a contiguous
// 128-B piece -- into its LDS table.  No scatter pass, no column scan.
//
// HIST (OR-Set, <= 64 chunks per top byte): also each run's counts by chunk
// (the 6 key bits under the top byte), one byte per chunk, 64 B per run, at
// sh_.rows[(bucket * ntiles + tile) * 16 ..] (u32 words of four byte
// counts): the bucket pass then sums 64-B rows instead of gathering every
// composite once more to count it.  A run of more than 255 composites
// (a byte could wrap) sets sh_.flag[bucket]: that bucket counts by gathers.
struct SubHist {
    uint32_t *rows;
    uint32_t *flag;
};
template <int UB, int TILE, bool HIST = false>
__global__ __launch_bounds__(UB) void k_lww_up_tiled(crdt_tuples in, size_t n, const SortPlan *__restrict__ plan_,
                                                     uint32_t ntiles, uint32_t *__restrict__ run,
                                                     uint64_t *__restrict__ comp, uint32_t *__restrict__ viol,
                                                     unsigned long long *__restrict__ zero, SubHist sh_ = {},
                                                     PlanGuard pg = {}) {
    constexpr int UR = TILE / UB;                     // composites per thread
    static_assert(TILE < 65536, "16-bit run starts and counts");
    __shared__ uint32_t h[256], hs[256];
    __shared__ uint64_t stage[TILE];
    static_assert(!HIST || TILE * 2 >= 256 * 16, "the run counts fit the staging area");
    uint32_t *const hr = reinterpret_cast<uint32_t *>(stage);   // HIST: each run's byte counts by chunk (written
                                                                //   out before the tile is staged)
    const int tid = threadIdx.x;
    if (tid < 256) h[tid] = 0;
    if (HIST)
        for (int i = tid; i < 256 * 16; i += UB) hr[i] = 0;
    if (zero && blockIdx.x == 0 && tid < 256) {       // the buckets' flags (k_lww_table_g, k_or_bucket), the
        zero[tid] = 0;                                //   OR-Set chunks' fallback word
        if (tid == 0) zero[256] = 0;
    }
    const SortPlan p = *plan_;
    if (!plan_guard_ok(p, pg)) return;                 // (uniform: before any barrier)
    const size_t base = (size_t)blockIdx.x * TILE;
    uint64_t c[UR];
    uint32_t vm = 0;                                  // bit r: c[r] holds a tuple (e < n)
    bool bad = false;                                 // (viol) a field outside the plan's ranges
    auto out_of = [&](uint64_t k, uint64_t t, uint32_t r) {
        return outside(k - p.kmin, p.bk) || outside(t - p.tmin, p.bt) || outside((uint64_t)r - p.rmin, p.br);
    };
#pragma unroll
    for (int r = 0; r < UR / 2; ++r) {               // two tuples per lane per round (16-B key / ts loads)
        const size_t e = base + 2 * ((size_t)r * UB + tid);
        c[2 * r] = c[2 * r + 1] = 0;
        if (e >= n) continue;
        vm |= (e + 1 < n ? 3u : 1u) << (2 * r);
        const bool side = e >= p.n1;
        const crdt_tuples &T = side ? p.in2 : in;
        const size_t f = side ? e - p.n1 : e;
        if (e + 1 < n) {
            typedef uint64_t v2u64 __attribute__((ext_vector_type(2)));   // (nontemporal loads: each tuple is read once)
            typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));
            const v2u64 kv = __builtin_nontemporal_load((const v2u64 *)(T.key + f)),
                        tv = __builtin_nontemporal_load((const v2u64 *)(T.ts + f));
            const v2u32 rv = __builtin_nontemporal_load((const v2u32 *)(T.rep + f));
            const ulonglong2 k{kv.x, kv.y}, t{tv.x, tv.y};
            const uint2 rp{rv.x, rv.y};
            const uint16_t tb = __builtin_nontemporal_load((const uint16_t *)(T.tomb + f));
            if (viol) bad = bad || out_of(k.x, t.x, rp.x) || out_of(k.y, t.y, rp.y);
            c[2 * r] = compose<1>(p, k.x, t.x, rp.x, (uint8_t)(tb & 0xFF), side).w[0];
            c[2 * r + 1] = compose<1>(p, k.y, t.y, rp.y, (uint8_t)(tb >> 8), side).w[0];
        } else {
            if (viol) bad = bad || out_of(T.key[f], T.ts[f], T.rep[f]);
            c[2 * r] = compose<1>(p, T.key[f], T.ts[f], T.rep[f], T.tomb[f], side).w[0];
        }
    }
    if (viol && __ballot(bad) && (tid & 63) == 0) atomicOr(viol, 1u);
    __syncthreads();
    const uint32_t sh = p.W - 8;                      // the bucket: the composite's (the key's) top byte
    const uint32_t ssh = p.b0 + p.br + p.bt + 9;      // HIST: the chunk bits under it (as k_or_bucket's sub-bucket)
    const uint32_t smask = (p.bk > 17 ? 1u << (p.bk - 17) : 1u) - 1u;
    uint32_t d[UR];
#pragma unroll
    for (int r = 0; r < UR; ++r) {
        d[r] = ((vm >> r) & 1u) ? (uint32_t)(c[r] >> sh) & 255u : 256u;
        if (d[r] < 256) {
            atomicAdd(&h[d[r]], 1u);
            if (HIST) {
                const uint32_t sb = (uint32_t)(c[r] >> ssh) & smask;   // (<= 63: HIST only for <= 64 chunks)
                atomicAdd(&hr[d[r] * 16 + (sb >> 2)], 1u << (8 * (sb & 3)));
            }
        }
    }
    __syncthreads();
    if (HIST) {                                       // the rows out (16 lanes per 64-B row); wide runs flagged
        for (int i = tid; i < 256 * 16; i += UB)
            sh_.rows[((size_t)(i >> 4) * ntiles + blockIdx.x) * 16 + (i & 15)] = hr[i];
        if (tid < 256 && h[tid] > 255) sh_.flag[tid] = 1;
    }
    if (tid < 64) {                                   // exclusive scan of the 256 bucket counts (wave 0, 4 per lane)
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[k] = h[tid * 4 + k];
            sum += v[k];
        }
        uint32_t y = sum;
#pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) {
            const uint32_t t = __shfl_up(y, dd, 64);
            if (tid >= dd) y += t;
        }
        uint32_t ex = y - sum;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t b = (uint32_t)tid * 4 + k;
            hs[b] = ex;
            run[(size_t)b * ntiles + blockIdx.x] = ex << 16 | v[k];   // (bucket, tile) run: start | count (<= 4096 each)
            ex += v[k];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < UR; ++r)
        if (d[r] < 256) stage[atomicAdd(&hs[d[r]], 1u)] = c[r];
    __syncthreads();
    const uint32_t m = n - base < (size_t)TILE ? (uint32_t)(n - base) : (uint32_t)TILE;
    for (uint32_t i = 2 * tid; i < m; i += 2 * UB) {   // the tile, bucket by bucket (16-B stores)
        if (i + 1 < m) *(ulonglong2 *)(comp + base + i) = ulonglong2{stage[i], stage[i + 1]};
        else comp[base + i] = stage[i];
    }
}

constexpr uint32_t kRunLds = 6144;                 // (bucket, tile) runs staged in LDS (24 KB; config D: 2442 tiles of 8192)
template <typename E, uint32_t GL>
__global__ __launch_bounds__(LTB) void k_lww_table_g(const uint64_t *__restrict__ c, const SortPlan *__restrict__ plan_,
                                                     const uint32_t *__restrict__ run, uint32_t ntiles,
                                                     unsigned long long *__restrict__ flag, crdt_tuples out,
                                                     uint64_t *__restrict__ out_count, uint32_t *__restrict__ err, PlanGuard pg = {}) {
    constexpr uint32_t NE = kLtBytes / sizeof(E);  // 2^15 u32 / 2^14 u64 entries
    constexpr uint32_t NR = NE / LTB;
    static_assert(NR * LT_WAVES <= 64 * 8, "one wave scans the round counts");
    __shared__ E tab[NE];
    __shared__ uint32_t s_run[kRunLds];
    __shared__ uint32_t s_cnt[NR * LT_WAVES];
    __shared__ unsigned long long s_sum[3];
    const SortPlan p = *plan_;
    if (!plan_guard_ok(p, pg)) return;                 // (uniform: before any barrier)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t b = blockIdx.x, L = p.tl, ne = 1u << L;
    const uint32_t kb = p.b0 + p.br + p.bt;
    const E marker = (E)1 << kb, tmask = marker - 1;
    if (tid < 3) s_sum[tid] = 0;
    for (uint32_t i = tid; i < ne; i += LTB) tab[i] = 0;
    const uint32_t *rg = run + (size_t)b * ntiles;    // this bucket's run in every tile
    const bool lds = ntiles <= kRunLds;
    if (lds)
        for (uint32_t i = tid; i < ntiles; i += LTB) s_run[i] = rg[i];
    __syncthreads();
    // lane group g (16 lanes) takes KT tiles per iteration, t = t0 + g +
    // 64 k, its lanes elements l + 16 j (j < GL) of each run: 8 loads in
    // flight per lane, every load instruction four contiguous 128-B pieces
    // (GL = 2: 4096-tuple tiles, runs of ~16; GL = 4: 8192, runs of ~32)
    constexpr uint32_t KT = 8 / GL, NG = 4 * LT_WAVES;  // tiles per group per iteration, lane groups
    constexpr uint32_t TILE = 2048 * GL;
    const uint32_t g = (uint32_t)tid >> 4, l = (uint32_t)lane & 15;
    auto put = [&](uint64_t x) { atomicMax(&tab[(uint32_t)(x >> kb) & (ne - 1)], ((E)(x ^ 3u) & tmask) | marker); };
    for (uint32_t t0 = 0; t0 < ntiles; t0 += NG * KT) {
        uint32_t rn[KT];
        const uint64_t *rp[KT];
#pragma unroll
        for (uint32_t k = 0; k < KT; ++k) {
            const uint32_t t = t0 + g + NG * k;
            rn[k] = t < ntiles ? (lds ? s_run[t] : rg[t]) : 0u;
            rp[k] = c + (size_t)t * TILE + (rn[k] >> 16);
            rn[k] &= 0xFFFFu;
        }
        uint64_t x[GL * KT];
#pragma unroll
        for (uint32_t k = 0; k < KT; ++k)
#pragma unroll
            for (uint32_t j = 0; j < GL; ++j) x[GL * k + j] = l + 16 * j < rn[k] ? rp[k][l + 16 * j] : 0;
#pragma unroll
        for (uint32_t k = 0; k < KT; ++k) {
#pragma unroll
            for (uint32_t j = 0; j < GL; ++j)
                if (l + 16 * j < rn[k]) put(x[GL * k + j]);
            for (uint32_t i = l + 16 * GL; i < rn[k]; i += 16) put(rp[k][i]);   // (rare: longer runs)
        }
    }
    __syncthreads();
    // present keys per (round, wave), their exclusive prefix, and the total
    const uint32_t R = (ne + LTB - 1) / LTB, NC = R * LT_WAVES;
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t e = r * LTB + tid;
        const uint64_t m = __ballot(e < ne && tab[e] != 0);
        if (lane == 0) s_cnt[r * LT_WAVES + w] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (w == 0) {
        uint32_t v[8], sum = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t i = lane * 8 + k;
            v[k] = i < NC ? s_cnt[i] : 0u;
            sum += v[k];
        }
        uint32_t x = sum;
#pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) {
            const uint32_t y = __shfl_up(x, dd, 64);
            if (lane >= dd) x += y;
        }
        uint32_t run = x - sum;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t i = lane * 8 + k;
            if (i < NC) s_cnt[i] = run;
            run += v[k];
        }
        if (lane == 63) {
            s_sum[2] = x;
            __hip_atomic_store(&flag[b], kLtReady | x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // the predecessors' counts (as k_lww_table: every count is published before its workgroup waits)
    unsigned long long pre = 0;
    if ((uint32_t)tid < b) {
        unsigned long long f;
        uint32_t spins = 0;
        while (!((f = __hip_atomic_load(&flag[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) & kLtReady)) {
            if (++spins > (1u << 22)) {            // bounded: report, never hang
                atomicOr(err, CRDT_DEV_LOOKBACK);
                f = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        pre = f & 0xFFFFFFFFull;
    }
    for (int o = 32; o >= 1; o >>= 1) pre += __shfl_xor(pre, o, 64);
    if (lane == 0 && w < 4 && pre) atomicAdd(&s_sum[1], pre);
    __syncthreads();
    const uint64_t off = s_sum[1];
    if (b == gridDim.x - 1 && tid == 0) *out_count = off + s_sum[2];
    const uint64_t kbase = (uint64_t)b << L;
    const uint32_t sr = p.b0, st = p.b0 + p.br;
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t e = r * LTB + tid;
        const E v = e < ne ? tab[e] : (E)0;
        const uint64_t m = __ballot(v != 0);
        if (v == 0) continue;
        const size_t o = off + s_cnt[r * LT_WAVES + w] + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        const uint64_t win = (uint64_t)(v & tmask) ^ 3u;
        out.key[o] = p.kmin + (kbase | e);
        out.ts[o] = p.tmin + lt_field(win, st, p.bt);
        out.rep[o] = (uint32_t)(p.rmin + lt_field(win, sr, p.br));
        out.tomb[o] = (uint8_t)(win & 1u);
    }
}

// OR-Set D2 without radix passes (sort.or_bucket): the composing pass groups
// each tile by the key's top byte T (k_lww_up_tiled); one 1024-thread
// workgroup per T then gathers T's runs from every tile TWICE -- first to
// count them by the chunk-id bits under T (chunks of 2^9 keys: 2^(bk-17)
// per T), then to place each into its chunk's contiguous range of T's
// region (LDS cursors; any order within a chunk: the chunk kernel sorts
// it) -- and writes the chunk bounds.  T's region starts after the regions
// of T' < T: each workgroup publishes its total and sums its predecessors'
// (all 256 are co-resident; polls bounded).  Replaces two radix passes
// (upsweep, column scan, scatter each) and the chunk-bounds search.
constexpr int OBB = 1024;                          // threads per bucket workgroup
constexpr int OB_WAVES = OBB / 64;
constexpr uint32_t kObSub = 256;                   // chunks per top-byte bucket at most (bk <= 25)
constexpr uint32_t kObLoads = 12;                  // gathered elements per lane per round (KT tiles x GL)
constexpr uint32_t kObBatch = 4 * OB_WAVES * kObLoads * 16;   // a placement round's tuples at most (16 lanes per group)
template <uint32_t GL>
__global__ __launch_bounds__(OBB) void k_or_bucket(const uint64_t *__restrict__ c, const SortPlan *__restrict__ plan_,
                                                   const uint32_t *__restrict__ run, uint32_t ntiles, size_t n,
                                                   unsigned long long *__restrict__ flag, uint64_t *__restrict__ dst,
                                                   uint64_t *__restrict__ bounds, unsigned long long *__restrict__ cst,
                                                   uint32_t nch, uint32_t *__restrict__ err, int diag_,
                                                   bool place_batch, SubHist shist, PlanGuard pg = {}) {
    const int diag = kDiagBuild ? diag_ : 0;          // (the product build has no timing diagnostics)
    __shared__ uint32_t s_run[kRunLds];
    __shared__ uint32_t s_h[OB_WAVES][kObSub];        // per-wave counts by sub-bucket, then the cursors (row 0)
    __shared__ uint64_t s_buf[kObBatch];              // (batched placement) one round's tuples by sub-bucket
    __shared__ uint32_t s_nb;
    __shared__ unsigned long long s_sum[3];
    const SortPlan p = *plan_;
    if (!plan_guard_ok(p, pg)) return;                 // (uniform: before any barrier)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t T = blockIdx.x;
    const uint32_t kb = p.b0 + p.br + p.bt;           // the key's bits start here
    const uint32_t s6 = p.bk > 17 ? p.bk - 17 : 0;    // chunk-id bits under the top byte
    const uint32_t nsub = 1u << s6, ssh = kb + 9;     // sub-bucket = (x >> ssh) & (nsub - 1)
    const uint32_t *rg = run + (size_t)T * ntiles;
    const bool lds = ntiles <= kRunLds;
    if (tid < 3) s_sum[tid] = 0;
    for (uint32_t i = tid; i < OB_WAVES * kObSub; i += OBB) (&s_h[0][0])[i] = 0;
    unsigned long long tot = 0;                       // this bucket's tuples
    for (uint32_t i = tid; i < ntiles; i += OBB) {
        const uint32_t r = rg[i];
        if (lds) s_run[i] = r;
        tot += r & 0xFFFFu;
    }
    for (int o = 32; o >= 1; o >>= 1) tot += __shfl_xor(tot, o, 64);
    __syncthreads();
    if (lane == 0 && tot) atomicAdd(&s_sum[2], tot);
    __syncthreads();
    if (tid == 0) __hip_atomic_store(&flag[T], kLtReady | s_sum[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // gather the runs (as k_lww_table_g: 16-lane groups, KT tiles each per round, GL elements per lane per tile)
    constexpr uint32_t KT = kObLoads / GL, NG = 4 * OB_WAVES;
    constexpr uint32_t TILE = 2048 * GL;
    const uint32_t g = (uint32_t)tid >> 4, l = (uint32_t)lane & 15;
    auto load = [&](uint32_t t0, uint32_t *rn, const uint64_t **rp, uint64_t *x) {
#pragma unroll
        for (uint32_t k = 0; k < KT; ++k) {
            const uint32_t t = t0 + g + NG * k;
            rn[k] = t < ntiles ? (lds ? s_run[t] : rg[t]) : 0u;
            rp[k] = c + (size_t)t * TILE + (rn[k] >> 16);
            rn[k] &= 0xFFFFu;
        }
#pragma unroll
        for (uint32_t k = 0; k < KT; ++k)
#pragma unroll
            for (uint32_t j = 0; j < GL; ++j) x[GL * k + j] = l + 16 * j < rn[k] ? rp[k][l + 16 * j] : 0;
    };
    auto sweep = [&](auto &&put) {
        for (uint32_t t0 = 0; t0 < ntiles; t0 += NG * KT) {
            uint32_t rn[KT];
            const uint64_t *rp[KT];
            uint64_t x[GL * KT];
            load(t0, rn, rp, x);
#pragma unroll
            for (uint32_t k = 0; k < KT; ++k) {
#pragma unroll
                for (uint32_t j = 0; j < GL; ++j)
                    if (l + 16 * j < rn[k]) put(x[GL * k + j]);
                for (uint32_t i = l + 16 * GL; i < rn[k]; i += 16) put(rp[k][i]);   // (rare: longer runs)
            }
        }
    };
    // 1. counts by sub-bucket: from the grouping pass's per-run chunk counts
    // (shist: four lanes per 64-B row, sixteen byte counts each), else by a
    // gather of every run (a row per wave: fewer same-address LDS atomics)
    bool rows = shist.rows != nullptr && nsub <= 64;
    if (rows) {
        rows = shist.flag[T] == 0;                    // (uniform) no run of T over 255
        __syncthreads();                              // (every lane has read the flag)
        if (tid == 0) shist.flag[T] = 0;              // clean for the next call
    }
    if (rows) {
        const uint32_t q = (uint32_t)tid & 3;
        uint32_t cnt[16] = {};
        const uint4 *rp4 = (const uint4 *)shist.rows + (size_t)T * ntiles * 4;
        for (uint32_t t = (uint32_t)tid >> 2; t < ntiles; t += OBB / 4) {
            const uint4 v = rp4[(size_t)t * 4 + q];
            const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 16; ++j) cnt[j] += (wv[j >> 2] >> (8 * (j & 3))) & 255u;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if (cnt[j]) atomicAdd(&s_h[w][16 * q + j], cnt[j]);
    } else {
        sweep([&](uint64_t x) { atomicAdd(&s_h[w][(uint32_t)(x >> ssh) & (nsub - 1)], 1u); });
    }
    // the predecessors' totals (every bucket published its own above)
    unsigned long long pre = 0;
    if ((uint32_t)tid < T) {
        unsigned long long f;
        uint32_t spins = 0;
        while (!((f = __hip_atomic_load(&flag[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) & kLtReady)) {
            if (++spins > (1u << 22)) {            // bounded: report, never hang
                atomicOr(err, CRDT_DEV_LOOKBACK);
                f = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        pre = f & 0xFFFFFFFFull;
    }
    for (int o = 32; o >= 1; o >>= 1) pre += __shfl_xor(pre, o, 64);
    __syncthreads();                                  // every wave's counts
    if (lane == 0 && w < 4 && pre) atomicAdd(&s_sum[1], pre);
    if (w == 0) {                                     // sub-bucket totals -> exclusive prefix -> cursors (row 0)
        uint32_t v[kObSub / 64], sum = 0;
#pragma unroll
        for (uint32_t k = 0; k < kObSub / 64; ++k) {
            const uint32_t b = (uint32_t)lane * (kObSub / 64) + k;
            uint32_t t = 0;
            for (int q = 0; q < OB_WAVES; ++q) t += s_h[q][b];
            v[k] = t;
            sum += t;
        }
        uint32_t x = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        uint32_t run0 = x - sum;
#pragma unroll
        for (uint32_t k = 0; k < kObSub / 64; ++k) {
            s_h[0][(uint32_t)lane * (kObSub / 64) + k] = run0;
            run0 += v[k];
        }
    }
    __syncthreads();
    const uint64_t base = s_sum[1];
    // the chunk bounds (chunk = 2^9 keys: sub-buckets of T, or runs of 2^(17 - bk) buckets) and
    // the chunk kernel's look-back words
    if (s6 > 0 || (T & ((1u << (17 - p.bk)) - 1u)) == 0) {
        for (uint32_t b = tid; b < nsub; b += OBB) {
            const uint32_t ch = s6 > 0 ? (T << s6) + b : T >> (17 - p.bk);
            bounds[ch] = base + s_h[0][b];
            if (cst) cst[ch] = 0;
        }
    }
    if (T == gridDim.x - 1 && tid == 0) bounds[nch] = n;
    __syncthreads();
    // 2. each tuple into its chunk's range of T's region (any order within it)
    uint64_t *out = dst + base;
    if (diag == 8) return;                            // (timing only: the chunk ranges left unfilled)
    if (diag == 7) {                                  // (timing only: placement ranks, no stores)
        sweep([&](uint64_t x) { atomicAdd(&s_h[0][(uint32_t)(x >> ssh) & (nsub - 1)], 1u); });
        return;
    }
    if (!place_batch) {
        sweep([&](uint64_t x) { out[atomicAdd(&s_h[0][(uint32_t)(x >> ssh) & (nsub - 1)], 1u)] = x; });
        return;
    }
    // batched placement (sort.or_place_batch): a round's tuples (256 runs)
    // ranked per sub-bucket in LDS (row 1 of s_h), the round's ranges
    // reserved from the cursors (row 0) by one wave, the tuples sorted by
    // sub-bucket in s_buf, then stored in order -- each sub-bucket's part one
    // contiguous piece of its chunk range (one-by-one 8-B stores to 64
    // ranges cost 65 of the pass's 153 us).  Row 2: the round's offsets in
    // s_buf, row 3: its bases in the chunk ranges.  Tuples past 32 in a run
    // (rare) are placed one by one from the cursors directly.  (Issuing the
    // next round's loads before this round's stores: no faster.)
    uint32_t *bc = s_h[1], *bo = s_h[2], *gb = s_h[3];
    for (uint32_t i = tid; i < kObSub; i += OBB) bc[i] = 0;
    __syncthreads();
    for (uint32_t t0 = 0; t0 < ntiles; t0 += NG * KT) {
        uint32_t rn[KT], rk[GL * KT];
        const uint64_t *rp[KT];
        uint64_t x[GL * KT];
        load(t0, rn, rp, x);
#pragma unroll
        for (uint32_t k = 0; k < KT; ++k) {
#pragma unroll
            for (uint32_t j = 0; j < GL; ++j)
                if (l + 16 * j < rn[k]) rk[GL * k + j] = atomicAdd(&bc[(uint32_t)(x[GL * k + j] >> ssh) & (nsub - 1)], 1u);
            for (uint32_t i = l + 16 * GL; i < rn[k]; i += 16) {   // (rare: longer runs)
                const uint64_t y = rp[k][i];
                out[atomicAdd(&s_h[0][(uint32_t)(y >> ssh) & (nsub - 1)], 1u)] = y;
            }
        }
        __syncthreads();
        if (w == 0) {                                 // the round's counts -> offsets in s_buf, ranges reserved
            uint32_t v[kObSub / 64], sum = 0;
#pragma unroll
            for (uint32_t k = 0; k < kObSub / 64; ++k) {
                const uint32_t b = (uint32_t)lane * (kObSub / 64) + k;
                v[k] = b < nsub ? bc[b] : 0u;
                sum += v[k];
            }
            uint32_t y = sum;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t t = __shfl_up(y, d, 64);
                if (lane >= d) y += t;
            }
            uint32_t o = y - sum;
#pragma unroll
            for (uint32_t k = 0; k < kObSub / 64; ++k) {
                const uint32_t b = (uint32_t)lane * (kObSub / 64) + k;
                if (b < nsub) {
                    bo[b] = o;
                    gb[b] = s_h[0][b];
                    s_h[0][b] += v[k];
                    bc[b] = 0;
                }
                o += v[k];
            }
            if (lane == 63) s_nb = y;                 // the round's tuples
        }
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < KT; ++k)
#pragma unroll
            for (uint32_t j = 0; j < GL; ++j)
                if (l + 16 * j < rn[k])
                    s_buf[bo[(uint32_t)(x[GL * k + j] >> ssh) & (nsub - 1)] + rk[GL * k + j]] = x[GL * k + j];
        __syncthreads();
        const uint32_t nb = s_nb;
        for (uint32_t i = tid; i < nb; i += OBB) {
            const uint64_t y = s_buf[i];
            const uint32_t b = (uint32_t)(y >> ssh) & (nsub - 1);
            out[gb[b] + (i - bo[b])] = y;
        }
    }
}

// ---------------------------------------------------------------- OR-Set D2: key chunks sorted in LDS
// sort.or_table (default 1).  The radix sort runs only TWO passes, on the
// key's top 16 bits; the key space is then cut into chunks of 2^9 keys
// (config D: 16384 chunks of ~1.2k tuples), each contiguous in the sorted
// composites because a chunk is a run of top-16 buckets.  Per chunk, one
// 512-thread workgroup holds the chunk in LDS and finishes the sort there:
//   k_chunk_bounds: the chunk starts, one 64-ary search per chunk;
//   k_or_chunk: the chunk's tuples into registers, a counting sort by key
//     into LDS (count per key, scan, scatter by LDS atomics), then one thread
//     per key finds the key's distinct tags -- a key of <= kOtRun tuples
//     sorted in registers by a sorting network, <= kOtMid by an insertion
//     sort of its own slots in LDS, a longer key by the whole workgroup
//     (first-copy marks in LDS, ranks by counting) -- and places them in tag
//     order, tomb = the OR of the tag's copies, as composites (side bit
//     cleared) in LDS; then (sort.or_lookback, default) finds the chunk's
//     output offset by a decoupled look-back and stores the SoA output
//     itself, or copies the composites to the chunk's own input range of
//     `tmp` with the chunk's count, for
//   k_sort_colscan over the chunk counts and
//   k_or_emit: each chunk's tags decoded into the SoA output at its offset.
// A chunk of more than kOcCap tuples (skewed keys) or of more than kOcLong
// keys with over kOtMid tuples raises the fallback word and stores nothing;
// the host then runs the radix path (inputs untouched).
// (Round 4, first form: one radix pass on the key's top byte and a counting
// sort of each 78k-tuple bucket through global memory -- its scattered 8-B
// stores over 256 x 625 KB alone took 375 us)
constexpr int OCB = 512;                 // threads per chunk workgroup
constexpr int OC_WAVES = OCB / 64;
constexpr uint32_t kOcBits = 9;          // keys per chunk: 2^9
constexpr uint32_t kOcKeys = 1u << kOcBits;
constexpr uint32_t kOcCap = 1536;        // tuples per chunk (LDS); more -> fallback
constexpr uint32_t kOcPer = kOcCap / OCB;
constexpr uint32_t kOtRun = 8;           // keys of up to this many tuples: one thread, registers
constexpr uint32_t kOtMid = 32;          // up to this many: one thread, an insertion sort of its slots in LDS
constexpr uint32_t kOcLong = 64;         // longer keys per chunk (LDS list); more -> fallback

// a key's <= kOtRun tuples sorted in registers (Batcher's 19-comparator
// network; unused slots hold ~0 and sort last), so its distinct tags are the
// slots whose tag differs from the previous slot's -- the first copy of each
// tag its smallest composite.  (Pairwise first-copy tests and ranks over all
// slots, 8 x 8 64-bit compares per key twice, made the pass VALU-bound: 428 us.)
__device__ __forceinline__ void ot_cswap(uint64_t &a, uint64_t &b) {
    const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
    a = lo;
    b = hi;
}
__device__ __forceinline__ void ot_sort8(uint64_t *v) {
    ot_cswap(v[0], v[1]); ot_cswap(v[2], v[3]); ot_cswap(v[4], v[5]); ot_cswap(v[6], v[7]);
    ot_cswap(v[0], v[2]); ot_cswap(v[1], v[3]); ot_cswap(v[4], v[6]); ot_cswap(v[5], v[7]);
    ot_cswap(v[1], v[2]); ot_cswap(v[5], v[6]);
    ot_cswap(v[0], v[4]); ot_cswap(v[1], v[5]); ot_cswap(v[2], v[6]); ot_cswap(v[3], v[7]);
    ot_cswap(v[2], v[4]); ot_cswap(v[3], v[5]);
    ot_cswap(v[1], v[2]); ot_cswap(v[3], v[4]); ot_cswap(v[5], v[6]);
}
// the same on the low 32 bits, when every tag bit lies below bit 32 (kb <=
// 32: the bits above are the key's, equal over a key's slots) -- u32 min /
// max instead of 64-bit compares and selects
__device__ __forceinline__ void ot_cswap32(uint32_t &a, uint32_t &b) {
    const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
    a = lo;
    b = hi;
}
__device__ __forceinline__ void ot_sort8_32(uint32_t *v) {
    ot_cswap32(v[0], v[1]); ot_cswap32(v[2], v[3]); ot_cswap32(v[4], v[5]); ot_cswap32(v[6], v[7]);
    ot_cswap32(v[0], v[2]); ot_cswap32(v[1], v[3]); ot_cswap32(v[4], v[6]); ot_cswap32(v[5], v[7]);
    ot_cswap32(v[1], v[2]); ot_cswap32(v[5], v[6]);
    ot_cswap32(v[0], v[4]); ot_cswap32(v[1], v[5]); ot_cswap32(v[2], v[6]); ot_cswap32(v[3], v[7]);
    ot_cswap32(v[2], v[4]); ot_cswap32(v[3], v[5]);
    ot_cswap32(v[1], v[2]); ot_cswap32(v[3], v[4]); ot_cswap32(v[5], v[6]);
}
__device__ __forceinline__ uint32_t ot_firsts32(const uint32_t *v, uint32_t m, uint32_t tb) {
    uint32_t fm = m ? 1u : 0u;
#pragma unroll
    for (uint32_t j = 1; j < kOtRun; ++j) fm |= (j < m && (v[j] >> tb) != (v[j - 1] >> tb)) ? 1u << j : 0u;
    return fm;
}

// bit j: slot j (< m) starts a tag in the sorted slots
__device__ __forceinline__ uint32_t ot_firsts(const uint64_t *v, uint32_t m, uint32_t tb) {
    uint32_t fm = m ? 1u : 0u;
#pragma unroll
    for (uint32_t j = 1; j < kOtRun; ++j) fm |= (j < m && (v[j] >> tb) != (v[j - 1] >> tb)) ? 1u << j : 0u;
    return fm;
}

// bounds[i] = first composite of chunk i (0 < i < nch; bounds[0] = 0,
// bounds[nch] = n): a 64-ary search per chunk over the chunk index c >> cs,
// non-decreasing in the sorted composites (every index probed once the span
// is <= 64)
__global__ __launch_bounds__(256) void k_chunk_bounds(const uint64_t *__restrict__ c, size_t n, uint32_t cs,
                                                      uint32_t nch, uint64_t *__restrict__ bounds,
                                                      unsigned long long *__restrict__ st) {
    const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);      // one wave per bound
    const int lane = threadIdx.x & 63;
    if (i > nch) return;
    if (st && i < nch && lane == 0) st[i] = 0;        // k_or_chunk<true>'s look-back words
    if (i == 0 || i == nch) {
        if (lane == 0) bounds[i] = i == 0 ? 0 : n;
        return;
    }
    size_t lo = 0, hi = n;                            // the answer lies in [lo, hi]
    while (lo < hi) {
        const size_t span = hi - lo;
        const size_t q = lo + span * (size_t)lane / 64;
        const uint64_t ge = __ballot((c[q] >> cs) >= i);
        if (ge == 0) {
            lo += span * 63 / 64 + 1;
        } else {
            const int t = __ffsll((long long)ge) - 1;
            hi = lo + span * (size_t)t / 64;
            if (t > 0) lo += span * (size_t)(t - 1) / 64 + 1;
        }
    }
    if (lane == 0) bounds[i] = lo;
}

// LB (sort.or_lookback): the chunk finds its output offset itself by a
// decoupled look-back over the chunks before it and stores the SoA output
// directly (no tmp round trip, no scan, no emit).  Status word per chunk:
// kOcA | count once counted, kOcP | inclusive prefix once resolved; wave 0
// reads 64 predecessors per poll, nearest first, and sums back to the
// nearest resolved one.  Chunks are dispatched in index order, so every
// polled chunk has been dispatched; polls are bounded (CRDT_DEV_LOOKBACK).
// K (sort.or_pair): chunks per workgroup.  K = 2 processes two consecutive
// chunks in turn, each into its own LDS output buffer, and looks back ONCE,
// for the first, after both are placed -- by then its predecessors have had
// a whole chunk's time to publish -- then stores both (the second's offset
// is the first's plus its count).
// (wave-uniform returns / continues only: every barrier below is reached by
// the whole workgroup or by none of it)
template <bool LB, bool NARROW, int K>
__global__ __launch_bounds__(OCB) __attribute__((amdgpu_waves_per_eu(8))) void k_or_chunk(const uint64_t *__restrict__ c, uint64_t *__restrict__ tmp,
                                                  const SortPlan *__restrict__ plan_,
                                                  const uint64_t *__restrict__ bounds, uint32_t *__restrict__ cnt,
                                                  uint32_t *__restrict__ fbw, int diag_,
                                                  unsigned long long *__restrict__ st, crdt_tuples out,
                                                  uint64_t *__restrict__ out_count, uint32_t *__restrict__ err,
                                                  uint32_t nch, PlanGuard pg = {}) {
    constexpr uint32_t R = kOcKeys / OCB;             // keys per thread (round-major)
    __shared__ uint32_t tab[kOcKeys];
    __shared__ uint64_t stg[kOcCap];
    __shared__ uint64_t ostb[K][kOcCap];              // each chunk's tags in order (one coalesced copy out)
    __shared__ uint32_t s_first[kOcCap / 32];         // a long key's first-copy marks
    __shared__ uint32_t s_cnt[R * OC_WAVES], s_wsum[OC_WAVES], s_long[kOcLong], s_lrk[kOcLong], s_nlong, s_totk[K];
    __shared__ unsigned long long s_off;
    const SortPlan p = *plan_;
    if (!plan_guard_ok(p, pg)) return;                 // (uniform: before any barrier)
    const int diag = kDiagBuild ? diag_ : 0;          // (the product build has no timing diagnostics)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t kb = p.b0 + p.br + p.bt, tb = p.b0;
    bool fb = false;                                  // (uniform) a chunk of this workgroup fell back
    bool stop = false;                                // (timing diagnostics 1..4: every chunk stops at that phase)
    for (int kk = 0; kk < K; ++kk) {
    const uint32_t ci = blockIdx.x * K + (uint32_t)kk;
    uint64_t *ost = ostb[kk];
    const size_t s = bounds[ci], e = bounds[ci + 1];
    if (e - s > kOcCap) {                             // skewed keys: the radix path instead
        if (tid == 0) {
            atomicOr(fbw, 1u);
            cnt[ci] = 0;
            if (LB) __hip_atomic_store(&st[ci], kOcA, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        fb = true;
        continue;
    }
    const uint32_t len = (uint32_t)(e - s);
    __syncthreads();                                  // (the previous chunk's LDS reads are done)
    for (uint32_t i = tid; i < kOcKeys; i += OCB) tab[i] = 0;
    for (uint32_t i = tid; i < kOcCap / 32; i += OCB) s_first[i] = 0;
    if (tid == 0) s_nlong = 0;
    uint64_t x[kOcPer];
#pragma unroll
    for (uint32_t k = 0; k < kOcPer; ++k) {
        const uint32_t j = k * OCB + tid;
        x[k] = j < len ? c[s + j] : 0;
    }
    __syncthreads();
    // counting sort by key into LDS
#pragma unroll
    for (uint32_t k = 0; k < kOcPer; ++k)
        if (k * OCB + tid < len) atomicAdd(&tab[(uint32_t)(x[k] >> kb) & (kOcKeys - 1)], 1u);
    __syncthreads();
    if (diag == 1) {                                  // timing diagnostics (sort.rdd_diag): counts only
        if (tid == 0) cnt[ci] = 0;
        stop = true;
        continue;
    }
    {                                                 // exclusive scan: wave w the contiguous entries [w P, (w+1) P)
        constexpr uint32_t P = kOcKeys / OC_WAVES;
        uint32_t carry = 0;
#pragma unroll
        for (uint32_t e0 = 0; e0 < P; e0 += 64) {
            const uint32_t i = (uint32_t)w * P + e0 + (uint32_t)lane;
            const uint32_t v = tab[i];
            uint32_t y = v;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t t = __shfl_up(y, d, 64);
                if (lane >= d) y += t;
            }
            tab[i] = carry + y - v;
            carry += (uint32_t)__shfl((int)y, 63, 64);
        }
        if (lane == 0) s_wsum[w] = carry;
        __syncthreads();
        uint32_t woff = 0;
        for (int k = 0; k < w; ++k) woff += s_wsum[k];
#pragma unroll
        for (uint32_t e0 = 0; e0 < P; e0 += 64) tab[(uint32_t)w * P + e0 + (uint32_t)lane] += woff;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kOcPer; ++k)
        if (k * OCB + tid < len) stg[atomicAdd(&tab[(uint32_t)(x[k] >> kb) & (kOcKeys - 1)], 1u)] = x[k];
    __syncthreads();                                  // tab[k] = the end of key k
    if (diag == 2) {                                  // + the scan and the scatter into LDS
        if (tid == 0) cnt[ci] = 0;
        stop = true;
        continue;
    }
    // distinct tags per key (long keys listed, resolved below); each short
    // key's slots stay sorted in registers for the stores
    // (NARROW: kb <= 32, every tag bit in the low word -- the key's slots are
    // sorted on their low words, the high word kept once per key)
    uint32_t dk[R], fk[R];
    uint64_t sv[NARROW ? 1 : R][NARROW ? 1 : kOtRun];
    uint32_t sl[NARROW ? R : 1][NARROW ? kOtRun : 1], sh[NARROW ? R : 1];
    auto slot = [&](uint32_t r, uint32_t j) -> uint64_t {   // slot j of key r's sorted slots (the full composite)
        if constexpr (NARROW) return (uint64_t)sh[r] << 32 | sl[r][j];
        else return sv[r][j];
    };
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t kl = r * OCB + tid;
        const uint32_t s0 = kl ? tab[kl - 1] : 0u, m = tab[kl] - s0;
        const uint32_t ms = m <= kOtRun ? m : 0u;
        if constexpr (NARROW) {
#pragma unroll
            for (uint32_t k = 0; k < kOtRun; ++k) {
                const uint64_t v = k < ms ? stg[s0 + k] : ~0ull;
                sl[r][k] = (uint32_t)v;
                if (k == 0) sh[r] = (uint32_t)(v >> 32);
            }
            if (ms > 1) ot_sort8_32(sl[r]);
            fk[r] = ot_firsts32(sl[r], ms, tb);
        } else {
#pragma unroll
            for (uint32_t k = 0; k < kOtRun; ++k) sv[r][k] = k < ms ? stg[s0 + k] : ~0ull;
            if (ms > 1) ot_sort8(sv[r]);
            fk[r] = ot_firsts(sv[r], ms, tb);
        }
        dk[r] = (uint32_t)__popc(fk[r]);
        if (m > kOtMid) {
            const uint32_t q = atomicAdd(&s_nlong, 1u);
            if (q < kOcLong) s_long[q] = kl;
        } else if (m > kOtRun) {                      // (rare: a wave with such a key waits for it)
            for (uint32_t i = 1; i < m; ++i) {
                const uint64_t xv = stg[s0 + i];
                uint32_t j = i;
                for (; j > 0 && stg[s0 + j - 1] > xv; --j) stg[s0 + j] = stg[s0 + j - 1];
                stg[s0 + j] = xv;
            }
            uint32_t d = 1;
            for (uint32_t i = 1; i < m; ++i) d += (stg[s0 + i] >> tb) != (stg[s0 + i - 1] >> tb) ? 1u : 0u;
            dk[r] = d;
        }
    }
    __syncthreads();
    const uint32_t nl = s_nlong;
    if (diag == 3) {                                  // + the short keys' distinct tags
        if (tid == 0) cnt[ci] = 0;
        stop = true;
        continue;
    }
    if (nl > kOcLong) {                               // (uniform) too many long keys: the radix path
        if (tid == 0) {
            atomicOr(fbw, 1u);
            cnt[ci] = 0;
            if (LB) __hip_atomic_store(&st[ci], kOcA, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        fb = true;
        continue;
    }
    for (uint32_t q = 0; q < nl; ++q) {               // a long key: first-copy marks, their count to its owner
        const uint32_t kl = s_long[q];
        const uint32_t s0 = kl ? tab[kl - 1] : 0u, m = tab[kl] - s0;
        uint32_t f = 0;
        for (uint32_t i = tid; i < m; i += OCB) {
            const uint64_t xi = stg[s0 + i];
            bool first = true;
            for (uint32_t k = 0; k < m && first; ++k) {
                const uint64_t y = stg[s0 + k];
                if (k != i && (y >> tb) == (xi >> tb) && (y < xi || (y == xi && k < i))) first = false;
            }
            if (first) atomicOr(&s_first[(s0 + i) >> 5], 1u << ((s0 + i) & 31));
            f += first ? 1u : 0u;
        }
        for (int o = 32; o >= 1; o >>= 1) f += __shfl_xor(f, o, 64);
        if (lane == 0) s_wsum[w] = f;
        __syncthreads();
        if ((uint32_t)tid == kl % OCB) {
            uint32_t t = 0;
            for (int k = 0; k < OC_WAVES; ++k) t += s_wsum[k];
#pragma unroll
            for (uint32_t r = 0; r < R; ++r)
                if (r == kl / OCB) dk[r] = t;
        }
        __syncthreads();
    }
    // ranks: per (round, wave) sums, their prefix, in-wave prefixes
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
        uint32_t d = dk[r];
        for (int o = 32; o >= 1; o >>= 1) d += __shfl_xor(d, o, 64);
        if (lane == 0) s_cnt[r * OC_WAVES + w] = d;
    }
    __syncthreads();
    if (w == 0) {
        constexpr uint32_t NC = R * OC_WAVES;
        static_assert(NC <= 64, "one wave");
        const uint32_t c0 = lane < (int)NC ? s_cnt[lane] : 0u;
        uint32_t y = c0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(y, o, 64);
            if (lane >= o) y += t;
        }
        if (lane < (int)NC) s_cnt[lane] = y - c0;
        if (lane == 63) {
            cnt[ci] = y;
            s_totk[kk] = y;
            if (LB)                                   // counted: published at once
                __hip_atomic_store(&st[ci], (ci ? kOcA : kOcP) | y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    if (diag == 4) {                                  // + the long keys and the ranks
        if (tid == 0) cnt[ci] = 0;
        stop = true;
        continue;
    }
    // LB: the offset -- the counts of the chunks before this one -- found by
    // wave 0 while the other waves place their keys' tags (the barrier after
    // the placement joins them)
    if (K == 1 && LB && w == 0 && diag == 6 && lane == 0) s_off = s;   // (timing only: no look-back, a fake offset)
    if (K == 1 && LB && w == 0 && diag != 6) {
        const uint32_t nt0 = s_totk[0];
        unsigned long long acc = 0;
        if (ci > 0) {
            acc = lookback_sum<1>(st, (long long)ci - 1, lane, err);
            if (lane == 0)
                __hip_atomic_store(&st[ci], kOcP | (acc + nt0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            s_off = acc;
            if (ci == nch - 1) *out_count = acc + nt0;
        }
    }
    // placement: composites with the side bit cleared and the tomb = the OR of the tag's copies
    const uint64_t keep = ~3ull;
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t kl = r * OCB + tid;
        const uint32_t s0 = kl ? tab[kl - 1] : 0u, m = tab[kl] - s0, d = dk[r];
        uint32_t y = d;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(y, o, 64);
            if (lane >= o) y += t;
        }
        const uint32_t rk0 = s_cnt[r * OC_WAVES + w] + y - d;   // the key's first rank in the chunk
        if (m > kOtMid) {
            for (uint32_t q = 0; q < nl; ++q)
                if (s_long[q] == kl) s_lrk[q] = rk0;
        } else if (m > kOtRun) {                      // its sorted slots in LDS: one walk
            uint32_t rk = rk0;
            for (uint32_t i = 0; i < m;) {
                const uint64_t x0 = stg[s0 + i];
                uint32_t tomb = (uint32_t)(x0 & 1u), k = i + 1;
                for (; k < m && (stg[s0 + k] >> tb) == (x0 >> tb); ++k) tomb |= (uint32_t)(stg[s0 + k] & 1u);
                ost[rk++] = (x0 & keep) | tomb;
                i = k;
            }
        } else if (m > 0) {
            // the OR of each tag's tombs, from the right: run = slot j's tomb,
            // plus the run after it while the tag continues
            uint32_t tt = 0, run = 0;
#pragma unroll
            for (int j = kOtRun - 1; j >= 0; --j) {
                const bool in = (uint32_t)j < m;
                const bool cont = (uint32_t)j + 1 < m && !((fk[r] >> (j + 1)) & 1u);
                run = (in ? (uint32_t)(slot(r, (uint32_t)j) & 1u) : 0u) | (cont ? run : 0u);
                tt |= run << j;
            }
            uint32_t rk = rk0;
#pragma unroll
            for (uint32_t j = 0; j < kOtRun; ++j)
                if ((fk[r] >> j) & 1u) ost[rk++] = (slot(r, j) & keep) | ((tt >> j) & 1u);
        }
    }
    __syncthreads();
    for (uint32_t q = 0; q < nl; ++q) {               // long keys' stores: ranks by counting the marks
        const uint32_t kl = s_long[q], rk0 = s_lrk[q];
        const uint32_t s0 = kl ? tab[kl - 1] : 0u, m = tab[kl] - s0;
        for (uint32_t i = tid; i < m; i += OCB) {
            if (!((s_first[(s0 + i) >> 5] >> ((s0 + i) & 31)) & 1u)) continue;
            const uint64_t xi = stg[s0 + i];
            uint32_t rk = 0, tomb = 0;
            for (uint32_t k = 0; k < m; ++k) {
                const uint64_t y = stg[s0 + k];
                if ((y >> tb) == (xi >> tb)) tomb |= (uint32_t)(y & 1u);
                else if (((s_first[(s0 + k) >> 5] >> ((s0 + k) & 31)) & 1u) && (y >> tb) < (xi >> tb)) ++rk;
            }
            ost[rk0 + rk] = (xi & keep) | tomb;
        }
    }
    }                                                 // (the next chunk of this workgroup)
    __syncthreads();
    if (stop) return;
    if (fb) return;                                   // (uniform; the call falls back to the radix path)
    if constexpr (!LB) {
        for (int kk = 0; kk < K; ++kk)
            for (uint32_t i = tid; i < s_totk[kk]; i += OCB) tmp[bounds[blockIdx.x * K + kk] + i] = ostb[kk][i];
        return;
    }
    if (K == 2 && w == 0 && diag == 6 && lane == 0) s_off = bounds[blockIdx.x * K];
    if (K == 2 && w == 0 && diag != 6) {              // one look-back for both chunks, after both are placed
        const uint32_t ci = blockIdx.x * K, n0 = s_totk[0], n1 = K == 2 ? s_totk[K - 1] : 0u;
        unsigned long long acc = 0;
        if (ci > 0) {
            acc = lookback_sum<1>(st, (long long)ci - 1, lane, err);
            if (lane == 0)
                __hip_atomic_store(&st[ci], kOcP | (acc + n0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            __hip_atomic_store(&st[ci + 1], kOcP | (acc + n0 + n1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_off = acc;
            if (ci + 1 == nch - 1) *out_count = acc + n0 + n1;
        }
    }
    __syncthreads();
    if (diag == 5) return;                            // (timing only: everything but the output stores)
    const uint32_t sr = p.b0 + p.br;
    size_t o = s_off;
    for (int kk = 0; kk < K; ++kk) {
        const uint32_t nt = s_totk[kk];
        const uint64_t *ost = ostb[kk];
        for (uint32_t i = tid; i < nt; i += OCB) {
            const uint64_t xv = ost[i];
            __builtin_nontemporal_store(p.kmin + lt_field(xv, kb, p.bk), &out.key[o + i]);   // (nontemporal: 2 % faster)
            __builtin_nontemporal_store(p.tmin + lt_field(xv, sr, p.bt), &out.ts[o + i]);
            __builtin_nontemporal_store((uint32_t)(p.rmin + lt_field(xv, p.b0, p.br)), &out.rep[o + i]);
            __builtin_nontemporal_store((uint8_t)(xv & 1u), &out.tomb[o + i]);
        }
        o += nt;
    }
}

// chunk i's tags (tmp[bounds[i], + cnt[i])) decoded to out[loc[i], ...)
__global__ __launch_bounds__(256) void k_or_emit(const uint64_t *__restrict__ tmp, const SortPlan *__restrict__ plan_,
                                                 const uint64_t *__restrict__ bounds, const uint32_t *__restrict__ cnt,
                                                 const uint32_t *__restrict__ loc, const uint32_t *__restrict__ tot,
                                                 crdt_tuples out, uint64_t *__restrict__ out_count, PlanGuard pg = {}) {
    const SortPlan p = *plan_;
    if (!plan_guard_ok(p, pg)) return;                 // (uniform: before any barrier)
    const uint32_t i = blockIdx.x, m = cnt[i];
    if (i == 0 && threadIdx.x == 0) *out_count = tot[0];
    const uint64_t *src = tmp + bounds[i];
    const size_t o = loc[i];
    const uint32_t kb = p.b0 + p.br + p.bt, st = p.b0 + p.br;
    for (uint32_t j = threadIdx.x; j < m; j += 256) {
        const uint64_t x = src[j];
        out.key[o + j] = p.kmin + lt_field(x, kb, p.bk);
        out.ts[o + j] = p.tmin + lt_field(x, st, p.bt);
        out.rep[o + j] = (uint32_t)(p.rmin + lt_field(x, p.b0, p.br));
        out.tomb[o + j] = (uint8_t)(x & 1u);
    }
}

// ---------------------------------------------------------------- OR-Set: groups put in tag order
// The fused OR-Set merge sorts on the KEY's bits and one more tag digit
// (sort.or_key_only = 2; config D: 32 of 51 bits, 4 passes instead of 7):
// tuples with equal sorted bits -- a GROUP -- come out contiguous, in input
// order, and every tag's copies lie in one group.  The dedup needs each group
// in full (key, ts, rep, side, tomb) order; groups are nearly all one tuple
// (config D: 20M tuples over ~2^32 group values), so the dedup's two passes
// work on GROUP-ALIGNED tiles and order the rare longer groups in LDS
// themselves (no extra pass over HBM):
//   k_run_bounds : tile t = [first group start >= t RT, first group start
//                  >= (t+1) RT), one thread per boundary (galloping search);
//   k_or_rdd_count: per tile (staged in LDS by LDS-DMA), 1 per one-tuple
//                  group, and at a longer group's first element its distinct
//                  tags (groups of more than kInsMax tuples rank-sorted in
//                  place first);
//   k_sort_colscan of the counts;
//   k_or_rdd_apply: the same counts, their prefix, then one-tuple groups
//                  store themselves and a longer group's first element
//                  stores its distinct tags at their ranks with the OR of
//                  each tag's tombs (a tag never leaves its tile).
// (sort.or_key_only = 1 keeps key runs of ~2.5 tuples as the groups; round 2
// sorted each by one thread's insertion sort: count 199 / apply 270 us at
// config D, instruction- and latency-bound -- the 4th pass costs less.)
// A run longer than the LDS tile (adversarial data: many copies of one key)
// makes its tile take the global path: the count pass sorts it in place
// (RCAP-chunks bitonic-sorted in LDS, then merged pairwise through a scratch
// buffer) and both passes read it from HBM.
constexpr int RT = 2048;                 // nominal tile (composites)
constexpr int RCAP = 3072;               // LDS capacity of a run-aligned tile
constexpr int RB = 512;                  // threads (6 composites each; 256 x 12: 0.985 ms, 1024 x 3: 1.10)
constexpr uint32_t kInsMax = 32;         // runs up to this length: element-wise marks, unsorted

// first run start at or after p (keys = composite >> ks): galloping, then binary search
__device__ __forceinline__ size_t run_start_from(const uint64_t *__restrict__ c, size_t n, size_t p, uint32_t ks) {
    if (p == 0 || p >= n) return p < n ? p : n;
    const uint64_t k = c[p - 1] >> ks;
    if ((c[p] >> ks) != k) return p;
    size_t lo = p, step = 1, hi = p;         // c[lo] has key k
    for (;;) {
        hi = lo + step;
        if (hi >= n || (c[hi] >> ks) != k) break;
        lo = hi;
        step <<= 1;
    }
    if (hi > n) hi = n;
    while (hi - lo > 1) {                    // c[lo] == k, c[hi] != k (or hi == n)
        const size_t mid = lo + (hi - lo) / 2;
        if ((c[mid] >> ks) == k) lo = mid;
        else hi = mid;
    }
    return hi;
}

__global__ void k_run_bounds(const uint64_t *__restrict__ c, size_t n, const SortPlan *__restrict__ plan_,
                             size_t ntiles, uint64_t *__restrict__ bounds, PlanGuard pg = {}) {
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (t > ntiles || !plan_guard_ok(*plan_, pg)) return;
    const size_t a = t * (size_t)RT;
    bounds[t] = run_start_from(c, n, a < n ? a : n, plan_->s0);
}

// in-place rank sort of s[r0, r0 + L) (L <= RCAP) by the workgroup
__device__ void lds_rank_sort(uint64_t *s, uint32_t r0, uint32_t L) {
    constexpr int PER = RCAP / RB;
    uint64_t v[PER];
    uint32_t rk[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = threadIdx.x + q * RB;
        v[q] = i < L ? s[r0 + i] : 0;
        rk[q] = 0;
    }
    for (uint32_t j = 0; j < L; ++j) {
        const uint64_t x = s[r0 + j];
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint32_t i = threadIdx.x + q * RB;
            rk[q] += (x < v[q] || (x == v[q] && j < i)) ? 1u : 0u;
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = threadIdx.x + q * RB;
        if (i < L) s[r0 + rk[q]] = v[q];
    }
    __syncthreads();
}

// bitonic sort of s[0, m) in LDS, m a power of two <= 4096
__device__ void lds_bitonic(uint64_t *s, uint32_t m) {
    for (uint32_t k = 2; k <= m; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < m; i += RB) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const uint64_t a = s[i], b = s[l];
                    if ((a > b) == ((i & k) == 0)) {
                        s[i] = b;
                        s[l] = a;
                    }
                }
            }
            __syncthreads();
        }
}

// sort x[0, L) by the workgroup: 2048-chunks in LDS, then merges through tmp
__device__ void long_run_sort(uint64_t *__restrict__ x, size_t L, uint64_t *__restrict__ tmp, uint64_t *s) {
    constexpr size_t CH = 2048;               // power-of-two chunk (<= RCAP)
    for (size_t c0 = 0; c0 < L; c0 += CH) {
        const uint32_t m = (uint32_t)(L - c0 < CH ? L - c0 : CH);
        uint32_t m2 = 1;
        while (m2 < m) m2 <<= 1;
        for (uint32_t i = threadIdx.x; i < m2; i += RB) s[i] = i < m ? x[c0 + i] : ~0ULL;
        __syncthreads();
        lds_bitonic(s, m2);
        for (uint32_t i = threadIdx.x; i < m; i += RB) x[c0 + i] = s[i];
        __syncthreads();
    }
    uint64_t *src = x, *dst = tmp;
    for (size_t w = CH; w < L; w <<= 1) {
        for (size_t lo = 0; lo < L; lo += 2 * w) {
            const size_t mid = lo + w < L ? lo + w : L, hi = lo + 2 * w < L ? lo + 2 * w : L;
            const size_t na = mid - lo, nb = hi - mid, tot = na + nb;
            const size_t per = (tot + RB - 1) / RB;
            const size_t d0 = (size_t)threadIdx.x * per < tot ? (size_t)threadIdx.x * per : tot;
            const size_t d1 = d0 + per < tot ? d0 + per : tot;
            if (d0 < d1) {
                size_t a_lo = d0 > nb ? d0 - nb : 0, a_hi = d0 < na ? d0 : na;   // merge path at d0
                while (a_lo < a_hi) {
                    const size_t am = (a_lo + a_hi) >> 1;
                    if (src[lo + am] <= src[mid + (d0 - 1 - am)]) a_lo = am + 1;
                    else a_hi = am;
                }
                size_t ia = a_lo, ib = d0 - a_lo;
                for (size_t d = d0; d < d1; ++d) {
                    const bool ta = ia < na && (ib >= nb || src[lo + ia] <= src[mid + ib]);
                    dst[lo + d] = ta ? src[lo + ia++] : src[mid + ib++];
                }
            }
        }
        __syncthreads();
        uint64_t *t = src;
        src = dst;
        dst = t;
    }
    if (src != x) {
        for (size_t i = threadIdx.x; i < L; i += RB) x[i] = src[i];
        __syncthreads();
    }
}

// the global path of a tile over RCAP: each of its runs sorted in place in c
__device__ void sort_runs_global(uint64_t *__restrict__ c, size_t n, size_t start, size_t end, uint32_t ks,
                                 uint64_t *__restrict__ scratch, uint64_t *s) {
    for (size_t cur = start; cur < end;) {
        const size_t re = run_start_from(c, n, cur + 1, ks);
        const size_t L = re - cur;
        if (L > (size_t)RCAP) {
            long_run_sort(c + cur, L, scratch + cur, s);
        } else if (L > 1) {
            for (uint32_t i = threadIdx.x; i < L; i += RB) s[i] = c[cur + i];
            __syncthreads();
            lds_rank_sort(s, 0, (uint32_t)L);
            for (uint32_t i = threadIdx.x; i < L; i += RB) c[cur + i] = s[i];
            __syncthreads();
        }
        cur = re;
    }
}

__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t *s_w) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = v;
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < RB / 64; ++w) t += s_w[w];
    return t;
}

// The run-aligned tile c[start, start + len) (len <= RCAP) into LDS by
// LDS-DMA from its 16-byte aligned-down start; returns the index of c[start]
// in dst.  (A strided load / store loop waited one HBM round trip per
// iteration: the count and apply passes took 221 / 261 us at config D.)
__device__ __forceinline__ int rdd_stage(const uint64_t *__restrict__ c, size_t start, uint32_t len, uint64_t *dst) {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), ln = threadIdx.x & 63;
    uint32_t at = 0;
    const int o = dma_run<uint64_t, RB / 64>(c, start, len, dst, &at, wv, ln);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    return o;
}

// A group = a run of equal sorted bits (composite >> ks) in a run-aligned
// tile s[0, L) in LDS; with the key and one more tag digit sorted (config D)
// nearly every group is ONE tuple, which emits itself.  Only the first
// element of a longer group does work: a short group (<= kInsMax, in input
// order) by pairwise compares -- element j is its tag's first copy when no
// other element has its tag and a smaller composite (an equal one: a lower
// index) -- a long one (sorted by lds_sort_long) by one linear walk.  (Marks
// of every element by itself, with walks or shuffles over its run, were
// instruction-bound: 87-215 us count, 186-417 us apply at config D.)

// the group starting at g0: its end, and its distinct tags
__device__ __forceinline__ uint32_t group_end(const uint64_t *s, uint32_t L, uint32_t g0, uint32_t ks) {
    const uint64_t k = s[g0] >> ks;
    uint32_t e = g0 + 1;
    while (e < L && (s[e] >> ks) == k) ++e;
    return e;
}
__device__ __forceinline__ bool group_first(const uint64_t *s, uint32_t g0, uint32_t e, uint32_t j, uint32_t tb) {
    const uint64_t x = s[j];
    for (uint32_t k = g0; k < e; ++k) {
        const uint64_t y = s[k];
        if (k != j && (y >> tb) == (x >> tb) && (y < x || (y == x && k < j))) return false;
    }
    return true;
}
__device__ uint32_t group_distinct(const uint64_t *s, uint32_t g0, uint32_t e, uint32_t tb) {
    uint32_t d = 0;
    if (e - g0 > kInsMax) {                              // sorted: count tag changes
        for (uint32_t j = g0; j < e; ++j) d += (j == g0 || (s[j] >> tb) != (s[j - 1] >> tb)) ? 1u : 0u;
        return d;
    }
    for (uint32_t j = g0; j < e; ++j) d += group_first(s, g0, e, j, tb) ? 1u : 0u;
    return d;
}

// The tile's group marks, every element's in registers: thread tid holds
// elements r RB + tid (r < RR), so wave w's lanes hold 64 consecutive ones
// per round.  All LDS reads of the elements and of each wave-round's two
// outer neighbours are issued before the first use; a group's start / end
// come from the neighbours (shuffles).  Groups longer than kInsMax are found
// at their starts and rank-sorted in LDS (rare; the elements are then read
// again).  (Per-element walks, shuffle windows and a separate detection pass,
// each a chain of dependent LDS reads: count 87-215 us, apply 186-417 us.)
constexpr int RR = (RCAP + RB - 1) / RB;                 // wave-rounds per thread
struct RddMarks {
    uint64_t x[RR];
    uint32_t kind;                                       // 2 bits per round: 1 one-tuple group, 2 a pair's first
};                                                       // (its mate in the next lane), 3 a longer group's first
__device__ __forceinline__ void rdd_marks(uint64_t *s, uint32_t L, uint32_t ks, uint32_t *s_big, uint32_t *s_nbig,
                                          RddMarks &m) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) *s_nbig = 0;
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (int r = 0; r < RR; ++r) {
            const uint32_t i = (uint32_t)r * RB + threadIdx.x;
            m.x[r] = i < L ? s[i] : 0;
        }
        m.kind = 0;
        bool any_long = false;
#pragma unroll
        for (int r = 0; r < RR; ++r) {
            const uint32_t i0 = (uint32_t)r * RB + 64u * (uint32_t)w, i = i0 + (uint32_t)lane;
            const uint64_t x = m.x[r], k = x >> ks;
            uint64_t xp = __shfl_up((unsigned long long)x, 1, 64), xn = __shfl_down((unsigned long long)x, 1, 64);
            if (lane == 0 && i0 > 0 && i0 < L) xp = s[i0 - 1];     // the wave-round's outer neighbours
            if (lane == 63 && i + 1 < L) xn = s[i + 1];
            const bool valid = i < L;
            const bool st = valid && (i == 0 || (xp >> ks) != k);
            const bool en = valid && (i + 1 >= L || (xn >> ks) != k);
            // a pair: the group is this lane's element and the next lane's (the
            // common longer group: an A tuple and its B copy)
            const bool en1 = ((__ballot(en) >> 1) >> lane) & 1u;   // the next lane ends a group
            const uint32_t kd = !st ? 0u : en ? 1u : (lane < 63 && en1) ? 2u : 3u;
            m.kind |= kd << (2 * r);
            if (pass == 0 && st && !en && i + kInsMax < L && (s[i + kInsMax] >> ks) == k) {   // > kInsMax
                s_big[atomicAdd(s_nbig, 1u)] = i;
                any_long = true;
            }
        }
        (void)any_long;
        __syncthreads();
        const uint32_t nbig = *s_nbig;
        if (pass == 1 || nbig == 0) return;              // (uniform)
        for (uint32_t q = 0; q < nbig; ++q) {
            const uint32_t r0 = s_big[q];
            lds_rank_sort(s, r0, group_end(s, L, r0, ks) - r0);   // (barriers inside)
        }
    }
}

__global__ __launch_bounds__(RB) void k_or_rdd_count(uint64_t *__restrict__ c, size_t n,
                                                      const SortPlan *__restrict__ plan_,
                                                      const uint64_t *__restrict__ bounds,
                                                      uint64_t *__restrict__ scratch, uint32_t *__restrict__ cnt,
                                                      int diag_, PlanGuard pg = {}) {
    const int diag = kDiagBuild ? diag_ : 0;          // (the product build has no timing diagnostics)
    __shared__ alignas(16) uint64_t s_raw[RCAP + 2];
    __shared__ uint32_t s_big[RCAP / (kInsMax + 1) + 1], s_nbig, s_w[RB / 64];
    const SortPlan p = *plan_;
    if (!plan_guard_ok(p, pg)) return;                 // (uniform: before any barrier)
    const uint32_t ks = p.s0, tb = p.b0;                 // group bits from ks; tag bits from b0
    const size_t t = blockIdx.x, start = bounds[t], end = bounds[t + 1];
    const size_t len = end > start ? end - start : 0;
    uint32_t m = 0;
    if (len <= (size_t)RCAP) {
        uint64_t *s = s_raw + rdd_stage(c, start, (uint32_t)len, s_raw);
        if (diag == 1) {                                 // timing diagnostic: staging only, no outputs
            if (threadIdx.x == 0) cnt[t] = 0;
            return;
        }
        RddMarks mk;
        rdd_marks(s, (uint32_t)len, ks, s_big, &s_nbig, mk);
        if (diag == 2) {                                 // timing diagnostic: + the marks
            if (threadIdx.x == 0) cnt[t] = (uint32_t)mk.kind & 0;
            return;
        }
#pragma unroll
        for (int r = 0; r < RR; ++r) {
            const uint32_t kind = (mk.kind >> (2 * r)) & 3u;
            const uint64_t x1 = __shfl_down((unsigned long long)mk.x[r], 1, 64);   // (uniform)
            if (kind == 1) {
                ++m;
            } else if (kind == 2) {
                m += (mk.x[r] >> tb) == (x1 >> tb) ? 1u : 2u;
            } else if (kind == 3) {
                const uint32_t i = (uint32_t)r * RB + threadIdx.x;
                m += group_distinct(s, i, group_end(s, (uint32_t)len, i, ks), tb);
            }
        }
    } else {
        sort_runs_global(c, n, start, end, ks, scratch, s_raw);
        __threadfence();
        __syncthreads();
        for (size_t i = start + threadIdx.x; i < end; i += RB)
            m += (i == start || (c[i] >> tb) != (c[i - 1] >> tb)) ? 1u : 0u;
    }
    const uint32_t tot = block_sum(m, s_w);
    if (threadIdx.x == 0) cnt[t] = tot;
}

__global__ __launch_bounds__(RB) void k_or_rdd_apply(const uint64_t *__restrict__ c, size_t n,
                                                      const SortPlan *__restrict__ plan_,
                                                      const uint64_t *__restrict__ bounds,
                                                      const uint32_t *__restrict__ loc, const uint32_t *__restrict__ tot,
                                                      crdt_tuples out, uint64_t *__restrict__ out_count, int diag_, PlanGuard pg = {}) {
    const int diag = kDiagBuild ? diag_ : 0;          // (the product build has no timing diagnostics)
    __shared__ alignas(16) uint64_t s_raw[RCAP + 2];
    __shared__ uint32_t s_c[RR * (RB / 64)];             // outputs per (round, wave), then their exclusive prefix
    __shared__ uint32_t s_big[RCAP / (kInsMax + 1) + 1], s_nbig, s_w[RB / 64];
    const SortPlan p = *plan_;
    if (!plan_guard_ok(p, pg)) return;                 // (uniform: before any barrier)
    const uint32_t ks = p.s0, tb = p.b0, sk = p.b0 + p.br + p.bt;
    const size_t t = blockIdx.x, start = bounds[t], end = bounds[t + 1];
    if (t == 0 && threadIdx.x == 0) *out_count = tot[0];
    const size_t len = end > start ? end - start : 0;
    if (len == 0) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    size_t base = loc[t];
    auto store = [&](size_t o, uint64_t x, uint32_t tomb) {
        CKey<1> v;
        v.w[0] = x;
        out.key[o] = p.kmin + get_bits(v, sk, p.bk);
        out.ts[o] = p.tmin + get_bits(v, p.b0 + p.br, p.bt);
        out.rep[o] = (uint32_t)(p.rmin + get_bits(v, p.b0, p.br));
        out.tomb[o] = (uint8_t)tomb;
    };
    if (len > (size_t)RCAP) {                            // the global path: runs sorted in c by the count pass
        for (size_t r0 = 0; r0 < len; r0 += RB) {
            const size_t i = r0 + threadIdx.x;
            const uint64_t x = i < len ? c[start + i] : 0;
            const bool f = i < len && (i == 0 || (x >> tb) != (c[start + i - 1] >> tb));
            const uint64_t em = __ballot(f);
            __syncthreads();                             // s_w of the previous round read
            if (lane == 0) s_w[w] = (uint32_t)__popcll(em);
            __syncthreads();
            uint32_t before = 0, all = 0;
#pragma unroll
            for (int k = 0; k < RB / 64; ++k) {
                before += k < w ? s_w[k] : 0u;
                all += s_w[k];
            }
            if (f) {
                uint32_t tomb = (uint32_t)(x & 1u);
                for (size_t j = i + 1; j < len; ++j) {   // the tag's other copies (never past the tile)
                    const uint64_t y = c[start + j];
                    if ((y >> tb) != (x >> tb)) break;
                    tomb |= (uint32_t)(y & 1u);
                }
                store(base + before + (uint32_t)__popcll(em & ((1ULL << lane) - 1ULL)), x, tomb);
            }
            base += all;
        }
        return;
    }
    const uint32_t L = (uint32_t)len;
    uint64_t *s = s_raw + rdd_stage(c, start, L, s_raw);
    if (diag == 1) return;                               // timing diagnostics (no stores)
    RddMarks mk;
    rdd_marks(s, L, ks, s_big, &s_nbig, mk);
    if (diag == 2) return;
    // pass 1: every element's output count and its exclusive prefix within
    // the wave-round (mbcnt when every count is 0 / 1, else a shuffle scan)
    uint32_t pre[RR];
#pragma unroll
    for (int r = 0; r < RR; ++r) {
        const uint32_t kind = (mk.kind >> (2 * r)) & 3u, i = (uint32_t)r * RB + threadIdx.x;
        const uint64_t x1 = __shfl_down((unsigned long long)mk.x[r], 1, 64);   // (uniform)
        uint32_t cn = kind == 1 ? 1u : kind == 2 ? ((mk.x[r] >> tb) == (x1 >> tb) ? 1u : 2u) : 0u;
        if (kind == 3) cn = group_distinct(s, i, group_end(s, L, i, ks), tb);
        uint32_t ex, all;
        if (__ballot(cn > 1) == 0) {
            const uint64_t one = __ballot(cn == 1);
            ex = __builtin_amdgcn_mbcnt_hi((uint32_t)(one >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)one, 0u));
            all = (uint32_t)__popcll(one);
        } else {
            uint32_t x = cn;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o, 64);
                if (lane >= o) x += y;
            }
            ex = x - cn;
            all = (uint32_t)__shfl((int)x, 63, 64);
        }
        pre[r] = ex;
        if (lane == 0) s_c[r * (RB / 64) + w] = all;
    }
    __syncthreads();
    if (diag == 3) return;
    if (w == 0) {                                        // exclusive prefix over (round, wave), tile order
        constexpr int NC = RR * (RB / 64);
        static_assert(NC <= 64, "one wave");
        const uint32_t c0 = lane < NC ? s_c[lane] : 0u;
        uint32_t x = c0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane < NC) s_c[lane] = x - c0;
    }
    __syncthreads();
    // pass 2: one-tuple groups store themselves; a longer group's first
    // element stores the group's distinct tags in tag order
#pragma unroll
    for (int r = 0; r < RR; ++r) {
        const uint32_t kind = (mk.kind >> (2 * r)) & 3u;
        const uint64_t x1 = __shfl_down((unsigned long long)mk.x[r], 1, 64);   // (uniform)
        if (!kind) continue;
        const uint32_t i = (uint32_t)r * RB + threadIdx.x;
        const size_t o = base + s_c[r * (RB / 64) + w] + pre[r];
        const uint64_t x = mk.x[r];
        if (kind == 1) {
            store(o, x, (uint32_t)(x & 1u));
            continue;
        }
        if (kind == 2) {                                 // a pair, from registers
            if ((x >> tb) == (x1 >> tb)) {
                store(o, x < x1 ? x : x1, (uint32_t)((x | x1) & 1u));
            } else {
                const uint64_t lo = x < x1 ? x : x1, hi = x < x1 ? x1 : x;
                store(o, lo, (uint32_t)(lo & 1u));
                store(o + 1, hi, (uint32_t)(hi & 1u));
            }
            continue;
        }
        const uint32_t e = group_end(s, L, i, ks);
        if (e - i > kInsMax) {                           // sorted long group: one walk
            uint32_t q = 0;
            for (uint32_t j = i; j < e;) {
                const uint64_t y = s[j];
                uint32_t tomb = (uint32_t)(y & 1u), k = j + 1;
                for (; k < e && (s[k] >> tb) == (y >> tb); ++k) tomb |= (uint32_t)(s[k] & 1u);
                store(o + q++, y, tomb);
                j = k;
            }
            continue;
        }
        for (uint32_t j = i; j < e; ++j) {               // short group, input order: rank the first copies
            if (!group_first(s, i, e, j, tb)) continue;
            const uint64_t y = s[j];
            uint32_t rk = 0, tomb = 0;
            for (uint32_t k = i; k < e; ++k) {
                const uint64_t z = s[k];
                if ((z >> tb) == (y >> tb)) tomb |= (uint32_t)(z & 1u);
                else if ((z >> tb) < (y >> tb) && group_first(s, i, e, k, tb)) ++rk;
            }
            store(o + rk, y, tomb);
        }
    }
}

static int or_run_dedup(crdt_ctx *ctx, uint64_t *c, size_t n, const SortPlan *plan, uint64_t *scratch,
                        uint64_t *bounds, uint32_t *cnt, uint32_t *loc, uint32_t *tot, const crdt_tuples &out,
                        uint64_t *out_count) {
    const hipStream_t st = ctx->stream;
    const size_t nt = (n + RT - 1) / RT;
    k_run_bounds<<<(unsigned)((nt + 1 + 255) / 256), 256, 0, st>>>(c, n, plan, nt, bounds, cur_guard());
    k_or_rdd_count<<<(unsigned)nt, RB, 0, st>>>(c, n, plan, bounds, scratch, cnt, g_rdd_diag, cur_guard());
    k_sort_colscan<<<1, CSB, 0, st>>>(cnt, (uint32_t)nt, loc, tot);
    k_or_rdd_apply<<<(unsigned)nt, RB, 0, st>>>(c, n, plan, bounds, loc, tot, out, out_count, g_rdd_diag,
                                                 cur_guard());
    return check_launch(ctx);
}

// the device plan back to the host through the context's pinned buffer (a
// pageable destination costs a staged copy on every call)
static int read_plan(crdt_ctx *ctx, const SortPlan *plan, SortPlan *h) {
    static_assert(sizeof(SortPlan) % 4 == 0, "whole words");
    const void *hp = nullptr;
    int rc = ctx_read_words(ctx, plan, sizeof(SortPlan), &hp);
    if (rc) return rc;
    memcpy(h, hp, sizeof(SortPlan));
    return CRDT_OK;
}

template <int MODE, int WORDS>
static int dedup_words(crdt_ctx *ctx, const uint64_t *c, size_t n, const SortPlan *plan, uint32_t *cnt,
                       uint32_t *loc, uint32_t *tot, const crdt_tuples &out, uint64_t *out_count) {
    const hipStream_t st = ctx->stream;
    const unsigned nt = (unsigned)((n + DT - 1) / DT);
    k_dd_count<MODE, WORDS><<<nt, DB, 0, st>>>(c, n, plan, cnt, cur_guard());
    k_sort_colscan<<<1, CSB, 0, st>>>(cnt, nt, loc, tot);
    k_dd_apply<MODE, WORDS><<<nt, DB, 0, st>>>(c, n, plan, loc, tot, out, out_count, g_rdd_diag, cur_guard());
    return check_launch(ctx);
}

static bool tuples_full(const crdt_tuples *t) { return t && t->key && t->ts && t->rep && t->tomb; }

// any byte of out's four fields (cap tuples) inside any of in's (n tuples)?
// The dense-key D2 forms store into out before they know whether the call
// must be redone from the inputs, so out may not alias a or b.
static bool tuples_overlap(const crdt_tuples &out, size_t cap, const crdt_tuples &in, size_t n) {
    if (n == 0 || cap == 0) return false;
    const uintptr_t ob[4] = {(uintptr_t)out.key, (uintptr_t)out.ts, (uintptr_t)out.rep, (uintptr_t)out.tomb};
    const size_t ow[4] = {8, 8, 4, 1};
    const uintptr_t ib[4] = {(uintptr_t)in.key, (uintptr_t)in.ts, (uintptr_t)in.rep, (uintptr_t)in.tomb};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            if (ob[i] < ib[j] + n * ow[j] && ib[j] < ob[i] + cap * ow[i]) return true;
    return false;
}

// ---------------------------------------------------------------- the D2 merge's workspace
constexpr size_t kMaxChunks = 1u << 16;             // k_or_chunk: 2^(bk - 9), bk <= 25
struct D2Ws {
    SortMinMax *mm;
    SortPlan *plan;
    uint32_t *cnt, *loc, *tot;
    uint64_t *bufs;
    unsigned long long *flags;                      // [0, 256) bucket / look-back words, [256] the OR chunk fallback
    uint32_t *viol;                                 // the plan's range check (the upsweep raises it)
    uint64_t *cb;                                   // OR-Set chunk bounds, counts, offsets, look-back words
    uint32_t *cc, *cl, *ct;
    unsigned long long *cst;
    uint32_t *hrows, *hflag;                        // OR-Set: per-run chunk counts (SubHist), 64 B per (bucket, tile)
};

template <int MODE>
static size_t d2_ws_bytes(size_t n) {
    const size_t ntiles = (n + ST - 1) / ST, ncnt = ntiles * 256;
    const size_t b_mm = Carve::round(2 * MM_BLOCKS * sizeof(SortMinMax)), b_plan = Carve::round(sizeof(SortPlan));
    const size_t b_cnt = Carve::round(ncnt * 4), b_tot = Carve::round(256 * 4), b_bufs = Carve::round(2 * 3 * n * 8);
    const size_t b_flag = Carve::round(258 * 8);
    const size_t b_chunk = MODE == DD_OR ? 2 * Carve::round((kMaxChunks + 1) * 8) + 2 * Carve::round(kMaxChunks * 4) +
                                               Carve::round(64) + Carve::round(ntiles * 256 * 64) + Carve::round(256 * 4)
                                         : 0;
    return b_mm + b_plan + 2 * b_cnt + b_tot + b_bufs + b_flag + b_chunk + 1024;
}

template <int MODE>
static D2Ws d2_carve(void *ws, size_t n) {
    const size_t ntiles = (n + ST - 1) / ST, ncnt = ntiles * 256;   // >= the dedup's tile count
    Carve w(ws);
    D2Ws d{};
    d.mm = w.take<SortMinMax>(2 * MM_BLOCKS);
    d.plan = w.take<SortPlan>(1);
    d.cnt = w.take<uint32_t>(ncnt);
    d.loc = w.take<uint32_t>(ncnt);
    d.tot = w.take<uint32_t>(256);
    d.bufs = w.take<uint64_t>(2 * 3 * n);
    d.flags = w.take<unsigned long long>(258);
    d.viol = (uint32_t *)&d.flags[257];
    if (MODE == DD_OR) {
        d.cb = w.take<uint64_t>(kMaxChunks + 1);
        d.cc = w.take<uint32_t>(kMaxChunks);
        d.cl = w.take<uint32_t>(kMaxChunks);
        d.ct = w.take<uint32_t>(16);
        d.cst = w.take<unsigned long long>(kMaxChunks + 1);
        d.hrows = w.take<uint32_t>(ntiles * 256 * 16);   // (ntiles of 4096: enough for either grouping tile)
        d.hflag = w.take<uint32_t>(256);
    }
    return d;
}

// A planned call's plan on the device (by value: the launch captures it, so
// a graph replays it) and its range check cleared.
__global__ void k_put_plan(SortPlan h, SortPlan *plan, uint32_t *viol) {
    if (threadIdx.x == 0) {
        *plan = h;
        *viol = 0;
    }
}

// Failpoint "fail.d2_plan": the device plan's shape changed behind the
// host's back (more key bits: the bucket / chunk indices of the fault of
// commit 01a0e59).
__global__ void k_corrupt_plan(SortPlan *plan) {
    if (threadIdx.x == 0) plan->bk += 7;
}

// A planned call's end: a tuple outside the plan (the upsweep's range check)
// or an OR-Set chunk over its LDS limits leaves the output invalid -- raise
// CRDT_DEV_PLAN and set the count to ~0 (no host synchronisation).
__global__ void k_d2_check(const uint32_t *__restrict__ viol, const uint32_t *__restrict__ fb,
                           uint64_t *__restrict__ out_count, uint32_t *__restrict__ err) {
    if (threadIdx.x == 0 && ((viol && *viol) || (fb && *fb))) {
        atomicOr(err, CRDT_DEV_PLAN);
        *out_count = ~0ull;
    }
}

// The fresh (sampled) plan against the cached one the host launched from:
// any difference in the launch shape raises the range check (a miss) AND
// puts the cached shape into the device plan, so the passes launched on the
// cached grids index their tables, buckets and chunks by the shape those
// grids were sized for (the fresh plan's own shape -- e.g. a sample that
// caught a far key: 41 key bits -- would send the bucket pass past its 256
// sub-buckets and the chunk bounds).  The call's own fields (side pointer,
// n1, the range minima) stay; the output is discarded and the call redone.
__global__ void k_plan_match(SortPlan *__restrict__ fresh, SortPlan c, uint32_t *__restrict__ viol) {
    if (threadIdx.x != 0) return;
    SortPlan f = *fresh;
    if (f.words != c.words || f.P != c.P || f.s0 != c.s0 || f.tl != c.tl || f.tw != c.tw || f.bk != c.bk ||
        f.bt != c.bt || f.br != c.br || f.b0 != c.b0 || f.W != c.W) {
        f.words = c.words, f.P = c.P, f.s0 = c.s0, f.tl = c.tl, f.tw = c.tw;
        f.bk = c.bk, f.bt = c.bt, f.br = c.br, f.b0 = c.b0, f.W = c.W;
        *fresh = f;
        *viol = 1;
    }
}
static_assert(sizeof(SortPlan) <= sizeof(((crdt_ctx *)nullptr)->d2_plan[0]), "the context caches a plan per mode");

static bool d2_vec(const crdt_tuples &A, size_t na, const crdt_tuples &B, size_t nb) {
    auto vec_ok = [](const crdt_tuples &t, size_t m) {
        return m == 0 || !((((uintptr_t)t.key | (uintptr_t)t.ts) & 15) | ((uintptr_t)t.rep & 7) |
                           ((uintptr_t)t.tomb & 1));
    };
    return vec_ok(A, na) && vec_ok(B, nb) && na % 2 == 0 && g_sort_vec_up;
}

// The tile grouping pass of the gather forms (k_lww_up_tiled): tiles of
// sort.group_tile tuples (4096 or 8192) grouped by the key's top byte;
// returns the tile count.
static unsigned group_tiles(hipStream_t s, const crdt_tuples &A, size_t n, const D2Ws &w, uint32_t *vw,
                            const SubHist &hist = {}) {
    const unsigned tile = g_group_tile == 8192 ? 8192u : 4096u;
    const unsigned ntiles = (unsigned)((n + tile - 1) / tile);
    if (hist.rows && tile == 8192)
        k_lww_up_tiled<1024, 8192, true><<<ntiles, 1024, 0, s>>>(A, n, w.plan, ntiles, w.cnt, w.bufs, vw, w.flags, hist,
                                                                     cur_guard());
    else if (hist.rows)
        k_lww_up_tiled<512, ST, true><<<ntiles, 512, 0, s>>>(A, n, w.plan, ntiles, w.cnt, w.bufs, vw, w.flags, hist,
                                                                     cur_guard());
    else if (tile == 8192)
        k_lww_up_tiled<1024, 8192><<<ntiles, 1024, 0, s>>>(A, n, w.plan, ntiles, w.cnt, w.bufs, vw, w.flags, SubHist{},
                                                                     cur_guard());
    else if (g_up_threads == 512)
        k_lww_up_tiled<512, ST><<<ntiles, 512, 0, s>>>(A, n, w.plan, ntiles, w.cnt, w.bufs, vw, w.flags, SubHist{},
                                                                     cur_guard());
    else
        k_lww_up_tiled<SB, ST><<<ntiles, SB, 0, s>>>(A, n, w.plan, ntiles, w.cnt, w.bufs, vw, w.flags, SubHist{},
                                                                     cur_guard());
    return ntiles;
}

// The passes of a D2 merge whose plan h is known on the host (w.plan holds
// it on the device).  vw: the range check of a sampled or given plan
// (nullptr: the plan is exact for these inputs).
//   planned (crdt_*_merge_unsorted_planned): no host synchronisation at all
//     -- a tuple outside the plan, or an OR-Set chunk over its LDS limits,
//     raises CRDT_DEV_PLAN and sets *out_count = ~0 (k_d2_check);
//   otherwise the dense-key forms read their check words back at the end:
//     *miss = the call must be redone from the exact plan (the caller does);
//     the OR-Set chunk fallback runs the radix path here.
template <int MODE>
static int d2_body(crdt_ctx *ctx, const crdt_tuples &A, size_t na, const crdt_tuples &B, size_t nb,
                   const crdt_tuples &out, uint64_t *out_count, const D2Ws &w, SortPlan h, uint32_t *vw, bool vec,
                   bool planned, bool *miss) {
    const size_t n = na + nb;
    const hipStream_t s = ctx->stream;
    const uint32_t key_only = MODE == DD_LWW ? 1u : g_or_key_sort ? (uint32_t)g_or_key_sort : 0u;
    *miss = false;
    GuardScope guard(h, vw);                           // every pass below checks the device plan against h
    if (vw && take_fail_d2_plan()) {                   // failpoint (diagnostic build): a plan of another shape
        k_corrupt_plan<<<1, 64, 0, s>>>(w.plan);       //   in device memory -- the guards must catch it
        int rc0 = check_launch(ctx);
        if (rc0) return rc0;
    }
    const void *hw = nullptr;                          // the end-of-call check words, on the host
    auto read_words = [&](const void *src, size_t bytes) -> int { return ctx_read_words(ctx, src, bytes, &hw); };
    auto finish = [&](const uint32_t *fb) -> int {     // after the last pass: the range check
        int rc = check_launch(ctx);
        if (rc || !vw) return rc;
        if (planned) {
            k_d2_check<<<1, 64, 0, s>>>(vw, fb, out_count, ctx->dev_status);
            return check_launch(ctx);
        }
        rc = read_words(vw, 4);
        if (!rc) *miss = *(const uint32_t *)hw != 0;
        return rc;
    };
    uint64_t *sorted = nullptr;
    int rc;
    if (h.words == 1) {
        if (MODE == DD_LWW && h.tw && vec && g_lww_gather) {   // tiles grouped by bucket, tables gather their runs
            const unsigned ntiles = group_tiles(s, A, n, w, vw);
#define LWW_G(E, GLV) \
    k_lww_table_g<E, GLV><<<256, LTB, 0, s>>>(w.bufs, w.plan, w.cnt, ntiles, w.flags, out, out_count, ctx->dev_status, \
                                              cur_guard())
            if (h.tw == 4) {
                if (g_group_tile == 8192) LWW_G(uint32_t, 4);
                else LWW_G(uint32_t, 2);
            } else {
                if (g_group_tile == 8192) LWW_G(uint64_t, 4);
                else LWW_G(uint64_t, 2);
            }
#undef LWW_G
            return finish(nullptr);
        }
        if (MODE == DD_LWW && h.tw) {                   // one pass on the key's top byte, then bucket tables
            rc = sort_words<1>(ctx, A, n, out, w.plan, 1, w.bufs, w.cnt, w.loc, w.tot, false, &sorted, vec, w.flags,
                               vw);
            if (rc) return rc;
            if (h.tw == 4)
                k_lww_table<uint32_t><<<256, LTB, 0, s>>>(sorted, w.plan, w.tot, w.flags, out, out_count,
                                                          ctx->dev_status, cur_guard());
            else
                k_lww_table<uint64_t><<<256, LTB, 0, s>>>(sorted, w.plan, w.tot, w.flags, out, out_count,
                                                          ctx->dev_status, cur_guard());
            return finish(nullptr);
        }
        if (MODE == DD_OR && h.tw) {                    // the key's top 16 bits grouped, then chunks in LDS
            const uint32_t nch = 1u << (h.bk - kOcBits), kb = h.b0 + h.br + h.bt;
            const bool lb = g_or_lookback && (!g_rdd_diag || g_rdd_diag >= 5);   // (diag 5 / 6: the look-back form's timings)
            if (vec && g_or_bucket) {                   // tiles grouped by top byte, buckets gathered into chunks
                // per-run chunk counts from the grouping pass (<= 64 chunks per top byte)
                const SubHist hist = (g_or_sub_hist && h.bk <= 23) ? SubHist{w.hrows, w.hflag} : SubHist{};
                const unsigned gt = group_tiles(s, A, n, w, vw, hist);
                if (g_group_tile == 8192)
                    k_or_bucket<4><<<256, OBB, 0, s>>>(w.bufs, w.plan, w.cnt, gt, n, w.flags, w.bufs + n, w.cb,
                                                       lb ? w.cst : nullptr, nch, ctx->dev_status, g_rdd_diag,
                                                       g_or_place_batch != 0, hist, cur_guard());
                else
                    k_or_bucket<2><<<256, OBB, 0, s>>>(w.bufs, w.plan, w.cnt, gt, n, w.flags, w.bufs + n, w.cb,
                                                       lb ? w.cst : nullptr, nch, ctx->dev_status, g_rdd_diag,
                                                       g_or_place_batch != 0, hist, cur_guard());
                sorted = w.bufs + n;
            } else {                                    // two radix passes on the top 16 bits
                rc = sort_words<1>(ctx, A, n, out, w.plan, 2, w.bufs, w.cnt, w.loc, w.tot, false, &sorted, vec,
                                   w.flags, vw);
                if (rc) return rc;
            }
            uint64_t *tmp = sorted == w.bufs ? w.bufs + n : w.bufs;
            uint32_t *fbw = (uint32_t *)&w.flags[256];
            if (!(vec && g_or_bucket))
                k_chunk_bounds<<<(nch + 1 + 3) / 4, 256, 0, s>>>(sorted, n, kb + kOcBits, nch, w.cb,
                                                                  lb ? w.cst : nullptr);
            const bool narrow = kb <= 32 && g_or_narrow;
            const int kpair = g_or_pair && nch % 2 == 0 ? 2 : 1;
            const unsigned grid = nch / (unsigned)kpair;
#define OR_CHUNK(LBV, NAR, KV)                                                                                 \
    k_or_chunk<LBV, NAR, KV><<<grid, OCB, 0, s>>>(sorted, tmp, w.plan, w.cb, w.cc, fbw, g_rdd_diag, LBV ? w.cst : nullptr, \
                                                   out, out_count, ctx->dev_status, nch, cur_guard())
            if (lb) {
                if (narrow) {
                    if (kpair == 2) OR_CHUNK(true, true, 2);
                    else OR_CHUNK(true, true, 1);
                } else {
                    if (kpair == 2) OR_CHUNK(true, false, 2);
                    else OR_CHUNK(true, false, 1);
                }
            } else {
                if (narrow) {
                    if (kpair == 2) OR_CHUNK(false, true, 2);
                    else OR_CHUNK(false, true, 1);
                } else {
                    if (kpair == 2) OR_CHUNK(false, false, 2);
                    else OR_CHUNK(false, false, 1);
                }
#undef OR_CHUNK
                k_sort_colscan<<<1, CSB, 0, s>>>(w.cc, nch, w.cl, w.ct);
                k_or_emit<<<nch, 256, 0, s>>>(tmp, w.plan, w.cb, w.cc, w.cl, w.ct, out, out_count, cur_guard());
            }
            rc = check_launch(ctx);
            if (rc) return rc;
            if (planned) {
                k_d2_check<<<1, 64, 0, s>>>(vw, fbw, out_count, ctx->dev_status);
                return check_launch(ctx);
            }
            rc = read_words(&w.flags[256], 16);        // the fallback word (long keys), the range check
            if (rc) return rc;
            const uint32_t fb = *(const uint32_t *)hw, mw = vw ? ((const uint32_t *)hw)[2] : 0u;
            if (mw) {
                *miss = true;
                return CRDT_OK;
            }
            if (fb == 0) return CRDT_OK;
            // the sort path from the untouched inputs, on the exact ranges
            const unsigned nmm = launch_minmax(ctx, A, na, B, nb, w.mm);
            k_sort_plan<<<1, 256, 0, s>>>(w.mm, nmm, w.plan, 1, B, na, key_only, 0u, 0u, (uint64_t)n);
            rc = read_plan(ctx, w.plan, &h);
            if (rc) return rc;
            vw = nullptr;
            guard.set(h, nullptr);                      // (the exact plan, read back: nothing to check)
        }
        rc = sort_words<1>(ctx, A, n, out, w.plan, h.P, w.bufs, w.cnt, w.loc, w.tot, false, &sorted, vec, nullptr, vw);
        if (!rc && MODE == DD_OR && h.s0)                 // key-only sort: key runs ordered in the dedup
            rc = or_run_dedup(ctx, sorted, n, w.plan, sorted == w.bufs ? w.bufs + n : w.bufs, w.bufs + 2 * n, w.cnt,
                              w.loc, w.tot, out, out_count);
        else if (!rc)
            rc = dedup_words<MODE, 1>(ctx, sorted, n, w.plan, w.cnt, w.loc, w.tot, out, out_count);
        return rc ? rc : finish(nullptr);
    }
    if (h.words == 2) {
        rc = sort_words<2>(ctx, A, n, out, w.plan, h.P, w.bufs, w.cnt, w.loc, w.tot, false, &sorted, false, nullptr, vw);
        if (!rc) rc = dedup_words<MODE, 2>(ctx, sorted, n, w.plan, w.cnt, w.loc, w.tot, out, out_count);
        return rc ? rc : finish(nullptr);
    }
    rc = sort_words<3>(ctx, A, n, out, w.plan, h.P, w.bufs, w.cnt, w.loc, w.tot, false, &sorted, false, nullptr, vw);
    if (!rc) rc = dedup_words<MODE, 3>(ctx, sorted, n, w.plan, w.cnt, w.loc, w.tot, out, out_count);
    return rc ? rc : finish(nullptr);
}

// argument checks shared by the planned and unplanned calls
static int d2_args(const crdt_tuples *a, size_t na, const crdt_tuples *b, size_t nb, const crdt_tuples *out,
                   const uint64_t *out_count) {
    if (!out_count || !tuples_full(out)) return CRDT_E_INVAL;
    if ((na && !tuples_full(a)) || (nb && !tuples_full(b))) return CRDT_E_INVAL;
    if (na + nb >= (1ULL << 32)) return CRDT_E_RANGE;  // 32-bit in-tile / bucket arithmetic
    const crdt_tuples none{nullptr, nullptr, nullptr, nullptr};
    if (tuples_overlap(*out, na + nb, na ? *a : none, na) || tuples_overlap(*out, na + nb, nb ? *b : none, nb))
        return CRDT_E_INVAL;
    return CRDT_OK;
}

template <int MODE>
static int set_merge_unsorted(crdt_ctx *ctx, const crdt_tuples *a, size_t na, const crdt_tuples *b, size_t nb,
                              crdt_tuples *out, uint64_t *out_count, bool allow_sample = true) {
    int rc = bind(ctx);
    if (rc) return rc;
    rc = d2_args(a, na, b, nb, out, out_count);
    if (rc) return rc;
    const size_t n = na + nb;
    const hipStream_t s = ctx->stream;
    if (n == 0) {
        hipError_t e = hipMemsetAsync(out_count, 0, sizeof(uint64_t), s);
        return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
    }
    const crdt_tuples none{nullptr, nullptr, nullptr, nullptr};
    const crdt_tuples A = na ? *a : none, B = nb ? *b : none;
    rc = ws_reserve(ctx, d2_ws_bytes<MODE>(n));
    if (rc) return rc;
    const D2Ws w = d2_carve<MODE>(ctx->ws, n);
    const bool vec = d2_vec(A, na, B, nb);
    const uint32_t key_only = MODE == DD_LWW ? 1u : g_or_key_sort ? (uint32_t)g_or_key_sort : 0u;
    const uint32_t lww_t = MODE == DD_LWW ? (uint32_t)g_lww_table : 0u, or_t = MODE == DD_OR ? (uint32_t)g_or_table : 0u;
    SortPlan h;
    // the dense-key paths from a sampled plan (sort.sample_plan): checked by
    // the composing upsweep, the call redone from the exact plan on a miss
    bool sampled = false;
    if (allow_sample && g_sample_plan && vec && (lww_t || or_t) && n >= (size_t)g_sample_min) {
        const uint64_t key0 = (uint64_t)n, key1 = (uint64_t)MODE | (uint64_t)key_only << 8 | (uint64_t)lww_t << 16 |
                                                  (uint64_t)or_t << 24 | (uint64_t)na << 32;
        const bool cached =
            g_plan_cache && ctx->d2_ok[MODE] && ctx->d2_key[MODE][0] == key0 && ctx->d2_key[MODE][1] == key1;
        if (cached && g_plan_cache == 2) {
            // sort.plan_cache = 2 (default): the last call's plan as it is --
            // these inputs' pointers, its shape and ranges -- no sample; the
            // grouping pass checks every tuple against its ranges, and one
            // outside redoes the call (as the planned calls, the plan a
            // shape validated by the whole of the last call's inputs)
            memcpy(&h, ctx->d2_plan[MODE], sizeof h);
            h.n1 = na;
            h.in2 = B;
            k_put_plan<<<1, 64, 0, s>>>(h, w.plan, w.viol);
            sampled = true;
        }
    }
    if (!sampled && allow_sample && g_sample_plan && vec && (lww_t || or_t) && n >= (size_t)g_sample_min) {
        k_sample_minmax<<<2 * SAMPLE_WG, 256, 0, s>>>(A, na, B, nb, w.mm);
        k_sort_plan<<<1, 256, 0, s>>>(w.mm, 2 * SAMPLE_WG, w.plan, 1, B, na, key_only, lww_t, or_t, (uint64_t)n, 1u,
                                      w.viol);
        // the launch shape of the last call of this kind, checked on the
        // device: no read-back (sort.plan_cache = 1)
        const uint64_t key0 = (uint64_t)n, key1 = (uint64_t)MODE | (uint64_t)key_only << 8 | (uint64_t)lww_t << 16 |
                                                  (uint64_t)or_t << 24 | (uint64_t)na << 32;
        if (g_plan_cache && ctx->d2_ok[MODE] && ctx->d2_key[MODE][0] == key0 && ctx->d2_key[MODE][1] == key1) {
            memcpy(&h, ctx->d2_plan[MODE], sizeof h);
            k_plan_match<<<1, 64, 0, s>>>(w.plan, h, w.viol);
            sampled = true;
        } else {
            rc = read_plan(ctx, w.plan, &h);
            if (rc) return rc;
            sampled = h.words == 1 && h.tw;
            ctx->d2_ok[MODE] = sampled && g_plan_cache;
            if (ctx->d2_ok[MODE]) {
                memcpy(ctx->d2_plan[MODE], &h, sizeof h);
                ctx->d2_key[MODE][0] = key0;
                ctx->d2_key[MODE][1] = key1;
            }
        }
    }
    if (!sampled) {
        const unsigned nmm = launch_minmax(ctx, A, na, B, nb, w.mm);
        k_sort_plan<<<1, 256, 0, s>>>(w.mm, nmm, w.plan, 1, B, na, key_only, lww_t, or_t, (uint64_t)n);
        rc = read_plan(ctx, w.plan, &h);
        if (rc) return rc;
    }
    bool miss = false;
    rc = d2_body<MODE>(ctx, A, na, B, nb, *out, out_count, w, h, sampled ? w.viol : nullptr, vec, false, &miss);
    if (rc) return rc;
    if (!miss) return CRDT_OK;
    ctx->d2_ok[MODE] = false;                           // (a shape change: the next call reads its plan back)
    return set_merge_unsorted<MODE>(ctx, a, na, b, nb, out, out_count, false);
}

// ---------------------------------------------------------------- planned D2 merges
// crdt_set_merge_plan's opaque result: the plan of one (mode, na, nb) shape.
struct PlanBlob {
    uint32_t magic, mode;
    uint64_t na, nb;
    SortPlan h;
};
constexpr uint32_t kPlanMagic = 0x43524450u;     // "CRDP"
static_assert(sizeof(PlanBlob) <= sizeof(crdt_set_plan), "crdt_set_plan holds the plan");

static int set_merge_plan(crdt_ctx *ctx, int mode, const crdt_tuples *a, size_t na, const crdt_tuples *b, size_t nb,
                          uint32_t widen, crdt_set_plan *plan) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!plan || (mode != DD_LWW && mode != DD_OR)) return CRDT_E_INVAL;
    if ((na && !tuples_full(a)) || (nb && !tuples_full(b))) return CRDT_E_INVAL;
    const size_t n = na + nb;
    if (n >= (1ULL << 32)) return CRDT_E_RANGE;
    const crdt_tuples none{nullptr, nullptr, nullptr, nullptr};
    const crdt_tuples A = na ? *a : none, B = nb ? *b : none;
    // the planned calls run in the workspace reserved here (no allocation
    // inside a captured graph)
    rc = ws_reserve(ctx, mode == DD_LWW ? d2_ws_bytes<DD_LWW>(n) : d2_ws_bytes<DD_OR>(n));
    if (!rc) rc = hio_reserve(ctx, 16);
    if (rc) return rc;
    PlanBlob pb{};
    pb.magic = kPlanMagic;
    pb.mode = (uint32_t)mode;
    pb.na = na;
    pb.nb = nb;
    if (n) {
        const D2Ws w = mode == DD_LWW ? d2_carve<DD_LWW>(ctx->ws, n) : d2_carve<DD_OR>(ctx->ws, n);
        const uint32_t key_only = mode == DD_LWW ? 1u : g_or_key_sort ? (uint32_t)g_or_key_sort : 0u;
        const uint32_t lww_t = mode == DD_LWW ? (uint32_t)g_lww_table : 0u, or_t = mode == DD_OR ? (uint32_t)g_or_table : 0u;
        const unsigned nmm = launch_minmax(ctx, A, na, B, nb, w.mm);
        k_sort_plan<<<1, 256, 0, ctx->stream>>>(w.mm, nmm, w.plan, 1, B, na, key_only, lww_t, or_t, (uint64_t)n,
                                                widen ? 1u : 0u);
        rc = read_plan(ctx, w.plan, &pb.h);
        if (rc) return rc;
    }
    memset(plan, 0, sizeof *plan);
    memcpy(plan, &pb, sizeof pb);
    return CRDT_OK;
}

template <int MODE>
static int set_merge_planned(crdt_ctx *ctx, const crdt_set_plan *plan, const crdt_tuples *a, size_t na,
                             const crdt_tuples *b, size_t nb, crdt_tuples *out, uint64_t *out_count) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!plan) return CRDT_E_INVAL;
    PlanBlob pb;
    memcpy(&pb, plan, sizeof pb);
    if (pb.magic != kPlanMagic || pb.mode != (uint32_t)MODE || pb.na != na || pb.nb != nb) return CRDT_E_INVAL;
    rc = d2_args(a, na, b, nb, out, out_count);
    if (rc) return rc;
    const size_t n = na + nb;
    const hipStream_t s = ctx->stream;
    if (n == 0) {
        hipError_t e = hipMemsetAsync(out_count, 0, sizeof(uint64_t), s);
        return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
    }
    if (ctx->ws_bytes < d2_ws_bytes<MODE>(n)) return CRDT_E_INVAL;   // (the plan call reserved it)
    const crdt_tuples none{nullptr, nullptr, nullptr, nullptr};
    const crdt_tuples A = na ? *a : none, B = nb ? *b : none;
    const D2Ws w = d2_carve<MODE>(ctx->ws, n);
    SortPlan h = pb.h;
    h.in2 = B;                                          // (the plan's shape, these inputs)
    h.n1 = na;
    k_put_plan<<<1, 64, 0, s>>>(h, w.plan, w.viol);
    rc = check_launch(ctx);
    if (rc) return rc;
    bool miss = false;
    return d2_body<MODE>(ctx, A, na, B, nb, *out, out_count, w, h, w.viol, d2_vec(A, na, B, nb), true, &miss);
}
}  // namespace crdt

using namespace crdt;

extern "C" int crdt_u64_lower_bound(crdt_ctx *ctx, const uint64_t *sorted, size_t n, const uint64_t *probes, size_t m,
                                    uint64_t *out) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (m == 0) return CRDT_OK;
    if (!probes || !out || (n && !sorted)) return CRDT_E_INVAL;
    k_lower_bound_u64<<<grid_for(m, 256, (unsigned)ctx->num_cus * 4), 256, 0, ctx->stream>>>(sorted, n, probes, m, out);
    return check_launch(ctx);
}

extern "C" int crdt_tuples_sort(crdt_ctx *ctx, const crdt_tuples *in, size_t n, crdt_tuples *out) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!in || !out) return CRDT_E_INVAL;
    if (n == 0) return CRDT_OK;
    if (!in->key || !in->ts || !in->rep || !in->tomb || !out->key || !out->ts || !out->rep || !out->tomb)
        return CRDT_E_INVAL;
    if (n >= (1ULL << 32)) return CRDT_E_RANGE;       // 32-bit in-tile / bucket arithmetic
    const size_t ntiles = (n + ST - 1) / ST, ncnt = ntiles * 256;
    const size_t b_mm = Carve::round(2 * MM_BLOCKS * sizeof(SortMinMax)), b_plan = Carve::round(sizeof(SortPlan));
    const size_t b_cnt = Carve::round(ncnt * 4), b_tot = Carve::round(256 * 4), b_bufs = Carve::round(2 * 3 * n * 8);
    rc = ws_reserve(ctx, b_mm + b_plan + 2 * b_cnt + b_tot + b_bufs + 1024);
    if (rc) return rc;
    Carve w(ctx->ws);
    SortMinMax *mm = w.take<SortMinMax>(2 * MM_BLOCKS);
    SortPlan *plan = w.take<SortPlan>(1);
    uint32_t *cnt = w.take<uint32_t>(ncnt);
    uint32_t *loc = w.take<uint32_t>(ncnt);
    uint32_t *tot = w.take<uint32_t>(256);
    uint64_t *bufs = w.take<uint64_t>(2 * 3 * n);
    const hipStream_t s = ctx->stream;
    const unsigned nmm = launch_minmax(ctx, *in, n, crdt_tuples{nullptr, nullptr, nullptr, nullptr}, 0, mm);
    k_sort_plan<<<1, 256, 0, s>>>(mm, nmm, plan, 0, crdt_tuples{nullptr, nullptr, nullptr, nullptr}, n);
    // the pass count and composite width decide the launches: one small read-back
    SortPlan h;
    rc = read_plan(ctx, plan, &h);
    if (rc) return rc;
    if (h.words == 1) return sort_words<1>(ctx, *in, n, *out, plan, h.P, bufs, cnt, loc, tot);
    if (h.words == 2) return sort_words<2>(ctx, *in, n, *out, plan, h.P, bufs, cnt, loc, tot);
    return sort_words<3>(ctx, *in, n, *out, plan, h.P, bufs, cnt, loc, tot);
}

extern "C" int crdt_lww_merge_unsorted(crdt_ctx *ctx, const crdt_tuples *a, size_t na, const crdt_tuples *b,
                                       size_t nb, crdt_tuples *out, uint64_t *out_count_dev) {
    return set_merge_unsorted<DD_LWW>(ctx, a, na, b, nb, out, out_count_dev);
}

extern "C" int crdt_orset_merge_unsorted(crdt_ctx *ctx, const crdt_tuples *a, size_t na, const crdt_tuples *b,
                                         size_t nb, crdt_tuples *out, uint64_t *out_count_dev) {
    return set_merge_unsorted<DD_OR>(ctx, a, na, b, nb, out, out_count_dev);
}

extern "C" int crdt_set_merge_plan(crdt_ctx *ctx, int mode, const crdt_tuples *a, size_t na, const crdt_tuples *b,
                                   size_t nb, uint32_t widen, crdt_set_plan *plan) {
    return set_merge_plan(ctx, mode, a, na, b, nb, widen, plan);
}

extern "C" int crdt_lww_merge_unsorted_planned(crdt_ctx *ctx, const crdt_set_plan *plan, const crdt_tuples *a,
                                               size_t na, const crdt_tuples *b, size_t nb, crdt_tuples *out,
                                               uint64_t *out_count_dev) {
    return set_merge_planned<DD_LWW>(ctx, plan, a, na, b, nb, out, out_count_dev);
}

extern "C" int crdt_orset_merge_unsorted_planned(crdt_ctx *ctx, const crdt_set_plan *plan, const crdt_tuples *a,
                                                 size_t na, const crdt_tuples *b, size_t nb, crdt_tuples *out,
                                                 uint64_t *out_count_dev) {
    return set_merge_planned<DD_OR>(ctx, plan, a, na, b, nb, out, out_count_dev);
}
