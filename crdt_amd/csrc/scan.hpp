// scan.hpp -- block-level scan helpers for 256-lane (4-wave) workgroups.
#pragma once
#include "common.hpp"

namespace crdt {

// Exclusive scan of one uint64 per lane across a 256-lane block; *total gets
// the block sum.  Every lane of the block must call it (contains barriers).
__device__ __forceinline__ uint64_t block_exclusive_scan_u64(uint64_t v, uint64_t *total) {
    __shared__ uint64_t wsum[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint64_t off = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint64_t s = wsum[k];
        off += (k < w) ? s : 0;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return off + x - v;
}

// Exclusive rank of a per-lane predicate across the 256-lane block using
// wave ballots (mbcnt) -- cheaper than the generic scan for 0/1 flags.
__device__ __forceinline__ uint32_t block_rank_flag(bool f, uint32_t *total) {
    __shared__ uint32_t wcnt[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t m = __ballot(f);
    const uint32_t below = (uint32_t)__popcll(m & ((lane == 0) ? 0ULL : (~0ULL >> (64 - lane))));
    if (lane == 0) wcnt[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t s = wcnt[k];
        off += (k < w) ? s : 0;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return off + below;
}

// ---- device-wide exclusive scan: reduce, scan the tile sums, apply --------
// Tile = 256 lanes x N items.  Three launches with no cross-workgroup
// waiting: per-tile sums, a one-workgroup scan of the sums, then every tile
// re-loads its items, scans them locally from its tile offset and stores the
// offsets (plus Act::apply on the lane's items, e.g. the copy of the
// segments, so producing and consuming the offsets is one pass).
// Why not a single pass with a decoupled look-back: the 8 XCDs' L2s are not
// coherent with each other, so every status word and ticket is a
// memory-side round trip; measured at 16M items (tools/bench_seg.py) the
// ticket and the look-back each cost about as much as the whole streaming
// pass (130 us single-pass vs 32 us for the apply pass alone).
// Items are loaded striped (coalesced), summed blocked through LDS, and the
// offsets stored striped again.  Src::load(i) returns an Item with a .len.
constexpr int kLbMinItems = 4;      // workspace is sized for the smallest tile
// items per lane: g_scan_items (knobs.inc "scan.items": 4, 8, 16)

struct NoAct {
    template <int N, class Item>
    __device__ void apply(const Item *, const uint64_t *) const {}
};

__device__ __forceinline__ int lb_pad(int i) { return i + (i >> 3); }

// branch-free (clamped index) so the loads of all items are in flight together
template <int N, class Src>
__device__ __forceinline__ void scan_load(const Src &src, uint64_t n, uint64_t tb, typename Src::Item *it) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int r = 0; r < N; ++r) {
        const uint64_t i = tb + (uint64_t)r * 256 + tid;
        if (n) it[r] = src.load(i < n ? i : n - 1);     // n == 0: one empty tile, nothing to load
    }
#pragma unroll
    for (int r = 0; r < N; ++r)
        if (tb + (uint64_t)r * 256 + tid >= n) it[r].len = 0;
}

template <int N, class Src>
__global__ __launch_bounds__(256) void k_scan_reduce(Src src, uint64_t n, uint64_t *__restrict__ tsum) {
    __shared__ uint64_t wsum[4];
    typename Src::Item it[N];
    scan_load<N>(src, n, (uint64_t)blockIdx.x * 256 * N, it);
    uint64_t s = 0;
#pragma unroll
    for (int r = 0; r < N; ++r) s += it[r].len;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) tsum[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// one workgroup: tsum[t] <- base + exclusive prefix; out[n] = base + total
static __global__ __launch_bounds__(256) void k_scan_tsums(uint64_t *__restrict__ tsum, uint64_t nt, uint64_t base,
                                                    uint64_t *__restrict__ out_n) {
    constexpr int K = 16;
    uint64_t carry = base;
    for (uint64_t b0 = 0; b0 < nt; b0 += 256 * K) {
        const uint64_t i0 = b0 + (uint64_t)threadIdx.x * K;
        uint64_t v[K], s = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            v[k] = i0 + k < nt ? tsum[i0 + k] : 0;
            s += v[k];
        }
        uint64_t tot;
        uint64_t run = carry + block_exclusive_scan_u64(s, &tot);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (i0 + k < nt) tsum[i0 + k] = run;
            run += v[k];
        }
        carry += tot;
    }
    if (threadIdx.x == 0) *out_n = carry;
}

// One workgroup of NT threads scans n <= R * NT values (exclusive, u64
// prefixes), read STRIPED: row r is items [r NT, (r + 1) NT), item r NT + tid
// per thread, so every load and store of a wave is one contiguous piece and
// all R loads are in flight at once.  Rows are scanned per wave by shuffles;
// wave 0 scans the rows' wave totals (row-major) in LDS; put(i, prefix) then
// stores striped.  Two barriers; returns the total.  (A contiguous run per
// thread made every access a strided one, which one workgroup's address unit
// pays per cache line: 11.7 us for 9.8k tile counts.)  s_pre: R * NT / 64 + 1.
template <int NT, int R, typename V, class Get, class Put>
__device__ __forceinline__ uint64_t wg_scan_rows(Get get, uint32_t n, Put put, uint64_t *s_pre) {
    constexpr int W = NT / 64;
    static_assert(R * W <= 4 * 64, "wave 0 scans the wave totals, four per lane");
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t nr = (n + NT - 1) / NT;            // rows present (uniform)
    V v[R], y[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i = (uint32_t)r * NT + (uint32_t)tid;
        v[r] = i < n ? (V)get(i) : (V)0;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        y[r] = 0;
        if ((uint32_t)r < nr) {                       // (uniform)
            V x = v[r];
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const V t = __shfl_up(x, o, 64);
                if (lane >= o) x += t;
            }
            y[r] = x;
            if (lane == 63) s_pre[r * W + w] = (uint64_t)x;
        }
    }
    __syncthreads();
    if (w == 0) {
        uint64_t a[4], sum = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t j = (uint32_t)lane * 4 + k;
            a[k] = j < nr * W ? s_pre[j] : 0;
            sum += a[k];
        }
        uint64_t x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t t = __shfl_up(x, o, 64);
            if (lane >= o) x += t;
        }
        uint64_t run = x - sum;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t j = (uint32_t)lane * 4 + k;
            if (j < nr * W) s_pre[j] = run;
            run += a[k];
        }
        if (lane == 63) s_pre[R * W] = x;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i = (uint32_t)r * NT + (uint32_t)tid;
        if ((uint32_t)r < nr && i < n) put(i, s_pre[r * W + w] + (uint64_t)(y[r] - v[r]));
    }
    return s_pre[R * W];
}

template <int N, class Src, class Act>
__global__ __launch_bounds__(256) void k_scan_apply(Src src, Act act, uint64_t n, const uint64_t *__restrict__ tsum,
                                                    uint64_t *__restrict__ out) {
    constexpr int kTile = 256 * N;
    __shared__ uint64_t buf[kTile + kTile / 8];
    __shared__ uint64_t wtot[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t tb = (uint64_t)blockIdx.x * kTile;
    typename Src::Item it[N];
    scan_load<N>(src, n, tb, it);
#pragma unroll
    for (int r = 0; r < N; ++r) buf[lb_pad(r * 256 + tid)] = it[r].len;
    __syncthreads();
    uint64_t v[N], sum = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        v[k] = buf[lb_pad(tid * N + k)];
        sum += v[k];
    }
    uint64_t x = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wtot[w] = x;
    __syncthreads();
    uint64_t run = tsum[blockIdx.x] + x - sum;
#pragma unroll
    for (int k = 0; k < 4; ++k) run += k < w ? wtot[k] : 0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        buf[lb_pad(tid * N + k)] = run;
        run += v[k];
    }
    __syncthreads();
    uint64_t d[N];
#pragma unroll
    for (int r = 0; r < N; ++r) {
        const uint64_t i = tb + (uint64_t)r * 256 + tid;
        d[r] = buf[lb_pad(r * 256 + tid)];
        if (i < n) out[i] = d[r];
    }
    act.template apply<N>(it, d);   // items past n have len 0
}

// Workspace for scan_lb: the tile sums.
inline size_t scan_lb_tmp_bytes(size_t n) {
    const size_t tile = 256 * kLbMinItems, nt = n ? (n + tile - 1) / tile : 1;
    return Carve::round((nt + 1) * sizeof(uint64_t));
}

template <int N, class Src, class Act>
int scan_lb_n(crdt_ctx *ctx, const Src &src, const Act &act, size_t n, uint64_t base, uint64_t *out, void *tmp) {
    const size_t tile = 256 * N, nt = n ? (n + tile - 1) / tile : 1;
    if (nt > 0xffffffffULL) return CRDT_E_RANGE;
    uint64_t *tsum = (uint64_t *)tmp;
    k_scan_reduce<N, Src><<<(unsigned)nt, 256, 0, ctx->stream>>>(src, n, tsum);
    k_scan_tsums<<<1, 256, 0, ctx->stream>>>(tsum, nt, base, out + n);
    k_scan_apply<N, Src, Act><<<(unsigned)nt, 256, 0, ctx->stream>>>(src, act, n, tsum, out);
    return check_launch(ctx);
}

// out[i] = base + sum(len(0..i)), out[n] = base + total; tmp from scan_lb_tmp_bytes(n).
template <class Src, class Act>
int scan_lb(crdt_ctx *ctx, const Src &src, const Act &act, size_t n, uint64_t base, uint64_t *out, void *tmp) {
    if (g_scan_items == 4) return scan_lb_n<4>(ctx, src, act, n, base, out, tmp);
    if (g_scan_items == 16) return scan_lb_n<16>(ctx, src, act, n, base, out, tmp);
    return scan_lb_n<8>(ctx, src, act, n, base, out, tmp);
}

struct CountSrc {
    const uint32_t *in;
    struct Item {
        uint64_t len = 0;
    };
    __device__ Item load(uint64_t i) const { return Item{in[i]}; }
};


// Decoupled look-back (OR-Set D2 chunks, the fused D1 set merges): status
// word per tile / chunk -- kOcA | count once counted, kOcP | inclusive prefix
// once resolved, 0 not yet published.  Tiles are dispatched in index order,
// so every polled one has been dispatched; polls are bounded
// (CRDT_DEV_LOOKBACK).
constexpr unsigned long long kOcA = 1ull << 62, kOcP = 2ull << 62, kOcVal = (1ull << 62) - 1;
// The sum of chunk counts from chunk j back to the nearest inclusive prefix
// (that prefix included): one wave, each lane loading U consecutive status
// words per window (64 U chunks per round trip; the aggregates are all
// published early, so a walk that has to reach far back costs round trips,
// not waits).  Polls bounded: CRDT_DEV_LOOKBACK, never a hang.
template <int U>
__device__ unsigned long long lookback_sum(const unsigned long long *st, long long j, int lane, uint32_t *err) {
    unsigned long long acc = 0;
    uint32_t spins = 0;
    for (;;) {
        unsigned long long f[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long q = j - (long long)(lane * U + u);
            f[u] = q >= 0 ? __hip_atomic_load(&st[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kOcP;
        }
        int fu = U;                                   // this lane's nearest inclusive prefix
#pragma unroll
        for (int u = U - 1; u >= 0; --u)
            if ((f[u] >> 62) == 2) fu = u;
        const uint64_t isp = __ballot(fu < U);
        const int pl = isp ? __ffsll((long long)isp) - 1 : 64;
        const int upto = lane < pl ? U - 1 : lane == pl ? fu : -1;   // this lane's words in the sum
        bool nr = false;
#pragma unroll
        for (int u = 0; u < U; ++u) nr = nr || (u <= upto && (f[u] >> 62) == 0);
        if (__ballot(nr)) {
            if (++spins > (1u << 22)) {               // bounded: report, never hang
                if (lane == 0) atomicOr(err, CRDT_DEV_LOOKBACK);
                return acc;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        unsigned long long v = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) v += u <= upto ? (f[u] & kOcVal) : 0ull;
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        acc += v;
        if (pl < 64) return acc;
        j -= 64 * U;
    }
}

}  // namespace crdt
