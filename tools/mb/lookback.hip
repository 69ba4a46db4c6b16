// lookback.hip -- does XCD-local tile placement make a single-pass decoupled
// look-back pay on MI355X?  (the fused set merge with the
// XCD-contiguous tile mapping)
//
// The fused set merge is a single-pass, look-back-chained kernel: per tile,
// stage + merge + count, publish the count, look back for the offset, store.
// This microbenchmark strips it to the chain itself -- an exclusive scan of
// 16M u32 in 4096-item tiles -- and times
//   * reduce / scan / apply (three launches, no waiting: the two-pass form);
//   * one pass, tiles in blockIdx order (consecutive tiles on different XCDs,
//     blocks being dealt round-robin over the 8 XCDs);
//   * one pass, XCD-chunked: XCD x takes chunks x, x + 8, x + 16, ... of C
//     consecutive tiles (a tile's predecessor is on its own XCD except at
//     chunk starts; C = 512 is one contiguous range per XCD);
//   * one pass without the look-back (timing only, wrong offsets).
// Status words are single 8-byte {flag, value} agent-scope atomics (one
// granule: no separate payload ordering, MI355X_MICROARCH.md "Valid forms").
// Spins are bounded (s_sleep between polls): a tile whose predecessor never
// publishes raises an error count instead of hanging.
//
// build: hipcc -O3 --offload-arch=gfx950 -o tools/mb/lookback tools/mb/lookback.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef TBV
#define TBV 256
#endif
#ifndef IPTV
#define IPTV 16
#endif
constexpr int TB = TBV, IPT = IPTV, TILE = TB * IPT;   // -DTBV=1024 for 16k-item tiles
constexpr unsigned long long FLAG_A = 1ull << 62, FLAG_P = 2ull << 62, VAL = (1ull << 62) - 1;

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

__device__ __forceinline__ uint32_t tile_of(uint32_t b, uint32_t chunk) {
    if (chunk == 0) return b;                              // blockIdx order
    const uint32_t x = b & 7u, q = b >> 3;
    return ((q / chunk) * 8u + x) * chunk + q % chunk;
}

// block exclusive scan of one value per thread; *tot = the block total
__device__ __forceinline__ uint64_t block_scan(uint64_t v, uint64_t *tot) {
    __shared__ uint64_t s_w[TB / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint64_t off = 0, all = 0;
#pragma unroll
    for (int k = 0; k < TB / 64; ++k) {
        off += k < w ? s_w[k] : 0;
        all += s_w[k];
    }
    __syncthreads();
    *tot = all;
    return off + x - v;
}

// Striped tile layout (round 6, VERDICT r05: the blocked layout above ran
// the no-look-back pass at half the copy rate -- each uint4 load touched 16 B
// of every 64 B across the wave): item (k, lane-major) = tile + (k * TB +
// tid) * 2 + j, so every load (u32x2) and store (u64x2) instruction covers a
// contiguous span of the wave.  Late round 6 (tools/mb/copy_shapes.hip,
// profiles/r06/copy_shapes.txt): the earlier u32x4 loads with two u64x2
// nontemporal stores 32 B apart ran the copy at 3.3 TB/s; this shape with
// default-policy stores runs it at 5.7-5.9 TB/s.  The block scan runs over the
// IPT / 2 groups in k-major order: wave scans of the group sums at once, one
// barrier.
constexpr int G = IPT / 2;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint64_t u64x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void load_striped(const uint32_t *__restrict__ in, size_t tile0, uint32_t (&v)[IPT],
                                             uint64_t (&s)[G]) {
#pragma unroll
    for (int k = 0; k < G; ++k) {
        const u32x2 q = __builtin_nontemporal_load((const u32x2 *)(in + tile0 + ((size_t)k * TB + threadIdx.x) * 2));
        v[2 * k] = q.x, v[2 * k + 1] = q.y;
        s[k] = (uint64_t)q.x + q.y;
    }
}
// in place: s[k] (the group sum of (k, tid)) -> its exclusive prefix within
// the tile; returns the tile total
__device__ __forceinline__ uint64_t block_scan_g(uint64_t (&s)[G]) {
    __shared__ uint64_t s_w[G][TB / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t x[G];
#pragma unroll
    for (int k = 0; k < G; ++k) x[k] = s[k];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const uint64_t y = __shfl_up(x[k], o);
            if (lane >= o) x[k] += y;
        }
    }
    if (lane == 63) {
#pragma unroll
        for (int k = 0; k < G; ++k) s_w[k][w] = x[k];
    }
    __syncthreads();
    // the wave sums of group k scanned by the first TB / 64 lanes of every
    // wave (shuffles, no unrolled LDS sweep: at TB = 1024 that spilled)
    constexpr int NW = TB / 64;
    uint64_t run = 0;
#pragma unroll
    for (int k = 0; k < G; ++k) {
        const uint64_t ws = lane < NW ? s_w[k][lane] : 0;
        uint64_t inc = ws;
#pragma unroll
        for (int o = 1; o < NW; o <<= 1) {
            const uint64_t y = __shfl_up(inc, o);
            if (lane >= o) inc += y;
        }
        const uint64_t before = __shfl(inc - ws, w), all = __shfl(inc, NW - 1);
        s[k] = run + before + x[k] - s[k];
        run += all;
    }
    __syncthreads();
    return run;
}
__device__ __forceinline__ void store_striped(uint64_t *__restrict__ out, size_t tile0, const uint32_t (&v)[IPT],
                                              const uint64_t (&ex)[G], uint64_t base) {
#pragma unroll
    for (int k = 0; k < G; ++k) {
        const uint64_t r = base + ex[k];
        *(u64x2v *)(out + tile0 + ((size_t)k * TB + threadIdx.x) * 2) = (u64x2v){r, r + v[2 * k]};
    }
}

// the 64-lane window look-back of status word t (wave 0 calls it, every
// lane): publishes tot, returns the exclusive prefix
__device__ __forceinline__ uint64_t window_lookback(unsigned long long *st, uint32_t t, uint64_t tot, int lane,
                                                    unsigned *err) {
    uint64_t pre = 0;
    if (t == 0) {
        if (lane == 0) __hip_atomic_store(&st[0], FLAG_P | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(&st[t], FLAG_A | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int64_t j = (int64_t)t - 1;                             // window [j - 63, j], lane l reads j - l
    uint32_t spins = 0;
    for (;;) {
        const int64_t q = j - lane;
        const unsigned long long w =
            q >= 0 ? __hip_atomic_load(&st[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : FLAG_P;
        const uint64_t isp = __ballot((w & ~VAL) == FLAG_P), nr = __ballot((w & ~VAL) == 0);
        const int pl = isp ? __ffsll((long long)isp) - 1 : 64;
        const uint64_t need = pl >= 63 ? ~0ull : ((2ull << pl) - 1ull);
        if (nr & need) {
            if (++spins > (1u << 20)) {
                if (lane == 0) atomicAdd(err, 1u);
                break;
            }
            if (spins > 1) __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint64_t v = lane <= pl ? (w & VAL) : 0;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        pre += v;
        if (pl < 64) break;
        j -= 64;
    }
    if (lane == 0) __hip_atomic_store(&st[t], FLAG_P | (pre + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return pre;
}

// VERDICT r05 item 1's form: one workgroup per chunk of C consecutive tiles.
// Phase 1 loads and sums the C tiles; wave 0 publishes the chunk total and
// looks back ONCE (64-lane window; LB = false: no look-back, wrong offsets,
// timing only); phase 2 loads the C tiles again (served by L2 / MALL when
// they are still there), scans and stores them.  Reads 2x the input.
template <bool LB>
__global__ __launch_bounds__(TB) void k_chunked(const uint32_t *__restrict__ in, uint64_t *__restrict__ out,
                                                unsigned long long *st, uint32_t C, unsigned *err) {
    __shared__ uint64_t s_base, s_red[TB / 64];
    const uint32_t ch = blockIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t sum = 0;
    for (uint32_t c = 0; c < C; ++c) {
        const size_t tile0 = ((size_t)ch * C + c) * TILE;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const u32x2 q = __builtin_nontemporal_load((const u32x2 *)(in + tile0 + ((size_t)k * TB + threadIdx.x) * 2));
            sum += (uint64_t)q.x + q.y;
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if (lane == 0) s_red[w] = sum;
    __syncthreads();
    if (w == 0) {
        uint64_t tot = 0;
#pragma unroll
        for (int k = 0; k < TB / 64; ++k) tot += s_red[k];
        const uint64_t pre = LB ? window_lookback(st, ch, tot, lane, err) : (uint64_t)ch * C * TILE * 512;
        if (lane == 0) s_base = pre;
    }
    __syncthreads();
    uint64_t base = s_base;
    for (uint32_t c = 0; c < C; ++c) {
        const size_t tile0 = ((size_t)ch * C + c) * TILE;
        uint32_t v[IPT];
        uint64_t ex[G];
        load_striped(in, tile0, v, ex);
        const uint64_t tt = block_scan_g(ex);
        store_striped(out, tile0, v, ex, base);
        base += tt;
    }
}

// mode 0: serial look-back by one thread; mode 1: no look-back (timing only);
// mode 2: 64-lane window look-back (one status per lane, a ballot for the
// first inclusive flag, a wave reduction; first poll without s_sleep)
template <int MODE>
__global__ __launch_bounds__(TB) void k_onepass(const uint32_t *__restrict__ in, uint64_t *__restrict__ out,
                                                unsigned long long *st, uint32_t chunk, unsigned *err) {
    __shared__ uint64_t s_base;
    const uint32_t t = tile_of(blockIdx.x, chunk);
    const size_t tile0 = (size_t)t * TILE;
    uint32_t v[IPT];
    uint64_t ex[G];
    load_striped(in, tile0, v, ex);
    const uint64_t tot = block_scan_g(ex);
    if (MODE == 2) {                                        // 64-lane window look-back by wave 0
        if (threadIdx.x < 64) {
            const uint64_t pre = window_lookback(st, t, tot, threadIdx.x, err);
            if (threadIdx.x == 0) s_base = pre;
        }
    } else if (threadIdx.x == 0) {
        uint64_t pre = 0;
        if (MODE == 0) {
            if (t == 0) {
                __hip_atomic_store(&st[0], FLAG_P | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                __hip_atomic_store(&st[t], FLAG_A | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                int64_t j = (int64_t)t - 1;
                uint32_t spins = 0;
                while (j >= 0) {
                    const unsigned long long w = __hip_atomic_load(&st[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if ((w & ~VAL) == 0) {
                        if (++spins > (1u << 20)) {          // bounded: report, never hang
                            atomicAdd(err, 1u);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                        continue;
                    }
                    pre += w & VAL;
                    if ((w & ~VAL) == FLAG_P) break;
                    --j;
                }
                __hip_atomic_store(&st[t], FLAG_P | (pre + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        s_base = pre;
    }
    __syncthreads();
    store_striped(out, tile0, v, ex, s_base);
}

__global__ __launch_bounds__(TB) void k_reduce(const uint32_t *__restrict__ in, uint64_t *__restrict__ sums) {
    uint32_t v[IPT];
    uint64_t ex[G];
    load_striped(in, (size_t)blockIdx.x * TILE, v, ex);
    const uint64_t tot = block_scan_g(ex);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void k_scan_sums(uint64_t *sums, uint32_t n) {
    __shared__ uint64_t s_w[16];
    const uint32_t per = (n + 1023) / 1024, b = threadIdx.x * per, e = b + per < n ? b + per : n;
    uint64_t s = 0;
    for (uint32_t i = b; i < e && i < n; ++i) s += sums[i];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t x = s;
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint64_t off = 0;
    for (int k = 0; k < w; ++k) off += s_w[k];
    uint64_t run = off + x - s;
    for (uint32_t i = b; i < e && i < n; ++i) {
        const uint64_t v = sums[i];
        sums[i] = run;
        run += v;
    }
}

__global__ __launch_bounds__(TB) void k_apply(const uint32_t *__restrict__ in, const uint64_t *__restrict__ sums,
                                              uint64_t *__restrict__ out) {
    uint32_t v[IPT];
    uint64_t ex[G];
    const size_t tile0 = (size_t)blockIdx.x * TILE;
    load_striped(in, tile0, v, ex);
    (void)block_scan_g(ex);
    store_striped(out, tile0, v, ex, sums[blockIdx.x]);
}

// the copy-rate reference of this access pattern: read the u32s, write u64s
__global__ __launch_bounds__(TB) void k_copy(const uint32_t *__restrict__ in, uint64_t *__restrict__ out) {
    uint32_t v[IPT];
    uint64_t ex[G];
    const size_t tile0 = (size_t)blockIdx.x * TILE;
    load_striped(in, tile0, v, ex);
    const uint64_t b = ex[0];
#pragma unroll
    for (int k = 0; k < G; ++k) ex[k] = 0;
    store_striped(out, tile0, v, ex, b);
}

int main(int argc, char **argv) {
    const uint32_t ntiles = argc > 1 ? (uint32_t)atoi(argv[1]) : 4096;     // multiple of 8 * 512
    const size_t n = (size_t)ntiles * TILE;
    const int reps = 20;
    std::vector<uint32_t> h(n);
    uint64_t seed = 88172645463325252ull;
    for (size_t i = 0; i < n; ++i) {
        seed ^= seed << 13, seed ^= seed >> 7, seed ^= seed << 17;
        h[i] = (uint32_t)(seed & 1023);
    }
    std::vector<uint64_t> ref(n);
    uint64_t run = 0;
    for (size_t i = 0; i < n; ++i) ref[i] = run, run += h[i];
    uint32_t *d_in;
    uint64_t *d_out, *d_sums;
    unsigned long long *d_st;
    unsigned *d_err;
    CK(hipMalloc(&d_in, n * 4));
    CK(hipMalloc(&d_out, n * 8));
    CK(hipMalloc(&d_sums, ntiles * 8));
    CK(hipMalloc(&d_st, ntiles * 8));
    CK(hipMalloc(&d_err, 4));
    CK(hipMemcpy(d_in, h.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(d_err, 0, 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<uint64_t> got(n);
    auto check = [&](const char *name) {
        CK(hipMemcpy(got.data(), d_out, n * 8, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < n; ++i) bad += got[i] != ref[i];
        unsigned err = 0;
        CK(hipMemcpy(&err, d_err, 4, hipMemcpyDeviceToHost));
        printf("  %-28s check: %zu wrong, %u spin timeouts\n", name, bad, err);
    };
    auto timeit = [&](const char *name, auto fn, bool verify) {
        fn();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) fn();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-30s %8.1f us  (%.2f TB/s of in + out)\n", name, ms * 1e3 / reps,
               (double)n * 12 / (ms * 1e-3 / reps) / 1e12);
        if (verify) check(name);
    };
    printf("exclusive scan of %zu u32 (%u tiles of %d), 20 reps\n", n, ntiles, TILE);
    timeit("reduce/scan/apply (3 launches)", [&] {
        k_reduce<<<ntiles, TB>>>(d_in, d_sums);
        k_scan_sums<<<1, 1024>>>(d_sums, ntiles);
        k_apply<<<ntiles, TB>>>(d_in, d_sums, d_out);
    }, true);
    timeit("copy (no scan: the access-pattern peak)", [&] { k_copy<<<ntiles, TB>>>(d_in, d_out); }, false);
    timeit("one pass, no look-back", [&] { k_onepass<1><<<ntiles, TB>>>(d_in, d_out, d_st, 0, d_err); }, false);
    const uint32_t chunks[] = {0, 1, 4, 16, 64, 512};
    for (uint32_t c : chunks) {
        if (c && ntiles % (8 * c)) continue;
        char name[64];
        if (c == 0) snprintf(name, sizeof name, "look-back, blockIdx order");
        else snprintf(name, sizeof name, "look-back, XCD chunks of %u", c);
        timeit(name, [&] {
            (void)hipMemsetAsync(d_st, 0, ntiles * 8);
            k_onepass<0><<<ntiles, TB>>>(d_in, d_out, d_st, c, d_err);
        }, true);
        if (c == 0) snprintf(name, sizeof name, "window look-back, blockIdx");
        else snprintf(name, sizeof name, "window look-back, XCD chunks %u", c);
        timeit(name, [&] {
            (void)hipMemsetAsync(d_st, 0, ntiles * 8);
            k_onepass<2><<<ntiles, TB>>>(d_in, d_out, d_st, c, d_err);
        }, true);
    }
    const uint32_t cs[] = {1, 2, 4, 8};
    for (uint32_t c : cs) {
        if (ntiles % c) continue;
        char name[64];
        snprintf(name, sizeof name, "chunks of %u tiles, no look-back", c);
        timeit(name, [&] { k_chunked<false><<<ntiles / c, TB>>>(d_in, d_out, d_st, c, d_err); }, false);
        snprintf(name, sizeof name, "chunks of %u tiles, look-back", c);
        timeit(name, [&] {
            (void)hipMemsetAsync(d_st, 0, ntiles * 8);
            k_chunked<true><<<ntiles / c, TB>>>(d_in, d_out, d_st, c, d_err);
        }, true);
    }
    timeit("memset of the status words", [&] { (void)hipMemsetAsync(d_st, 0, ntiles * 8); }, false);
    CK(hipFree(d_in));
    CK(hipFree(d_out));
    CK(hipFree(d_sums));
    CK(hipFree(d_st));
    CK(hipFree(d_err));
    return 0;
}
