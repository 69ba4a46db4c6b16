// copy_shapes.hip -- which load / store shape lets a tiled "u32 in, u64 out"
// pass (the look-back microbenchmark's access pattern, tools/mb/lookback.hip)
// reach the streaming rate?  VERDICT r05 item 1: the microbenchmark's copy
// line ran at 2.6 TB/s, so its look-back A/B could not bound the product.
//
// Every kernel moves 64M u32 in and 64M u64 out (805 MB) in 4096-item tiles of
// 256 threads, or copies 805 MB of float4 (the guide's 6.29 TB/s reference).
//   f4      float4 copy, one vector per lane per iteration, grid-stride
//   s32x4   lane loads u32x4, stores two u64x2 32 B apart (the old shape)
//   c32x2   lane loads u32x2, stores one u64x2: each instruction contiguous
//   c32x4t  lane loads u32x4, transposes through LDS, stores contiguous u64x2
// each with nontemporal (nt) and default-policy stores.
//
// build: hipcc -O3 --offload-arch=gfx950 -o tools/mb/copy_shapes tools/mb/copy_shapes.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

constexpr int TB = 256, IPT = 16, TILE = TB * IPT;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool NT, typename T>
__device__ __forceinline__ void st(T *p, T v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <bool NT>
__global__ __launch_bounds__(TB) void k_f4(const f32x4 *__restrict__ in, f32x4 *__restrict__ out, size_t n) {
    for (size_t i = (size_t)blockIdx.x * TB + threadIdx.x; i < n; i += (size_t)gridDim.x * TB)
        st<NT>(out + i, __builtin_nontemporal_load(in + i));
}

template <bool NT>
__global__ __launch_bounds__(TB) void k_s32x4(const uint32_t *__restrict__ in, uint64_t *__restrict__ out) {
    const size_t t0 = (size_t)blockIdx.x * TILE;
    u32x4 v[IPT / 4];
#pragma unroll
    for (int k = 0; k < IPT / 4; ++k)
        v[k] = __builtin_nontemporal_load((const u32x4 *)(in + t0 + ((size_t)k * TB + threadIdx.x) * 4));
#pragma unroll
    for (int k = 0; k < IPT / 4; ++k) {
        u64x2 *p = (u64x2 *)(out + t0 + ((size_t)k * TB + threadIdx.x) * 4);
        st<NT>(p, (u64x2){v[k].x, v[k].y});
        st<NT>(p + 1, (u64x2){v[k].z, v[k].w});
    }
}

template <bool NT>
__global__ __launch_bounds__(TB) void k_c32x2(const uint32_t *__restrict__ in, uint64_t *__restrict__ out) {
    const size_t t0 = (size_t)blockIdx.x * TILE;
    u32x2 v[IPT / 2];
#pragma unroll
    for (int k = 0; k < IPT / 2; ++k)
        v[k] = __builtin_nontemporal_load((const u32x2 *)(in + t0 + ((size_t)k * TB + threadIdx.x) * 2));
#pragma unroll
    for (int k = 0; k < IPT / 2; ++k)
        st<NT>((u64x2 *)(out + t0 + ((size_t)k * TB + threadIdx.x) * 2), (u64x2){v[k].x, v[k].y});
}

template <bool NT>
__global__ __launch_bounds__(TB) void k_c32x4t(const uint32_t *__restrict__ in, uint64_t *__restrict__ out) {
    __shared__ uint32_t s[TILE];
    const size_t t0 = (size_t)blockIdx.x * TILE;
#pragma unroll
    for (int k = 0; k < IPT / 4; ++k) {
        const int i = (k * TB + threadIdx.x) * 4;
        *(u32x4 *)(s + i) = __builtin_nontemporal_load((const u32x4 *)(in + t0 + i));
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < IPT / 2; ++k) {
        const int i = (k * TB + threadIdx.x) * 2;
        const u32x2 v = *(const u32x2 *)(s + i);
        st<NT>((u64x2 *)(out + t0 + i), (u64x2){v.x, v.y});
    }
}

int main(int argc, char **argv) {
    const uint32_t ntiles = argc > 1 ? (uint32_t)atoi(argv[1]) : 16384;
    const size_t n = (size_t)ntiles * TILE;
    const int reps = 20;
    uint32_t *d_in;
    uint64_t *d_out;
    CK(hipMalloc(&d_in, n * 4));
    CK(hipMalloc(&d_out, n * 8));
    std::vector<uint32_t> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = (uint32_t)(i * 2654435761u);
    CK(hipMemcpy(d_in, h.data(), n * 4, hipMemcpyHostToDevice));
    f32x4 *f_in, *f_out;
    const size_t nf = n * 12 / 2 / 16;          // 805 MB moved: 402.5 MB in, 402.5 MB out
    CK(hipMalloc(&f_in, nf * 16));
    CK(hipMalloc(&f_out, nf * 16));
    CK(hipMemset(f_in, 1, nf * 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<uint64_t> got(n);
    auto timeit = [&](const char *name, auto fn, bool check) {
        CK(hipMemset(d_out, 0, n * 8));
        fn();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) fn();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        size_t bad = 0;
        if (check) {
            CK(hipMemcpy(got.data(), d_out, n * 8, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < n; ++i) bad += got[i] != h[i];
        }
        printf("%-22s %8.1f us  %.2f TB/s%s\n", name, ms * 1e3 / reps, (double)n * 12 / (ms * 1e-3 / reps) / 1e12,
               check ? (bad ? "  WRONG" : "  ok") : "");
    };
    const unsigned fgrid = 256 * 8;
    printf("u32 -> u64 of %zu items (%u tiles of %d), 805 MB per pass, %d reps\n", n, ntiles, TILE, reps);
    timeit("f4 nt", [&] { k_f4<true><<<fgrid, TB>>>(f_in, f_out, nf); }, false);
    timeit("f4", [&] { k_f4<false><<<fgrid, TB>>>(f_in, f_out, nf); }, false);
    timeit("s32x4 nt (old)", [&] { k_s32x4<true><<<ntiles, TB>>>(d_in, d_out); }, true);
    timeit("s32x4", [&] { k_s32x4<false><<<ntiles, TB>>>(d_in, d_out); }, true);
    timeit("c32x2 nt", [&] { k_c32x2<true><<<ntiles, TB>>>(d_in, d_out); }, true);
    timeit("c32x2", [&] { k_c32x2<false><<<ntiles, TB>>>(d_in, d_out); }, true);
    timeit("c32x4t nt", [&] { k_c32x4t<true><<<ntiles, TB>>>(d_in, d_out); }, true);
    timeit("c32x4t", [&] { k_c32x4t<false><<<ntiles, TB>>>(d_in, d_out); }, true);
    CK(hipFree(d_in));
    CK(hipFree(d_out));
    CK(hipFree(f_in));
    CK(hipFree(f_out));
    return 0;
}
