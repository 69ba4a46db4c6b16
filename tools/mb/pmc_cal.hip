// pmc_cal.hip -- known-byte-count kernels for calibrating rocprofv3's
// FETCH_SIZE / WRITE_SIZE on gfx950 per access width (VERDICT r2 item 7;
// MI355X_MICROARCH.md §HBM: only 16 B/lane streaming reads and stores are
// calibrated there).  Every kernel touches a 1 GiB buffer (4x the Infinity
// Cache) exactly once, coalesced: lane i of a wave reads / writes bytes
// [W i, W i + W) of each 64 W-byte block, for W = 1, 2, 4, 8, 16, plus the
// LDS-DMA form (global_load_lds, 16 B/lane) the merge kernels stage with.
// Reads fold into one word per workgroup (sink); writes store a constant.
// Run under rocprofv3 --pmc FETCH_SIZE and, separately, --pmc WRITE_SIZE;
// tools/pmc_cal.py turns the counters into bytes-per-counted-byte factors.
// Build: hipcc -O3 --offload-arch=gfx950 -o pmc_cal pmc_cal.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int W> struct Vec;
template <> struct Vec<1> { using T = uint8_t; };
template <> struct Vec<2> { using T = uint16_t; };
template <> struct Vec<4> { using T = uint32_t; };
template <> struct Vec<8> { using T = uint64_t; };
template <> struct Vec<16> { using T = uint4; };

__device__ __forceinline__ uint32_t fold(uint8_t x) { return x; }
__device__ __forceinline__ uint32_t fold(uint16_t x) { return x; }
__device__ __forceinline__ uint32_t fold(uint32_t x) { return x; }
__device__ __forceinline__ uint32_t fold(uint64_t x) { return (uint32_t)x ^ (uint32_t)(x >> 32); }
__device__ __forceinline__ uint32_t fold(uint4 x) { return x.x ^ x.y ^ x.z ^ x.w; }

template <int W>
__global__ __launch_bounds__(256) void read_w(const void *__restrict__ src, size_t bytes, uint32_t *__restrict__ sink) {
    using T = typename Vec<W>::T;
    const T *p = (const T *)src;
    const size_t n = bytes / W;
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= fold(p[i]);
    for (int o = 32; o >= 1; o >>= 1) acc ^= __shfl_xor(acc, o);
    if (threadIdx.x == 0) sink[blockIdx.x] = acc;
}

template <int W>
__global__ __launch_bounds__(256) void write_w(void *__restrict__ dst, size_t bytes) {
    using T = typename Vec<W>::T;
    T *p = (T *)dst;
    const size_t n = bytes / W;
    T v;
    memset(&v, 0x5A, sizeof v);
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = v;
}

// LDS-DMA: each wave moves 1 KiB per instruction into its own LDS slot
__global__ __launch_bounds__(256) void read_lds_dma(const void *__restrict__ src, size_t bytes, uint32_t *__restrict__ sink) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 1024];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const char *g = (const char *)src;
    for (size_t off = ((size_t)blockIdx.x * 4 + w) * 1024; off < bytes; off += (size_t)gridDim.x * 4 * 1024)
        __builtin_amdgcn_global_load_lds((const void *)(g + off + 16 * lane),
                                         (__attribute__((address_space(3))) void *)(lds + w * 1024), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) sink[blockIdx.x] = lds[7];
}

int main() {
    const size_t bytes = (size_t)1 << 30;
    void *buf = nullptr;
    uint32_t *sink = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 1 << 20) != hipSuccess) return 1;
    hipDeviceProp_t pr;
    (void)hipGetDeviceProperties(&pr, 0);
    const unsigned g = (unsigned)pr.multiProcessorCount * 8;
    (void)hipMemset(buf, 1, bytes);
    for (int rep = 0; rep < 2; ++rep) {
        read_w<1><<<g, 256>>>(buf, bytes, sink);
        read_w<2><<<g, 256>>>(buf, bytes, sink);
        read_w<4><<<g, 256>>>(buf, bytes, sink);
        read_w<8><<<g, 256>>>(buf, bytes, sink);
        read_w<16><<<g, 256>>>(buf, bytes, sink);
        read_lds_dma<<<g, 256>>>(buf, bytes, sink);
        write_w<1><<<g, 256>>>(buf, bytes);
        write_w<2><<<g, 256>>>(buf, bytes);
        write_w<4><<<g, 256>>>(buf, bytes);
        write_w<8><<<g, 256>>>(buf, bytes);
        write_w<16><<<g, 256>>>(buf, bytes);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"bytes_per_kernel\": %zu}\n", bytes);
    (void)hipFree(buf);
    (void)hipFree(sink);
    return 0;
}
