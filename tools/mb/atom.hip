// micro-benchmark: throughput of device-scope atomicAdd-with-return spread over many addresses
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(1024) void k_atom(unsigned *cnt, unsigned nb, unsigned *sink) {
    unsigned acc = 0;
    for (unsigned b = threadIdx.x; b < nb; b += 1024) acc += atomicAdd(&cnt[(b * 2654435761u + blockIdx.x * 977u) % nb], 3u);
    if (acc == 0xFFFFFFFF) sink[0] = acc;
}
int main() {
    unsigned *cnt, *sink;
    hipMalloc(&cnt, 65536 * 4); hipMalloc(&sink, 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    int nbs[] = {4096, 16384, 65536};
    int grids[] = {306, 1221, 4883};
    for (int nb : nbs) for (int g : grids) {
        hipMemset(cnt, 0, 65536 * 4);
        k_atom<<<g, 1024>>>(cnt, nb, sink);
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) k_atom<<<g, 1024>>>(cnt, nb, sink);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
        printf("bins %6d grid %5d atomics %9.0f  %8.1f us  %.2f G atom/s\n", nb, g, (double)nb * g, ms * 1e3, (double)nb * g / (ms * 1e-3) / 1e9);
    }
    return 0;
}
