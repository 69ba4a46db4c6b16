// capi.hip -- context lifecycle, memory helpers, options, small host-side
// entry points of the C-ABI (include/crdt_amd.h).
#include <string.h>

#include <algorithm>
#include <atomic>
#include <new>

#include "common.hpp"

namespace crdt {
#ifdef CRDT_DIAG
#define KNOB(var, def, name, valid) int var = (def);
#include "knobs.inc"
#undef KNOB
std::atomic<int> g_fail_refmerge{0};
std::atomic<int> g_fail_zero_bits{0};
std::atomic<int> g_fail_d2_plan{0};

static bool take_count(std::atomic<int> &c) {
    for (int f = c.load(); f > 0;)
        if (c.compare_exchange_weak(f, f - 1)) return true;
    return false;
}
bool take_fail_zero_bits() { return take_count(g_fail_zero_bits); }
bool take_fail_refmerge() { return take_count(g_fail_refmerge); }
bool take_fail_d2_plan() { return take_count(g_fail_d2_plan); }
#endif

int ws_reserve(crdt_ctx *ctx, size_t bytes) {
    if (bytes <= ctx->ws_bytes) return CRDT_OK;
    size_t want = bytes + bytes / 4;                  // grow with headroom
    want = (want + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
    hipError_t e;
    if (ctx->ws) {
        e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e);
        e = hipFree(ctx->ws);
        ctx->ws = nullptr;
        ctx->ws_bytes = 0;
        if (e != hipSuccess) return hip_fail(ctx, e);
    }
    e = hipMalloc(&ctx->ws, want);
    if (e != hipSuccess) {
        ctx->ws = nullptr;
        return hip_fail(ctx, e);
    }
    ctx->ws_bytes = want;
    return CRDT_OK;
}

int ctx_aux(crdt_ctx *ctx) {
    if (ctx->aux) return CRDT_OK;
    hipError_t e = hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking);
    if (e != hipSuccess) {
        ctx->aux = nullptr;
        return hip_fail(ctx, e);
    }
    return CRDT_OK;
}

int ctx_events(crdt_ctx *ctx, size_t n) {
    if (n <= ctx->n_ev) return CRDT_OK;
    const size_t want = std::max<size_t>(n, 2 * ctx->n_ev);
    hipEvent_t *ev = new (std::nothrow) hipEvent_t[want];
    if (!ev) return CRDT_E_NOMEM;
    for (size_t i = 0; i < ctx->n_ev; ++i) ev[i] = ctx->ev[i];
    for (size_t i = ctx->n_ev; i < want; ++i) {
        hipError_t e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
        if (e != hipSuccess) {
            for (size_t j = ctx->n_ev; j < i; ++j) (void)hipEventDestroy(ev[j]);
            delete[] ev;
            return hip_fail(ctx, e);
        }
    }
    delete[] ctx->ev;                    // (events already handed to pending waits stay alive)
    ctx->ev = ev;
    ctx->n_ev = want;
    return CRDT_OK;
}
}  // namespace crdt

using namespace crdt;

extern "C" int crdt_abi_version(void) { return CRDT_AMD_ABI_VERSION; }

extern "C" const char *crdt_status_str(int s) {
    switch (s) {
        case CRDT_OK: return "ok";
        case CRDT_E_INVAL: return "invalid argument";
        case CRDT_E_HIP: return "HIP runtime error";
        case CRDT_E_NOMEM: return "device out of memory";
        case CRDT_E_NODEV: return "no gfx950 device";
        case CRDT_E_UNSORTED: return "input not sorted";
        case CRDT_E_RANGE: return "size exceeds kernel index range";
        case CRDT_E_COMM: return "RCCL error";
        case CRDT_E_DEVICE: return "device-side failure flag raised (output invalid)";
        default: return "unknown status";
    }
}

extern "C" int crdt_device_count(int *count) {
    if (!count) return CRDT_E_INVAL;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) { *count = 0; return CRDT_E_NODEV; }
    *count = n;
    return CRDT_OK;
}

extern "C" int crdt_ctx_create(int device, void *stream, crdt_ctx **out) {
    if (!out) return CRDT_E_INVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return CRDT_E_NODEV;
    if (device < 0 || device >= n) return CRDT_E_INVAL;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return CRDT_E_NODEV;
    // gfx950 only: the kernels are compiled for nothing else.
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return CRDT_E_NODEV;
    crdt_ctx *ctx = new (std::nothrow) crdt_ctx();
    if (!ctx) return CRDT_E_NOMEM;
    ctx->device = device;
    ctx->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (cur != device) (void)hipSetDevice(device);
    // NULL is the device's default (null) stream -- what torch's default
    // current stream reports as cuda_stream == 0 -- never a private stream:
    // work must stay ordered with the caller's copies on that stream.
    ctx->stream = (hipStream_t)stream;
    hipError_t e = hipMalloc((void **)&ctx->dev_status, 256);
    if (e == hipSuccess) e = hipMemset(ctx->dev_status, 0, 256);
    if (e != hipSuccess) {
        if (ctx->dev_status) (void)hipFree(ctx->dev_status);
    server_ctx_release(ctx);
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    if (ctx->hio) (void)hipHostFree(ctx->hio);
    (void)crdt_strtab_destroy(ctx->keys);
    (void)crdt_strtab_destroy(ctx->vals);
        delete ctx;
        return e == hipErrorOutOfMemory ? CRDT_E_NOMEM : CRDT_E_HIP;
    }
    *out = ctx;
    return CRDT_OK;
}

extern "C" int crdt_stream_create(int device, void **stream) {
    if (!stream) return CRDT_E_INVAL;
    *stream = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return CRDT_E_NODEV;
    if (device < 0 || device >= n) return CRDT_E_INVAL;
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (cur != device) (void)hipSetDevice(device);
    hipStream_t s = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (cur != device && cur >= 0) (void)hipSetDevice(cur);
    if (e != hipSuccess) return e == hipErrorOutOfMemory ? CRDT_E_NOMEM : CRDT_E_HIP;
    *stream = (void *)s;
    return CRDT_OK;
}

extern "C" int crdt_stream_destroy(void *stream) {
    if (!stream) return CRDT_OK;
    hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamDestroy((hipStream_t)stream);
    return e == hipSuccess ? CRDT_OK : CRDT_E_HIP;
}

namespace crdt {
__global__ __launch_bounds__(256) void k_read_words(const uint32_t *__restrict__ src, uint32_t n,
                                                    uint32_t *__restrict__ dst, uint64_t *__restrict__ flag,
                                                    uint64_t seq) {
    for (uint32_t i = threadIdx.x; i < n; i += 256) dst[i] = src[i];
    __threadfence_system();                    // each wave's stores, before the flag
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int ctx_read_begin(crdt_ctx *ctx, const void *dev_src, size_t bytes) {
    if (bytes > kCioBytes || (bytes & 3)) return CRDT_E_INVAL;
    if (!g_read_poll) {
        int rc = hio_reserve(ctx, bytes ? bytes : 4);
        if (rc) return rc;
        hipError_t e = bytes ? hipMemcpyAsync(ctx->hio, dev_src, bytes, hipMemcpyDeviceToHost, ctx->stream)
                             : hipSuccess;
        return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
    }
    if (!ctx->cio) {                                  // words | completion word (64 B after them)
        void *h = nullptr, *d = nullptr;
        hipError_t e = hipHostMalloc(&h, kCioBytes + 64, hipHostMallocCoherent | hipHostMallocMapped);
        if (e == hipSuccess) e = hipHostGetDevicePointer(&d, h, 0);
        if (e != hipSuccess) {
            if (h) (void)hipHostFree(h);
            return hip_fail(ctx, e);
        }
        ctx->cio = h;
        ctx->cio_d = d;
        *(volatile uint64_t *)((char *)h + kCioBytes) = 0;
        ctx->cio_seq = 0;
    }
    const uint64_t seq = ++ctx->cio_seq;
    k_read_words<<<1, 256, 0, ctx->stream>>>((const uint32_t *)dev_src, (uint32_t)(bytes / 4),
                                              (uint32_t *)ctx->cio_d, (uint64_t *)((char *)ctx->cio_d + kCioBytes),
                                              seq);
    return check_launch(ctx);
}

int ctx_read_end(crdt_ctx *ctx, const void **host) {
    if (!g_read_poll) {
        hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e);
        *host = ctx->hio;
        return CRDT_OK;
    }
    const uint64_t seq = ctx->cio_seq;
    const volatile uint64_t *f = (const volatile uint64_t *)((char *)ctx->cio + kCioBytes);
    while (*f != seq) {
        const hipError_t q = hipStreamQuery(ctx->stream);
        if (q == hipErrorNotReady) continue;
        if (*f == seq) break;
        return hip_fail(ctx, q == hipSuccess ? hipErrorUnknown : q);
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    *host = ctx->cio;
    return CRDT_OK;
}

int ctx_read_words(crdt_ctx *ctx, const void *dev_src, size_t bytes, const void **host) {
    int rc = ctx_read_begin(ctx, dev_src, bytes);
    return rc ? rc : ctx_read_end(ctx, host);
}
}  // namespace crdt

extern "C" int crdt_ctx_destroy(crdt_ctx *ctx) {
    if (!ctx) return CRDT_OK;
    (void)bind(ctx);
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->cio) (void)hipHostFree(ctx->cio);
    if (ctx->ws) (void)hipFree(ctx->ws);
    if (ctx->io) (void)hipFree(ctx->io);
    if (ctx->dev_status) (void)hipFree(ctx->dev_status);
    server_ctx_release(ctx);
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    if (ctx->hio) (void)hipHostFree(ctx->hio);
    (void)crdt_strtab_destroy(ctx->keys);
    (void)crdt_strtab_destroy(ctx->vals);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->aux) {
        (void)hipStreamSynchronize(ctx->aux);
        (void)hipStreamDestroy(ctx->aux);
    }
    for (size_t i = 0; i < ctx->n_ev; ++i) (void)hipEventDestroy(ctx->ev[i]);
    delete[] ctx->ev;
    delete ctx;
    return CRDT_OK;
}

extern "C" int crdt_ctx_set_stream(crdt_ctx *ctx, void *stream) {
    int rc = bind(ctx);
    if (rc) return rc;
    hipStream_t ns = (hipStream_t)stream;
    if (ns == ctx->stream) return CRDT_OK;
    // The workspace, staging buffer and status word are shared by every call
    // of the context: work still queued on the old stream must finish before
    // the new stream reuses (or ws_reserve frees) them.  The new stream waits
    // on an event recorded behind the old stream's work (no host sync).
    hipEvent_t ev = nullptr;
    hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(ev, ctx->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(ns, ev, 0);
    if (ev) (void)hipEventDestroy(ev);
    if (e != hipSuccess) return hip_fail(ctx, e);
    if (ctx->own_stream) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipStreamDestroy(ctx->stream);
        ctx->own_stream = false;
    }
    ctx->stream = ns;
    return CRDT_OK;
}

extern "C" int crdt_ctx_device_status(crdt_ctx *ctx, uint32_t *flags, int clear) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!flags) return CRDT_E_INVAL;
    const void *hw = nullptr;                         // (stream-ordered: every earlier pass has finished)
    rc = ctx_read_words(ctx, ctx->dev_status, sizeof(uint32_t), &hw);
    if (rc) return rc;
    const uint32_t v = *(const uint32_t *)hw;
    if (clear && v) {
        hipError_t e = hipMemsetAsync(ctx->dev_status, 0, sizeof(v), ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e);
    }
    *flags = v;
    return CRDT_OK;
}

extern "C" int crdt_ctx_sync(crdt_ctx *ctx) {
    int rc = bind(ctx);
    if (rc) return rc;
    hipError_t e = hipStreamSynchronize(ctx->stream);
    return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
}

extern "C" int crdt_ctx_last_hip_error(const crdt_ctx *ctx) { return ctx ? ctx->last_hip_error : 0; }

extern "C" int crdt_ctx_reserve(crdt_ctx *ctx, size_t bytes) {
    int rc = bind(ctx);
    if (rc) return rc;
    return ws_reserve(ctx, bytes);
}

// The knob table (knobs.inc): name, current value, validity of a new value.
struct KnobEntry {
    const char *name;
    int64_t (*get)();
    int (*set)(int64_t v);   // CRDT_E_INVAL when invalid (or in the product build)
};
#ifdef CRDT_DIAG
#define KNOB(var, def, kname, valid) \
    {kname, [] { return (int64_t)var; }, [](int64_t v) { if (!(valid)) return (int)CRDT_E_INVAL; var = (int)v; return (int)CRDT_OK; }},
#else
#define KNOB(var, def, kname, valid) \
    {kname, [] { return (int64_t)var; }, [](int64_t) { return (int)CRDT_E_INVAL; }},
#endif
static const KnobEntry kKnobs[] = {
#include "knobs.inc"
};
#undef KNOB

extern "C" int crdt_get_option(const char *name, int64_t *v) {
    if (!name || !v) return CRDT_E_INVAL;
    if (!strcmp(name, "build.diag")) {
#ifdef CRDT_DIAG
        *v = 1;
#else
        *v = 0;
#endif
        return CRDT_OK;
    }
    for (const KnobEntry &k : kKnobs)
        if (!strcmp(name, k.name)) {
            *v = k.get();
            return CRDT_OK;
        }
    return CRDT_E_INVAL;
}

// Product build: every name is refused (the knobs are compile-time constants).
// Diagnostic build: the knobs, validated, and the failpoints.
extern "C" int crdt_set_option(const char *name, int64_t v) {
    if (!name) return CRDT_E_INVAL;
#ifdef CRDT_DIAG
    std::atomic<int> *fp = !strcmp(name, "fail.refmerge")    ? &g_fail_refmerge
                           : !strcmp(name, "fail.zero_bits") ? &g_fail_zero_bits
                           : !strcmp(name, "fail.d2_plan")   ? &g_fail_d2_plan
                                                             : nullptr;
    if (fp) {
        if (v < 0 || v > 1000) return CRDT_E_INVAL;
        *fp = (int)v;
        return CRDT_OK;
    }
#endif
    for (const KnobEntry &k : kKnobs)
        if (!strcmp(name, k.name)) return k.set(v);
    return CRDT_E_INVAL;
}

extern "C" int crdt_dev_alloc(crdt_ctx *ctx, size_t bytes, void **dev) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!dev) return CRDT_E_INVAL;
    *dev = nullptr;
    if (bytes == 0) return CRDT_OK;
    hipError_t e = hipMalloc(dev, bytes);
    return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
}

extern "C" int crdt_dev_free(crdt_ctx *ctx, void *dev) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!dev) return CRDT_OK;
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess) e = hipFree(dev);
    return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
}

extern "C" int crdt_memcpy_h2d(crdt_ctx *ctx, void *dst, const void *src, size_t bytes) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (bytes == 0) return CRDT_OK;
    if (!dst || !src) return CRDT_E_INVAL;
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream);
    return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
}

extern "C" int crdt_memcpy_d2h(crdt_ctx *ctx, void *dst, const void *src, size_t bytes) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (bytes == 0) return CRDT_OK;
    if (!dst || !src) return CRDT_E_INVAL;
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);   // host buffer valid on return
    return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
}

extern "C" int crdt_memset(crdt_ctx *ctx, void *dst, int byte, size_t bytes) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (bytes == 0) return CRDT_OK;
    if (!dst) return CRDT_E_INVAL;
    hipError_t e = hipMemsetAsync(dst, byte, bytes, ctx->stream);
    return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
}

// utils.Int64Comparator (gods v1.18.1; main.go:106-107): signed order.
extern "C" int crdt_compare_int64(int64_t a, int64_t b) { return a < b ? -1 : (a > b ? 1 : 0); }

extern "C" int crdt_shard_range(uint64_t rows, int world, int rank, uint64_t *begin, uint64_t *end) {
    if (world <= 0 || rank < 0 || rank >= world || !begin || !end) return CRDT_E_INVAL;
    // Balanced contiguous split: the first (rows % world) ranks take one extra row.
    const uint64_t q = rows / (uint64_t)world, r = rows % (uint64_t)world;
    const uint64_t k = (uint64_t)rank;
    *begin = k * q + (k < r ? k : r);
    *end = *begin + q + (k < r ? 1 : 0);
    return CRDT_OK;
}
