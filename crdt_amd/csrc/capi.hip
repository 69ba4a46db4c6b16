// capi.hip -- context lifecycle, memory helpers, options, small host-side
// entry points of the C-ABI (include/crdt_amd.h).
#include <string.h>

#include <algorithm>
#include <atomic>
#include <new>

#include "common.hpp"

namespace crdt {
JoinTuning g_join;
FoldTuning g_fold;
int g_vclock_pairs_per_wave = 32;  // 10M x 128, one block/CU: 32 pairs 0.858-0.860 of 8 TB/s, 16 0.852-0.854,
int g_vclock_blocks_per_cu = 1;    //   8 0.833 (profiles/r05/ab/vclock_*.txt; 4 x 8 blocks/CU: 6.19 TB/s)
int g_lww_chunk = 0;      // LWW tiles per chunk, 0 = one chunk (chunked schedules measured slower: DESIGN.md §5.4)
int g_or_chunk = 0;       // OR-Set tiles per chunk (likewise)
int g_set_streams = 1;
int g_shard_exchange_always = 0;
int g_or_count_dma = 1;  // OR-Set count pass staged by LDS-DMA (sets.or_count_dma)
int g_or_key_sort = 2;   // OR-Set D2: 2 key + one more tag digit, marks within groups; 1 key only; 0 the 7-pass tag sort
int g_or_parts = 2;     // OR-Set write pass: half tiles (whole tiles 159 -> 152 us)
int g_rm_parts = 1;
int g_rm_count_dma = 1;
int g_short_tab = 3;
int g_dec_big_r = 4;
int g_dec_small = 1;
int g_rm_kvx = 0;
int g_rm_ld_all = 0;
int g_sort_xcd = 1;      // radix scatter: XCD-contiguous tiles
int g_sort_vec_up = 1;   // fused D2: vectorised composing upsweep
int g_lww_table = 1;     // LWW D2: key-bucket LDS tables when the key offsets span 12..23 bits
int g_sample_plan = 1;   // dense-key D2 paths from a sampled plan, checked in the upsweep (sort.sample_plan)
int g_plan_cache = 2;    // ... launched from the last such plan (2: as it is, no sample; 1: its shape, a fresh sample checked on the device) (sort.plan_cache)
int g_rm_affine = 1;     // one-pair populations: RefMerge pair indices computed, no kv range loads (refmerge.affine_kv)
int g_lww_gather = 1;    // LWW D2 tables gather their runs from bucket-grouped tiles, no scatter pass (sort.lww_gather)
int g_or_narrow = 1;
int g_pop_direct = 1;    // population rounds: staging kernel + polled host bounds, no copy engine (pop.direct)
int g_or_place_batch = 1;  // OR-Set D2 buckets: placement sorted per round in LDS, stored in pieces (sort.or_place_batch)
int g_up_threads = 512;  // D2 tile grouping pass: threads per 4096-tuple tile, 256 or 512 (sort.up_threads)
int g_group_tile = 8192;  // D2 gather forms: tuples per grouping tile, 4096 or 8192 (sort.group_tile)
int g_or_sub_hist = 1;   // OR-Set D2 buckets: chunk counts from per-run histograms (sort.or_sub_hist)
int g_read_poll = 1;     // small read-backs polled from coherent host memory (ctx.read_poll)
int g_pop_wire_early = 1;  // wire rounds: the merge enqueued behind the decode's claim pass (pop.wire_early)
int g_or_lb_words = 1;   // OR-Set D2 chunk look-back: status words per lane per window, 1 or 4 (sort.or_lb_words)
int g_or_bucket = 1;     // OR-Set D2: top-byte tile groups gathered into chunks, no radix passes (sort.or_bucket)
int g_or_pair = 1;       // OR-Set D2 chunks: two per workgroup, one look-back for both (sort.or_pair)     // OR-Set D2 chunks: keys' slots sorted on their low words when the tags fit 32 bits (sort.or_narrow)
int g_sample_min = 1 << 20;   // ... for calls of at least this many tuples (sort.sample_min)
int g_or_lookback = 1;   // OR-Set D2 chunks: offsets by a decoupled look-back (0: count scan + emit pass)
int g_or_table = 1;      // OR-Set D2: 2^9-key chunks sorted in LDS after two top-16-bit passes (16..25 key bits)
int g_rdd_diag = 0;
int g_mm_bpc = 1;        // sort minmax: workgroups per CU per input (1: 0.716 ms LWW D2 step, 4: 0.732)
int g_lww_parts = 4;     // LWW write pass: quarter tiles (half tiles 112 -> 105 us)
int g_rm_diag = 0;
int g_scan_items = 8;
std::atomic<int> g_fail_refmerge{0};
std::atomic<int> g_fail_zero_bits{0};

bool take_fail_zero_bits() {
    for (int f = g_fail_zero_bits.load(); f > 0;)
        if (g_fail_zero_bits.compare_exchange_weak(f, f - 1)) return true;
    return false;
}

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
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int ctx_read_words(crdt_ctx *ctx, const void *dev_src, size_t bytes, const void **host) {
    if (bytes > kCioBytes || (bytes & 3)) return CRDT_E_INVAL;
    if (!g_read_poll) {
        int rc = hio_reserve(ctx, bytes ? bytes : 4);
        if (rc) return rc;
        hipError_t e = bytes ? hipMemcpyAsync(ctx->hio, dev_src, bytes, hipMemcpyDeviceToHost, ctx->stream)
                             : hipSuccess;
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e);
        *host = ctx->hio;
        return CRDT_OK;
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
    int rc = check_launch(ctx);
    if (rc) return rc;
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
    uint32_t v = 0;
    hipError_t e = hipMemcpyAsync(&v, ctx->dev_status, sizeof(v), hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess && clear && v) e = hipMemsetAsync(ctx->dev_status, 0, sizeof(v), ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
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

extern "C" int crdt_set_option(const char *name, int64_t v) {
    if (!name) return CRDT_E_INVAL;
    if (!strcmp(name, "join.unroll")) {
        if (v != 1 && v != 2 && v != 4 && v != 8) return CRDT_E_INVAL;
        g_join.unroll = (int)v;
    } else if (!strcmp(name, "join.nontemporal")) {
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_join.nontemporal = (int)v;
    } else if (!strcmp(name, "join.blocks_per_cu")) {
        if (v < 1 || v > 64) return CRDT_E_INVAL;
        g_join.blocks_per_cu = (int)v;
    } else if (!strcmp(name, "fold.unroll")) {
        if (v != 1 && v != 2 && v != 4 && v != 8 && v != 16 && v != 32) return CRDT_E_INVAL;
        g_fold.unroll = (int)v;
    } else if (!strcmp(name, "fold.nontemporal")) {
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_fold.nontemporal = (int)v;
    } else if (!strcmp(name, "fold.blocks_per_cu")) {
        if (v < 1 || v > 64) return CRDT_E_INVAL;
        g_fold.blocks_per_cu = (int)v;
    } else if (!strcmp(name, "vclock.pairs_per_wave")) {
        if (v != 1 && v != 2 && v != 4 && v != 8 && v != 16 && v != 32) return CRDT_E_INVAL;
        g_vclock_pairs_per_wave = (int)v;
    } else if (!strcmp(name, "vclock.blocks_per_cu")) {
        if (v < 1 || v > 64) return CRDT_E_INVAL;
        g_vclock_blocks_per_cu = (int)v;
    } else if (!strcmp(name, "sets.lww_chunk")) {    // LWW tiles per count / write chunk (0: one chunk)
        if (v < 0 || v > 16384) return CRDT_E_INVAL;
        g_lww_chunk = (int)v;
    } else if (!strcmp(name, "sets.or_chunk")) {     // OR-Set tiles per count / write chunk (0: one chunk)
        if (v < 0 || v > 16384) return CRDT_E_INVAL;
        g_or_chunk = (int)v;
    } else if (!strcmp(name, "sets.streams")) {      // 1: one stream; 2: chunk c+1's count beside chunk c's write
        if (v != 1 && v != 2) return CRDT_E_INVAL;
        g_set_streams = (int)v;
    } else if (!strcmp(name, "shard.exchange_always")) {   // tests: the keyed-set exchange protocol even on 1 rank
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_shard_exchange_always = (int)v;
    } else if (!strcmp(name, "sets.or_count_dma")) { // OR-Set count pass: 1 LDS-DMA staging, 0 register staging
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_or_count_dma = (int)v;
    } else if (!strcmp(name, "sort.or_key_only")) {  // OR-Set D2: 2 key + 1-2 tag digits, 1 key-only sort, 0 full tag sort
        if (v < 0 || v > 2) return CRDT_E_INVAL;
        g_or_key_sort = (int)v;
    } else if (!strcmp(name, "sort.xcd_tiles")) {    // radix scatter pass: 1 XCD-contiguous tile ranges, 0 blockIdx order
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_sort_xcd = (int)v;
    } else if (!strcmp(name, "sort.mm_blocks_per_cu")) {   // sort minmax grid: workgroups per CU per input
        if (v < 1 || v > 16) return CRDT_E_INVAL;
        g_mm_bpc = (int)v;
    } else if (!strcmp(name, "sort.rdd_diag")) {     // timing diagnostic: the D2 dedup apply (OR-Set: and count)
        if (v < 0 || v > 8) return CRDT_E_INVAL;       //   stops after 1 staging, 2 marks, 3 counts (no stores);
                                                        //   OR-Set chunks: 1 key counts, 2 LDS sort, 3 per-key tags, 4 long keys + ranks,
                                                        //   5 all but the output stores, 6 no look-back (fake offsets);
                                                        //   OR-Set buckets: 7 no placement stores, 8 no placement sweep
        g_rdd_diag = (int)v;
    } else if (!strcmp(name, "sort.lww_table")) {    // LWW D2: 1 key-bucket LDS tables where they apply, 0 key-only sort
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_lww_table = (int)v;
    } else if (!strcmp(name, "sort.or_table")) {     // OR-Set D2: 1 key chunks sorted in LDS where they apply, 0 the radix sort
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_or_table = (int)v;
    } else if (!strcmp(name, "sort.sample_plan")) {  // D2 dense-key paths: 1 plan from a sample + range check, 0 full minmax
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_sample_plan = (int)v;
    } else if (!strcmp(name, "refmerge.affine_kv")) { // one-pair populations: 1 pair index = kv[0] + entry (no range loads)
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_rm_affine = (int)v;
    } else if (!strcmp(name, "sort.lww_gather")) {   // LWW D2 tables: 1 runs gathered from bucket-grouped tiles, 0 a scatter pass
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_lww_gather = (int)v;
    } else if (!strcmp(name, "sort.or_bucket")) {    // OR-Set D2: 1 tile groups + bucket gathers, 0 two radix passes
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_or_bucket = (int)v;
    } else if (!strcmp(name, "pop.direct")) {        // population rounds: 1 staging kernel + polled host bounds, 0 copies + sync
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_pop_direct = (int)v;
    } else if (!strcmp(name, "sort.or_place_batch")) {   // OR-Set D2 buckets: 1 placement batched in LDS, 0 one by one
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_or_place_batch = (int)v;
    } else if (!strcmp(name, "sort.up_threads")) {   // D2 tile grouping pass: 256 / 512 threads per 4096-tuple tile
        if (v != 256 && v != 512) return CRDT_E_INVAL;
        g_up_threads = (int)v;
    } else if (!strcmp(name, "sort.group_tile")) {   // D2 gather forms: 4096 / 8192 tuples per grouping tile
        if (v != 4096 && v != 8192) return CRDT_E_INVAL;
        g_group_tile = (int)v;
    } else if (!strcmp(name, "sort.or_sub_hist")) {  // OR-Set D2 buckets: 1 chunk counts from per-run rows, 0 a counting gather
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_or_sub_hist = (int)v;
    } else if (!strcmp(name, "ctx.read_poll")) {     // small read-backs: 1 kernel + polled coherent memory, 0 copy + sync
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_read_poll = (int)v;
    } else if (!strcmp(name, "pop.wire_early")) {    // wire rounds: 1 merge enqueued behind the claim pass, 0 after the decode
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_pop_wire_early = (int)v;
    } else if (!strcmp(name, "sort.or_lb_words")) {  // OR-Set D2 chunk look-back: 1 / 4 status words per lane per window
        if (v != 1 && v != 4) return CRDT_E_INVAL;
        g_or_lb_words = (int)v;
    } else if (!strcmp(name, "sort.or_pair")) {      // OR-Set D2 chunks: 1 two per workgroup (one look-back), 0 one
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_or_pair = (int)v;
    } else if (!strcmp(name, "sort.or_narrow")) {    // OR-Set D2 chunks: 1 u32 sorting networks where the tag fits 32 bits
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_or_narrow = (int)v;
    } else if (!strcmp(name, "sort.plan_cache")) {   // D2 sampled plans: 2 the cached plan (no sample), 1 its shape + a sample, 0 none
        if (v < 0 || v > 2) return CRDT_E_INVAL;
        g_plan_cache = (int)v;
    } else if (!strcmp(name, "sort.sample_min")) {   // fewest tuples for the sampled plan
        if (v < 0 || v > 0x7FFFFFFF) return CRDT_E_INVAL;
        g_sample_min = (int)v;
    } else if (!strcmp(name, "sort.or_lookback")) {  // OR-Set D2 chunks: 1 look-back offsets + direct stores, 0 scan + emit
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_or_lookback = (int)v;
    } else if (!strcmp(name, "sort.vec_up")) {       // fused D2 sort: 1 vectorised composing upsweep, 0 scalar
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_sort_vec_up = (int)v;
    } else if (!strcmp(name, "sets.lww_parts")) {    // LWW write-pass workgroups per 4096-item tile
        if (v != 2 && v != 4 && v != 8 && v != 16) return CRDT_E_INVAL;
        g_lww_parts = (int)v;
    } else if (!strcmp(name, "sets.or_parts")) {     // OR-Set write-pass workgroups per 2048-item tile
        if (v != 1 && v != 2 && v != 4) return CRDT_E_INVAL;
        g_or_parts = (int)v;
    } else if (!strcmp(name, "refmerge.load_all")) {   // tile pass loads non-emitted entries too (A/B)
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_rm_ld_all = (int)v;
    } else if (!strcmp(name, "refmerge.kv_one_launch")) {   // kv tile pass: both tile kinds in one launch at any grid
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_rm_kvx = (int)v;
    } else if (!strcmp(name, "codec.short_tab")) {   // string-table lookups: the short form beside the entry (2: + both home probes first)
        if (v < 0 || v > 4) return CRDT_E_INVAL;
        g_short_tab = (int)v;
    } else if (!strcmp(name, "codec.big_r")) {   // the coalesced one-pass decode: items per thread per chunk
        if (v != 4 && v != 8) return CRDT_E_INVAL;
        g_dec_big_r = (int)v;
    } else if (!strcmp(name, "codec.small")) {   // gossip decode in one pass: 0 off, 1 auto, 2 always, 3 always (coalesced form)
        if (v < 0 || v > 3) return CRDT_E_INVAL;
        g_dec_small = (int)v;
    } else if (!strcmp(name, "refmerge.count_dma")) {   // RefMerge count pass: ts runs staged by LDS-DMA
        if (v != 0 && v != 1) return CRDT_E_INVAL;
        g_rm_count_dma = (int)v;
    } else if (!strcmp(name, "refmerge.tile_parts")) {   // RefMerge tile-pass workgroups per 4096-item tile
        if (v != 1 && v != 2 && v != 4) return CRDT_E_INVAL;
        g_rm_parts = (int)v;
    } else if (!strcmp(name, "refmerge.diag_fold")) {   // timing diagnostic: 1 skip the replay fold; 2 no flush, 4 no table, 5 no Atoi gather
        if (v < 0 || v > 5) return CRDT_E_INVAL;
        g_rm_diag = (int)v;
    } else if (!strcmp(name, "scan.items")) {        // items per lane of the single-pass scan
        if (v != 4 && v != 8 && v != 16) return CRDT_E_INVAL;
        g_scan_items = (int)v;
    } else if (!strcmp(name, "fail.refmerge")) {     // fault injection: the next v RefMerge calls fail (CRDT_E_NOMEM)
        if (v < 0 || v > 1000) return CRDT_E_INVAL;
        g_fail_refmerge = (int)v;
    } else if (!strcmp(name, "fail.zero_bits")) {    // fault injection: the next v two-pass merges zero their
        if (v < 0 || v > 1000) return CRDT_E_INVAL;    //   merge bitmaps between the passes (CRDT_DEV_RANGE)
        g_fail_zero_bits = (int)v;
    } else {
        return CRDT_E_INVAL;
    }
    return CRDT_OK;
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
