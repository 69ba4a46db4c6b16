// common.hpp -- shared internals of libcrdt_amd (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <stddef.h>
#include <stdint.h>
#include <functional>
#include <vector>

#include "../../include/crdt_amd.h"

struct crdt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int num_cus = 256;
    int last_hip_error = 0;
    void *ws = nullptr;      // device workspace, grown on demand (crdt_ctx_reserve)
    size_t ws_bytes = 0;
    void *io = nullptr;      // device staging for host-facing calls (crdt_server_*)
    size_t io_bytes = 0;
    uint32_t *dev_status = nullptr;   // device-side failure flags (CRDT_DEV_*), read by crdt_ctx_device_status
    bool rm_nt = true;                // RefMerge kv tile passes with nontemporal hints (cleared around the
                                      // wire round's merge, whose R side the device decode has just written)
    crdt_strtab *keys = nullptr;      // device string tables of the context's Servers (key ids, value ids)
    crdt_strtab *vals = nullptr;
    void *srv_batch = nullptr;        // batched Server merge scratch (server.hip)
    void *pinned = nullptr;           // pinned host staging (pulled bodies on their way to HBM)
    size_t pinned_bytes = 0;
    // Pinned host staging of a call's small uploads / read-backs (descriptors,
    // counters, flags): a pinned copy is a DMA with no host round trip, where a
    // pageable device-to-host copy waits for the stream (~15 us each).  Owned
    // by one call at a time; every user synchronises before it returns.
    void *hio = nullptr;
    size_t hio_bytes = 0;
    // A second (non-blocking) stream for pipelined passes, created on first
    // use; every call that uses it joins it back into `stream` by an event
    // before returning, so callers only ever order against `stream`.
    hipStream_t aux = nullptr;
    hipEvent_t *ev = nullptr;         // event pool of the pipelined passes (timing disabled)
    size_t n_ev = 0;
    // D2 merges (sort.hip): the last sampled dense-key plan, by (mode, n,
    // knobs).  The next such call launches its passes from this shape with no
    // read-back; the device compares the fresh sampled plan with it and a
    // difference counts as a range miss (the call is redone exactly, the
    // entry dropped).
    alignas(8) unsigned char d2_plan[2][128];   // [mode: LWW, OR-Set]
    uint64_t d2_key[2][2] = {{0, 0}, {0, 0}};
    bool d2_ok[2] = {false, false};
    // Polled small read-backs (ctx_read_words): coherent pinned host memory
    // a kernel writes the words into, then a completion word (kCioWords on).
    void *cio = nullptr, *cio_d = nullptr;
    uint64_t cio_seq = 0;
};

namespace crdt {

constexpr int kWave = 64;     // CDNA wavefront width (never 32)

inline int hip_fail(crdt_ctx *ctx, hipError_t e) {
    if (ctx) ctx->last_hip_error = (int)e;
    return e == hipErrorOutOfMemory ? CRDT_E_NOMEM : CRDT_E_HIP;
}

// Kernel-shape knobs (knobs.inc): constexpr defaults in the product build,
// process-wide variables (crdt_set_option) in the diagnostic build only.
#ifdef CRDT_DIAG
#define KNOB(var, def, name, valid) extern int var;
#else
#define KNOB(var, def, name, valid) constexpr int var = (def);
#endif
#include "knobs.inc"
#undef KNOB
#ifdef CRDT_DIAG
constexpr bool kDiagBuild = true;          // kernels keep their timing-diagnostic branches
#else
constexpr bool kDiagBuild = false;         // kernels fold their timing-diagnostic branches away
#endif
#ifdef CRDT_DIAG
// Failpoints (crdt_set_option "fail.*", diagnostic build only): error-path tests.
extern std::atomic<int> g_fail_refmerge;   // the next n RefMerge calls return CRDT_E_NOMEM
extern std::atomic<int> g_fail_zero_bits;  // the next n two-pass merges zero their bitmaps between the passes
extern std::atomic<int> g_fail_d2_plan;    // the next n checked D2 calls find their device plan changed
bool take_fail_zero_bits();                // consumes one "fail.zero_bits" count
bool take_fail_refmerge();                 // consumes one "fail.refmerge" count
bool take_fail_d2_plan();                  // consumes one "fail.d2_plan" count
inline bool fail_refmerge_armed() { return g_fail_refmerge.load() != 0; }
inline bool fail_zero_bits_armed() { return g_fail_zero_bits.load() != 0; }
#else
constexpr bool take_fail_zero_bits() { return false; }
constexpr bool take_fail_refmerge() { return false; }
constexpr bool take_fail_d2_plan() { return false; }
constexpr bool fail_refmerge_armed() { return false; }
constexpr bool fail_zero_bits_armed() { return false; }
#endif

// The context's aux stream / an event pool of at least n events (capi.hip).
int ctx_aux(crdt_ctx *ctx);
int ctx_events(crdt_ctx *ctx, size_t n);

void server_ctx_release(crdt_ctx *ctx);   // server.hip: the context's Server-merge scratch
// sets.hip: out = the stable merge of A and B, all na + nb tuples (crdt_tuples_merge)
int tuples_merge_stable(crdt_ctx *ctx, const crdt_tuples &A, size_t na, const crdt_tuples &B, size_t nb,
                        const crdt_tuples &O);
// ... of many independent pairs, one split + one merge launch per 16 pairs
struct MergePairArg {
    crdt_tuples A;
    size_t na;
    crdt_tuples B;
    size_t nb;
    crdt_tuples O;
};
int tuples_merge_stable_batch(crdt_ctx *ctx, const std::vector<MergePairArg> &pairs);
// gossip.hip: crdt_seg_gather2 (4-byte elements, base 0) over n_max segments
// of which the first *n_dev are real (a count still on the device)
int seg_gather2_dev_count(crdt_ctx *ctx, size_t n_max, const uint64_t *n_dev, const int64_t *code,
                          const uint64_t *a_off, const uint64_t *b_off, uint64_t *dst_off, const uint32_t *a0,
                          const uint32_t *b0, uint32_t *dst0, const uint32_t *a1, const uint32_t *b1, uint32_t *dst1);
// codec.hip: crdt_gossip_decode of nb bodies at data + at[b] (mod 2^64, so the
// bodies may sit in separate device buffers), len[b] bytes each; optionally
// with work enqueued behind the claim pass before the host waits (see there)
int gossip_decode_at(crdt_ctx *ctx, uint32_t nb, const uint8_t *data, const uint64_t *at, const uint64_t *len,
                     uint32_t key_cap, uint64_t kv_base, const uint32_t *slot_base, const uint8_t *host_hdr,
                     crdt_strtab *keys, crdt_strtab *vals, const crdt_gossip_decoded *out, uint32_t *body_status,
                     const std::function<int()> *spec, void *scratch, size_t scratch_cap, bool *spec_stale,
                     uint64_t *multi_pair = nullptr);   // (entries whose pair count is not 1)
size_t gossip_decode_scratch_bytes(uint32_t nb, uint64_t n_e, uint64_t n_p);
// refmerge.hip: crdt_refmerge_batch_pull when every entry of L and of the
// pulled ranges is known to hold exactly one kv pair
int refmerge_batch_pull_one_pair(crdt_ctx *ctx, const crdt_refmerge_in *inp, const crdt_refmerge_out *outp,
                                 const crdt_refmerge_pull *pull, const crdt_refmerge_kv_out *kv);
// codec.hip: the first 32 bytes of each body (zeros if shorter) into host hdr[32 nb].  Synchronises.
int gossip_headers(crdt_ctx *ctx, uint32_t nb, const uint8_t *data, const uint64_t *at, const uint64_t *len,
                   uint8_t *hdr);

// shard.hip: the communicator's collective transport for other protocols
// (population.hip's sharded rounds).  One point-to-point transfer of a group:
// member `member` sends `bytes` from sbuf to global rank `peer`, or receives
// `bytes` from it into rbuf; sends and receives of one (sender, receiver)
// pair are matched in issue order.
struct XP2P {
    size_t member;
    int peer;
    bool send;
    const void *sbuf;
    void *rbuf;
    size_t bytes;
};
size_t comm_members(const crdt_comm *c);        // local members (0: not a valid communicator)
int comm_nranks(const crdt_comm *c);
int comm_rank0(const crdt_comm *c);
crdt_ctx *comm_member_ctx(crdt_comm *c, size_t i);
int comm_allgather(crdt_comm *c, const void *const *send, void *const *recv, size_t bytes);
int comm_p2p(crdt_comm *c, const std::vector<XP2P> &ops);

// ctx->hio at >= bytes (grow-only; the stream is drained before a regrow).
inline int hio_reserve(crdt_ctx *ctx, size_t bytes) {
    if (bytes <= ctx->hio_bytes) return CRDT_OK;
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
    if (ctx->hio) (void)hipHostFree(ctx->hio);
    ctx->hio = nullptr;
    ctx->hio_bytes = 0;
    const size_t want = bytes + bytes / 2 > (64u << 10) ? bytes + bytes / 2 : (64u << 10);
    e = hipHostMalloc(&ctx->hio, want, 0);
    if (e != hipSuccess) {
        ctx->hio = nullptr;
        return hip_fail(ctx, e);
    }
    ctx->hio_bytes = want;
    return CRDT_OK;
}

// Up to kCioBytes of device memory to the host, stream-ordered, without the
// copy engine or an interrupt-driven wait: one one-workgroup kernel copies
// the words into coherent pinned memory and then releases a completion
// word that the host polls (the stream's own state ends the wait if the
// kernel never ran).  *host = the pinned copy, valid until the next call.
// (ctx.read_poll = 0: hipMemcpyAsync + hipStreamSynchronize into ctx->hio.)
constexpr size_t kCioBytes = 4096;
int ctx_read_words(crdt_ctx *ctx, const void *dev_src, size_t bytes, const void **host);
// The same in two halves, so several contexts' reads can be in flight at once
// (one outstanding read per context; end returns its words).
int ctx_read_begin(crdt_ctx *ctx, const void *dev_src, size_t bytes);
int ctx_read_end(crdt_ctx *ctx, const void **host);

// Make the context's device current for this host thread.
inline int bind(crdt_ctx *ctx) {
    if (!ctx) return CRDT_E_INVAL;
    int cur = -1;
    hipError_t e = hipGetDevice(&cur);
    if (e != hipSuccess) return hip_fail(ctx, e);
    if (cur != ctx->device) {
        e = hipSetDevice(ctx->device);
        if (e != hipSuccess) return hip_fail(ctx, e);
    }
    return CRDT_OK;
}

inline int check_launch(crdt_ctx *ctx) {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
}

// Grow the workspace to at least `bytes` (synchronises the stream first so
// that in-flight kernels never see the old buffer freed).
int ws_reserve(crdt_ctx *ctx, size_t bytes);

// Bump allocator over the workspace (256-B aligned carve-outs).
struct Carve {
    char *base;
    size_t used = 0;
    explicit Carve(void *b) : base((char *)b) {}
    template <class T> T *take(size_t n) {
        used = (used + 255) & ~(size_t)255;
        T *p = (T *)(base + used);
        used += n * sizeof(T);
        return p;
    }
    static size_t round(size_t b) { return (b + 255) & ~(size_t)255; }
};

inline bool mul_overflows(size_t a, size_t b) {
    return a != 0 && b > SIZE_MAX / a;
}

inline unsigned grid_for(size_t work_items, unsigned block, unsigned cap) {
    size_t g = (work_items + block - 1) / block;
    if (g > cap) g = cap;
    if (g == 0) g = 1;
    return (unsigned)g;
}

// Device-wide exclusive scan of n uint32 flags/counts into uint64 offsets;
// out[n] receives the total.  Workspace from `tmp` (scan_tmp_bytes(n)).
size_t scan_tmp_bytes(size_t n);
int exclusive_scan_u32(crdt_ctx *ctx, const uint32_t *in, uint64_t *out, size_t n, void *tmp);

// ---- SplitMix64 (Steele, Lea, Flood 2014): the seeded synthetic generator.
__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
__host__ __device__ inline uint64_t stream_key(uint64_t seed, uint64_t stream) {
    return splitmix64(seed ^ splitmix64(stream));
}
// i-th output of a SplitMix64 sequence started at state k.
__host__ __device__ inline uint64_t rnd(uint64_t k, uint64_t i) {
    return splitmix64(k + i * 0x9E3779B97F4A7C15ULL);
}


// Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md
// "Workgroup dispatch": b and b + 8 share an XCD).  Block b -> tile such that
// each XCD's blocks take one contiguous range of the G tiles, in order (a
// bijection on [0, G); speed only, never relied on for correctness).
__device__ __forceinline__ uint32_t xcd_contig(uint32_t b, uint32_t G) {
    const uint32_t x = b & 7u, q = b >> 3, per = G >> 3, rem = G & 7u;
    return x * per + (x < rem ? x : rem) + q;
}

// LDS-DMA staging of one side's run of one field: elements [g0, g0 + cnt) of
// src into the byte array dst from byte *at (16-byte aligned), in 16-byte
// chunks from src + g0's aligned-down address (global_load_lds_dwordx4: 1 KB
// per wave instruction, no VGPRs), the workgroup's waves taking chunks in
// turn.  Returns the element index in dst of element g0; *at advances past
// the chunks.  (Reads at most 15 bytes before / past the run, inside its
// first / last 16-byte block.)
template <typename E, int NWV, int AUX = 0>           // AUX: cache policy bits (2: nontemporal)
__device__ __forceinline__ int dma_run(const E *src, size_t g0, uint32_t cnt, void *dst, uint32_t *at, int wv,
                                       int lane) {
    const char *p = (const char *)(src + g0);
    const uint32_t sh = (uint32_t)((uintptr_t)p & 15);
    const int idx = (int)((*at + sh) / sizeof(E));
    if (cnt == 0) return idx;
    const uint32_t bytes = (sh + cnt * (uint32_t)sizeof(E) + 15) & ~15u;
    const char *g = p - sh;
    char *d = (char *)dst + *at;
    for (uint32_t off = (uint32_t)wv * 1024u; off < bytes; off += NWV * 1024u)
        if (off + 16u * (uint32_t)lane < bytes)
            __builtin_amdgcn_global_load_lds((const void *)(g + off + 16 * lane),
                                             (__attribute__((address_space(3))) void *)(d + off), 16, 0, AUX);
    *at += bytes;
    return idx;
}

}  // namespace crdt
