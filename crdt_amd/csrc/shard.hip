// shard.hip -- replica-sharded joins over a collective transport (SURVEY §8(a) a9, §8(b) crdt_shard_*, §8(e)).
//
// The reference has no collective: its replicas exchange whole logs by HTTP
// pull gossip (main.go:226-258).  Here a replica population is sharded over
// the GPUs of one node and the cross-shard join is a collective over xGMI:
//   * counters / clocks: every member folds its contiguous row shard
//     (crdt_gcounter_fold), then ONE all-reduce(max) of the `nodes`-long fold
//     -- RCCL's unsigned 64-bit max is exactly the join, no order map;
//   * divergent full-state copies (config E2): all-reduce(max) in place;
//   * keyed sets: members own disjoint ordered key ranges, merge them locally,
//     and an all-gather-v (counts by an all-gather, then ONE group of
//     point-to-point transfers) concatenates the outputs in rank order, which
//     is already the globally sorted merged state (a key's LWW / OR-Set output
//     depends only on that key's tuples);
//   * keyed sets of a DISTRIBUTED population (every rank holds only its own
//     tuples, crdt_shard_*_merge_local): sampled splitters (one all-gather),
//     the count matrix (one all-gather), every rank's tuples sent to their
//     key-range owner in ONE point-to-point group (an all-to-all-v of every
//     field of both sides), the owner's stable rank-order merges of the
//     received runs (lengths known on the host: no read-back between levels)
//     and one set merge;
//   * RefMerge of one batch whose logs are split by ts range over the ranks
//     (crdt_shard_refmerge): all-reduce(max) of max(L), the local merge, then
//     integer all-reduces of the replay accumulators (main.go:35-100).
//
// Transport (SURVEY §4's pluggable collective): every protocol above is
// written against three collectives -- in-place all-reduce (sum / max),
// all-gather, and a group of point-to-point sends / receives -- that a
// communicator's transport implements:
//   * RCCL (crdt_shard_comm_create: ncclCommInitAll, one process drives every
//     listed GPU; crdt_shard_comm_init_rank: ncclCommInitRank, one process per
//     GPU) -- the transport of every real multi-GPU communicator;
//   * loopback (crdt_shard_comm_create_loopback): M members on ONE device in
//     one process, each with its own crdt_ctx and stream; the collectives are
//     device copies and a reduction kernel on a transport stream, fenced by
//     events against the member streams (no host synchronisation).  It runs
//     the same planning, offsets, tree merges and reductions at R > 1 on a
//     one-GPU machine.
// The compute (folds, merges, RefMerge) is the same code on either transport.
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <new>
#include <vector>

#include "common.hpp"

static_assert(sizeof(ncclUniqueId) == CRDT_SHARD_ID_BYTES, "RCCL unique id size");

namespace crdt {
enum class XType { U8, U32, I32, U64, I64 };
enum class XOp { Sum, Max };
struct Transport;
}  // namespace crdt

struct crdt_comm {
    struct Member {
        int device = 0;
        crdt_ctx *ctx = nullptr;
        bool own_ctx = false;
        ncclComm_t nccl = nullptr;    // RCCL transport only
        void *scratch = nullptr;      // per-member device scratch (set-merge slices, counts)
        size_t scratch_bytes = 0;
    };
    int nranks = 0;                   // ranks over all processes
    int rank0 = 0;                    // global rank of local member 0
    int last_nccl_error = 0;
    int kind = CRDT_SHARD_RCCL;
    std::vector<Member> m;
    crdt::Transport *x = nullptr;     // owned
};

namespace crdt {

int nccl_fail(crdt_comm *c, ncclResult_t r) {
    if (c) c->last_nccl_error = (int)r;
    return CRDT_E_COMM;
}

// The collectives every protocol of this file is written against.  Per-member
// arguments are indexed by local member; all work is enqueued on the member
// streams (stream-ordered with the member's earlier and later work).
struct Transport {
    virtual ~Transport() {}
    // buf[i] (n elements) := elementwise op over every rank's buf, in place
    virtual int allreduce(crdt_comm *c, void *const *buf, size_t n, XType t, XOp op) = 0;
    // every member's recv[i] + r * bytes := rank r's `bytes` at its send
    // (a send may alias its own rank's slot of recv)
    virtual int allgather(crdt_comm *c, const void *const *send, void *const *recv, size_t bytes) = 0;
    // one group of point-to-point transfers
    virtual int p2p(crdt_comm *c, const std::vector<XP2P> &ops) = 0;
};

namespace {

// ---------------------------------------------------------------- RCCL transport
ncclDataType_t nccl_type(XType t) {
    switch (t) {
        case XType::U8: return ncclUint8;
        case XType::U32: return ncclUint32;
        case XType::I32: return ncclInt32;
        case XType::U64: return ncclUint64;
        default: return ncclInt64;
    }
}

struct RcclTransport final : Transport {
    static int group_end(crdt_comm *c, ncclResult_t r) {
        const ncclResult_t r2 = ncclGroupEnd();
        if (r != ncclSuccess) return nccl_fail(c, r);
        if (r2 != ncclSuccess) return nccl_fail(c, r2);
        return CRDT_OK;
    }
    int allreduce(crdt_comm *c, void *const *buf, size_t n, XType t, XOp op) override {
        ncclResult_t r = ncclGroupStart();
        for (size_t i = 0; i < c->m.size() && r == ncclSuccess; ++i)
            r = ncclAllReduce(buf[i], buf[i], n, nccl_type(t), op == XOp::Max ? ncclMax : ncclSum, c->m[i].nccl,
                              c->m[i].ctx->stream);
        return group_end(c, r);
    }
    int allgather(crdt_comm *c, const void *const *send, void *const *recv, size_t bytes) override {
        ncclResult_t r = ncclGroupStart();
        for (size_t i = 0; i < c->m.size() && r == ncclSuccess; ++i)
            r = ncclAllGather(send[i], recv[i], bytes, ncclUint8, c->m[i].nccl, c->m[i].ctx->stream);
        return group_end(c, r);
    }
    int p2p(crdt_comm *c, const std::vector<XP2P> &ops) override {
        ncclResult_t r = ncclGroupStart();
        for (size_t k = 0; k < ops.size() && r == ncclSuccess; ++k) {
            const XP2P &o = ops[k];
            const auto &mb = c->m[o.member];
            r = o.send ? ncclSend(o.sbuf, o.bytes, ncclUint8, o.peer, mb.nccl, mb.ctx->stream)
                       : ncclRecv(o.rbuf, o.bytes, ncclUint8, o.peer, mb.nccl, mb.ctx->stream);
        }
        return group_end(c, r);
    }
};

// ---------------------------------------------------------------- loopback transport
constexpr int kLoopMax = 64;              // members of a loopback communicator
struct PtrTab {
    void *p[kLoopMax];
};

// buf[m][i] := op over m of buf[m][i], for every member m (in place: each
// element's inputs are read before any of its outputs is written).  Sums are
// taken in the unsigned type (two's complement wrap, main.go:95).
template <class T, bool MAX>
__global__ void k_loop_allreduce(PtrTab t, int M, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        T acc = ((const T *)t.p[0])[i];
        for (int m = 1; m < M; ++m) {
            const T v = ((const T *)t.p[m])[i];
            acc = MAX ? (v > acc ? v : acc) : (T)(acc + v);
        }
        for (int m = 0; m < M; ++m) ((T *)t.p[m])[i] = acc;
    }
}

// One launch for a whole group of device copies (the loopback form of an
// all-gather or a point-to-point group): segment s = (dst, src, bytes) in a
// device table, cut into 64-KB blocks; blk[s] = the first block of segment s
// (blk[nseg] = all blocks).  A workgroup finds its segment by binary search
// and copies its block with the widest access the block's alignment allows.
// (One hipMemcpyAsync per transfer cost ~8 us each on the transport stream:
// 512 of them per distributed set merge at R = 8.)
struct CopySeg {
    char *dst;
    const char *src;
    uint64_t bytes;
};
constexpr uint64_t kCopyBlk = 64u << 10;

__global__ __launch_bounds__(256) void k_batch_copy(const CopySeg *__restrict__ seg, const uint64_t *__restrict__ blk,
                                                    uint32_t nseg) {
    const uint64_t b = blockIdx.x;
    uint32_t lo = 0, hi = nseg;                          // the last s with blk[s] <= b
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (blk[mid] <= b) lo = mid;
        else hi = mid;
    }
    const CopySeg sg = seg[lo];
    const uint64_t o0 = (b - blk[lo]) * kCopyBlk;
    const uint64_t n = sg.bytes - o0 < kCopyBlk ? sg.bytes - o0 : kCopyBlk;
    char *d = sg.dst + o0;
    const char *s = sg.src + o0;
    const uintptr_t al = (uintptr_t)d | (uintptr_t)s;
    if ((al & 15) == 0) {
        const uint64_t nv = n >> 4;
        for (uint64_t i = threadIdx.x; i < nv; i += 256) ((uint4 *)d)[i] = ((const uint4 *)s)[i];
        for (uint64_t i = (nv << 4) + threadIdx.x; i < n; i += 256) d[i] = s[i];
    } else if ((al & 7) == 0) {
        const uint64_t nv = n >> 3;
        for (uint64_t i = threadIdx.x; i < nv; i += 256) ((uint64_t *)d)[i] = ((const uint64_t *)s)[i];
        for (uint64_t i = (nv << 3) + threadIdx.x; i < n; i += 256) d[i] = s[i];
    } else if ((al & 3) == 0) {
        const uint64_t nv = n >> 2;
        for (uint64_t i = threadIdx.x; i < nv; i += 256) ((uint32_t *)d)[i] = ((const uint32_t *)s)[i];
        for (uint64_t i = (nv << 2) + threadIdx.x; i < n; i += 256) d[i] = s[i];
    } else {
        for (uint64_t i = threadIdx.x; i < n; i += 256) d[i] = s[i];
    }
}

struct LoopTransport final : Transport {
    crdt_ctx *ctx = nullptr;              // the transport's own stream (a context for its errors)
    hipEvent_t done = nullptr;
    std::vector<hipEvent_t> ev;           // one per member
    // the copy tables: built in pinned host memory, uploaded on the transport
    // stream, read by k_batch_copy from device memory.  A ring of kTabs slots,
    // each with an event recorded after its upload, so the host only waits
    // when it reuses a slot whose upload (queued behind the members' work)
    // has not run yet -- kTabs collectives later.
    static constexpr int kTabs = 4;
    struct Tab {
        void *h = nullptr, *d = nullptr;
        size_t bytes = 0;
        hipEvent_t up = nullptr;
        bool pending = false;
    } tab[kTabs];
    int next_tab = 0;

    ~LoopTransport() override {
        if (ctx) {
            (void)bind(ctx);
            (void)hipStreamSynchronize(ctx->stream);
        }
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        if (done) (void)hipEventDestroy(done);
        for (Tab &t : tab) {
            if (t.up) (void)hipEventDestroy(t.up);
            if (t.h) (void)hipHostFree(t.h);
            if (t.d) (void)hipFree(t.d);
        }
        if (ctx) (void)crdt_ctx_destroy(ctx);
    }
    int init(int device, size_t members) {
        void *s = nullptr;
        int rc = crdt_stream_create(device, &s);
        if (rc) return rc;
        rc = crdt_ctx_create(device, s, &ctx);
        if (rc) {
            (void)crdt_stream_destroy(s);
            return rc;
        }
        ctx->own_stream = true;
        rc = bind(ctx);
        if (rc) return rc;
        ev.assign(members, nullptr);
        hipError_t e = hipEventCreateWithFlags(&done, hipEventDisableTiming);
        for (Tab &t : tab)
            if (e == hipSuccess) e = hipEventCreateWithFlags(&t.up, hipEventDisableTiming);
        for (size_t i = 0; i < members && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
        return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
    }
    // the transport stream waits for every member's earlier work ...
    int fence_in(crdt_comm *c) {
        int rc = bind(ctx);
        if (rc) return rc;
        hipError_t e = hipSuccess;
        for (size_t i = 0; i < c->m.size() && e == hipSuccess; ++i) {
            e = hipEventRecord(ev[i], c->m[i].ctx->stream);
            if (e == hipSuccess) e = hipStreamWaitEvent(ctx->stream, ev[i], 0);
        }
        return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
    }
    // ... and every member's later work waits for the collective
    int fence_out(crdt_comm *c) {
        hipError_t e = hipEventRecord(done, ctx->stream);
        for (size_t i = 0; i < c->m.size() && e == hipSuccess; ++i) e = hipStreamWaitEvent(c->m[i].ctx->stream, done, 0);
        return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
    }
    // every (dst, src, bytes) of `segs` in one k_batch_copy launch on the
    // transport stream (after fence_in, before fence_out)
    int copy_all(std::vector<CopySeg> &segs) {
        size_t k = 0;
        for (const CopySeg &g : segs)
            if (g.bytes && g.dst != g.src) segs[k++] = g;
        segs.resize(k);
        if (segs.empty()) return CRDT_OK;
        const size_t ns = segs.size();
        const size_t need = Carve::round(ns * sizeof(CopySeg)) + (ns + 1) * 8;
        Tab &t = tab[next_tab];
        next_tab = (next_tab + 1) % kTabs;
        hipError_t e = hipSuccess;
        if (t.pending) e = hipEventSynchronize(t.up);    // this slot's last upload has left its pinned copy
        t.pending = false;
        if (e != hipSuccess) return hip_fail(ctx, e);
        if (need > t.bytes) {
            e = hipStreamSynchronize(ctx->stream);       // (the old device table may still be read)
            if (t.h) (void)hipHostFree(t.h);
            if (t.d) (void)hipFree(t.d);
            t.h = t.d = nullptr;
            t.bytes = 0;
            const size_t want = need * 2 > (64u << 10) ? need * 2 : (64u << 10);
            if (e == hipSuccess) e = hipHostMalloc(&t.h, want, 0);
            if (e == hipSuccess) e = hipMalloc(&t.d, want);
            if (e != hipSuccess) return hip_fail(ctx, e);
            t.bytes = want;
        }
        CopySeg *hs = (CopySeg *)t.h;
        uint64_t *hb = (uint64_t *)((char *)t.h + Carve::round(ns * sizeof(CopySeg)));
        uint64_t nb = 0;
        for (size_t i = 0; i < ns; ++i) {
            hs[i] = segs[i];
            hb[i] = nb;
            nb += (segs[i].bytes + kCopyBlk - 1) / kCopyBlk;
        }
        hb[ns] = nb;
        if (nb >= (1ull << 31)) return CRDT_E_RANGE;
        e = hipMemcpyAsync(t.d, t.h, need, hipMemcpyHostToDevice, ctx->stream);
        if (e == hipSuccess) e = hipEventRecord(t.up, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e);
        t.pending = true;
        k_batch_copy<<<(unsigned)nb, 256, 0, ctx->stream>>>(
            (const CopySeg *)t.d, (const uint64_t *)((char *)t.d + Carve::round(ns * sizeof(CopySeg))),
            (uint32_t)ns);
        return check_launch(ctx);
    }
    int allreduce(crdt_comm *c, void *const *buf, size_t n, XType t, XOp op) override {
        const int M = (int)c->m.size();
        PtrTab p{};
        for (int i = 0; i < M; ++i) p.p[i] = buf[i];
        int rc = fence_in(c);
        if (rc) return rc;
        const unsigned g = grid_for(n, 256, (unsigned)ctx->num_cus * 4);
        const hipStream_t s = ctx->stream;
        const bool mx = op == XOp::Max;
        switch (t) {
            case XType::U8:
                mx ? k_loop_allreduce<uint8_t, true><<<g, 256, 0, s>>>(p, M, n)
                   : k_loop_allreduce<uint8_t, false><<<g, 256, 0, s>>>(p, M, n);
                break;
            case XType::U32:
                mx ? k_loop_allreduce<uint32_t, true><<<g, 256, 0, s>>>(p, M, n)
                   : k_loop_allreduce<uint32_t, false><<<g, 256, 0, s>>>(p, M, n);
                break;
            case XType::I32:
                mx ? k_loop_allreduce<int32_t, true><<<g, 256, 0, s>>>(p, M, n)
                   : k_loop_allreduce<uint32_t, false><<<g, 256, 0, s>>>(p, M, n);
                break;
            case XType::U64:
                mx ? k_loop_allreduce<uint64_t, true><<<g, 256, 0, s>>>(p, M, n)
                   : k_loop_allreduce<uint64_t, false><<<g, 256, 0, s>>>(p, M, n);
                break;
            case XType::I64:
                mx ? k_loop_allreduce<int64_t, true><<<g, 256, 0, s>>>(p, M, n)
                   : k_loop_allreduce<uint64_t, false><<<g, 256, 0, s>>>(p, M, n);
                break;
        }
        rc = check_launch(ctx);
        return rc ? rc : fence_out(c);
    }
    int allgather(crdt_comm *c, const void *const *send, void *const *recv, size_t bytes) override {
        std::vector<CopySeg> segs;
        for (size_t j = 0; j < c->m.size(); ++j)
            for (size_t q = 0; q < c->m.size(); ++q)
                segs.push_back(CopySeg{(char *)recv[j] + q * bytes, (const char *)send[q], bytes});
        int rc = fence_in(c);
        if (!rc) rc = copy_all(segs);
        return rc ? rc : fence_out(c);
    }
    int p2p(crdt_comm *c, const std::vector<XP2P> &ops) override {
        const size_t M = c->m.size();
        std::vector<std::vector<const XP2P *>> snd(M * M), rcv(M * M);   // [from * M + to]
        for (const XP2P &o : ops) {
            if (o.peer < 0 || (size_t)o.peer >= M || o.member >= M) return CRDT_E_INVAL;
            (o.send ? snd[o.member * M + o.peer] : rcv[(size_t)o.peer * M + o.member]).push_back(&o);
        }
        for (size_t k = 0; k < M * M; ++k) {
            if (snd[k].size() != rcv[k].size()) return nccl_fail(c, ncclInvalidUsage);
            for (size_t j = 0; j < snd[k].size(); ++j)
                if (snd[k][j]->bytes != rcv[k][j]->bytes) return nccl_fail(c, ncclInvalidUsage);
        }
        std::vector<CopySeg> segs;
        for (size_t k = 0; k < M * M; ++k)
            for (size_t j = 0; j < snd[k].size(); ++j)
                segs.push_back(CopySeg{(char *)rcv[k][j]->rbuf, (const char *)snd[k][j]->sbuf, snd[k][j]->bytes});
        int rc = fence_in(c);
        if (!rc) rc = copy_all(segs);
        return rc ? rc : fence_out(c);
    }
};

// ---------------------------------------------------------------- helpers
// Grow a member's scratch to `bytes` (the member's stream is drained first;
// the old contents are lost).
int scratch_reserve(crdt_comm::Member &mb, size_t bytes) {
    if (bytes <= mb.scratch_bytes) return CRDT_OK;
    int rc = bind(mb.ctx);
    if (rc) return rc;
    hipError_t e = hipStreamSynchronize(mb.ctx->stream);
    if (e != hipSuccess) return hip_fail(mb.ctx, e);
    if (mb.scratch) (void)hipFree(mb.scratch);
    mb.scratch = nullptr;
    mb.scratch_bytes = 0;
    const size_t want = (bytes + bytes / 4 + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
    e = hipMalloc(&mb.scratch, want);
    if (e != hipSuccess) {
        mb.scratch = nullptr;
        return hip_fail(mb.ctx, e);
    }
    mb.scratch_bytes = want;
    return CRDT_OK;
}

int sync_all(crdt_comm *c) {
    for (auto &mb : c->m) {
        int rc = bind(mb.ctx);
        if (rc) return rc;
        hipError_t e = hipStreamSynchronize(mb.ctx->stream);
        if (e != hipSuccess) return hip_fail(mb.ctx, e);
    }
    return CRDT_OK;
}

// Every member's device status word (cleared when raised): all members'
// polled reads in flight at once, then collected -- one wait for the slowest
// member instead of one synchronising copy per member.
int check_devices(crdt_comm *c) {
    for (auto &mb : c->m) {
        int rc = bind(mb.ctx);
        if (!rc) rc = ctx_read_begin(mb.ctx, mb.ctx->dev_status, sizeof(uint32_t));
        if (rc) return rc;
    }
    bool raised = false;
    for (auto &mb : c->m) {
        int rc = bind(mb.ctx);
        const void *hw = nullptr;
        if (!rc) rc = ctx_read_end(mb.ctx, &hw);
        if (rc) return rc;
        if (*(const uint32_t *)hw) {
            raised = true;
            hipError_t e = hipMemsetAsync(mb.ctx->dev_status, 0, sizeof(uint32_t), mb.ctx->stream);
            if (e != hipSuccess) return hip_fail(mb.ctx, e);
        }
    }
    return raised ? CRDT_E_DEVICE : CRDT_OK;
}

// Copy n words of member 0's device buffer to the host (synchronises member 0).
int read_member0(crdt_comm *c, const uint64_t *src, uint64_t *dst, size_t n) {
    auto &mb = c->m[0];
    int rc = bind(mb.ctx);
    if (rc || n == 0) return rc;
    if (n * 8 <= kCioBytes) {                          // small: the polled pinned read (no pageable copy)
        const void *hw = nullptr;
        rc = ctx_read_words(mb.ctx, src, n * 8, &hw);
        if (!rc) memcpy(dst, hw, n * 8);
        return rc;
    }
    hipError_t e = hipMemcpyAsync(dst, src, n * 8, hipMemcpyDeviceToHost, mb.ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(mb.ctx->stream);
    return e == hipSuccess ? CRDT_OK : hip_fail(mb.ctx, e);
}

bool valid(const crdt_comm *c) { return c && !c->m.empty() && c->x; }

// out[i] = key[i * n / per], i < per (evenly spaced sample of a sorted key array).
__global__ void k_sample_keys(const uint64_t *__restrict__ key, size_t n, unsigned per, uint64_t *__restrict__ out) {
    const unsigned i = blockIdx.x * 256 + threadIdx.x;
    if (i < per) out[i] = key[(size_t)((unsigned __int128)i * n / per)];
}

constexpr unsigned kSamplesPerSide = 256;
constexpr uint64_t kKeyEnd = ~0ULL;       // splitter sentinel: "to the end of the key space"

int comm_new(int n, crdt_comm **out) {
    crdt_comm *c = new (std::nothrow) crdt_comm();
    if (!c) return CRDT_E_NOMEM;
    c->nranks = n;
    c->m.resize(n);
    *out = c;
    return CRDT_OK;
}

// member i: a context on its own library-owned stream
int member_own_ctx(crdt_comm::Member &mb, int device) {
    void *s = nullptr;
    int rc = crdt_stream_create(device, &s);
    if (rc) return rc;
    rc = crdt_ctx_create(device, s, &mb.ctx);
    if (rc) {
        (void)crdt_stream_destroy(s);
        return rc;
    }
    mb.ctx->own_stream = true;                          // destroyed with the context
    mb.own_ctx = true;
    mb.device = device;
    return CRDT_OK;
}

}  // namespace

size_t comm_members(const crdt_comm *c) { return valid(c) ? c->m.size() : 0; }
int comm_nranks(const crdt_comm *c) { return c->nranks; }
int comm_rank0(const crdt_comm *c) { return c->rank0; }
crdt_ctx *comm_member_ctx(crdt_comm *c, size_t i) { return c->m[i].ctx; }
int comm_allgather(crdt_comm *c, const void *const *send, void *const *recv, size_t bytes) {
    return c->x->allgather(c, send, recv, bytes);
}
int comm_p2p(crdt_comm *c, const std::vector<XP2P> &ops) { return c->x->p2p(c, ops); }

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_shard_unique_id(void *id, size_t cap) {
    if (!id || cap < sizeof(ncclUniqueId)) return CRDT_E_INVAL;
    ncclUniqueId u;
    ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return CRDT_E_COMM;
    memcpy(id, &u, sizeof u);
    return CRDT_OK;
}

extern "C" int crdt_rccl_info(int *version, char *path, size_t cap) {
    if (!version) return CRDT_E_INVAL;
    int v = 0;
    if (ncclGetVersion(&v) != ncclSuccess) return CRDT_E_DEVICE;
    *version = v;
    if (path && cap) {
        Dl_info di{};
        const char *f = dladdr((const void *)&ncclGetVersion, &di) && di.dli_fname ? di.dli_fname : "";
        strncpy(path, f, cap - 1);
        path[cap - 1] = 0;
    }
    return CRDT_OK;
}

extern "C" int crdt_shard_comm_create(const int *devices, int n, crdt_comm **out) {
    if (!out) return CRDT_E_INVAL;
    *out = nullptr;
    if (!devices || n <= 0) return CRDT_E_INVAL;
    crdt_comm *c = nullptr;
    int rc = comm_new(n, &c);
    if (rc) return rc;
    c->x = new (std::nothrow) RcclTransport();
    if (!c->x) rc = CRDT_E_NOMEM;
    for (int i = 0; i < n && rc == CRDT_OK; ++i) {
        for (int j = 0; j < i; ++j)
            if (devices[j] == devices[i]) rc = CRDT_E_INVAL;      // RCCL: one rank per GPU (loopback: one GPU)
        if (!rc) rc = member_own_ctx(c->m[i], devices[i]);
    }
    if (rc == CRDT_OK) {
        std::vector<ncclComm_t> comms(n);
        ncclResult_t r = ncclCommInitAll(comms.data(), n, devices);
        if (r != ncclSuccess) rc = nccl_fail(c, r);
        else
            for (int i = 0; i < n; ++i) c->m[i].nccl = comms[i];
    }
    if (rc) {
        (void)crdt_shard_comm_destroy(c);
        return rc;
    }
    *out = c;
    return CRDT_OK;
}

extern "C" int crdt_shard_comm_create_loopback(int device, int members, crdt_comm **out) {
    if (!out) return CRDT_E_INVAL;
    *out = nullptr;
    if (members <= 0 || members > kLoopMax) return CRDT_E_INVAL;
    crdt_comm *c = nullptr;
    int rc = comm_new(members, &c);
    if (rc) return rc;
    c->kind = CRDT_SHARD_LOOPBACK;
    LoopTransport *lt = new (std::nothrow) LoopTransport();
    c->x = lt;
    rc = lt ? lt->init(device, (size_t)members) : CRDT_E_NOMEM;
    for (int i = 0; i < members && rc == CRDT_OK; ++i) rc = member_own_ctx(c->m[i], device);
    if (rc) {
        (void)crdt_shard_comm_destroy(c);
        return rc;
    }
    *out = c;
    return CRDT_OK;
}

extern "C" int crdt_shard_comm_init_rank(crdt_ctx *ctx, const void *id, int nranks, int rank, crdt_comm **out) {
    if (!out) return CRDT_E_INVAL;
    *out = nullptr;
    if (!ctx || !id || nranks <= 0 || rank < 0 || rank >= nranks) return CRDT_E_INVAL;
    int rc = bind(ctx);
    if (rc) return rc;
    crdt_comm *c = nullptr;
    rc = comm_new(1, &c);
    if (rc) return rc;
    c->nranks = nranks;
    c->rank0 = rank;
    c->m[0].device = ctx->device;
    c->m[0].ctx = ctx;                      // borrowed: the caller's context and stream
    c->x = new (std::nothrow) RcclTransport();
    if (!c->x) {
        (void)crdt_shard_comm_destroy(c);
        return CRDT_E_NOMEM;
    }
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    ncclResult_t r = ncclCommInitRank(&c->m[0].nccl, nranks, u, rank);
    if (r != ncclSuccess) {
        c->m[0].nccl = nullptr;
        rc = nccl_fail(c, r);
        (void)crdt_shard_comm_destroy(c);
        return rc;
    }
    *out = c;
    return CRDT_OK;
}

extern "C" int crdt_shard_comm_destroy(crdt_comm *c) {
    if (!c) return CRDT_OK;
    for (auto &mb : c->m) {
        if (mb.ctx) {
            (void)bind(mb.ctx);
            (void)hipStreamSynchronize(mb.ctx->stream);
        }
    }
    delete c->x;                            // (loopback: drains its stream)
    for (auto &mb : c->m) {
        if (mb.nccl) (void)ncclCommDestroy(mb.nccl);
        if (mb.scratch) (void)hipFree(mb.scratch);
        if (mb.own_ctx && mb.ctx) (void)crdt_ctx_destroy(mb.ctx);
    }
    delete c;
    return CRDT_OK;
}

extern "C" int crdt_shard_comm_info(const crdt_comm *c, int *members, int *nranks, int *rank0) {
    if (!valid(c) || !members || !nranks || !rank0) return CRDT_E_INVAL;
    *members = (int)c->m.size();
    *nranks = c->nranks;
    *rank0 = c->rank0;
    return CRDT_OK;
}

extern "C" int crdt_shard_comm_transport(const crdt_comm *c, int *kind) {
    if (!valid(c) || !kind) return CRDT_E_INVAL;
    *kind = c->kind;
    return CRDT_OK;
}

extern "C" int crdt_shard_member_ctx(crdt_comm *c, int member, crdt_ctx **ctx) {
    if (!valid(c) || !ctx || member < 0 || member >= (int)c->m.size()) return CRDT_E_INVAL;
    *ctx = c->m[member].ctx;
    return CRDT_OK;
}

extern "C" int crdt_shard_comm_last_error(const crdt_comm *c) { return c ? c->last_nccl_error : 0; }

extern "C" int crdt_shard_sync(crdt_comm *c) {
    if (!valid(c)) return CRDT_E_INVAL;
    return sync_all(c);
}

// buf[i] (member i, n uint64 on its device) := elementwise unsigned max over
// every rank's buf (RCCL: ncclAllReduce(ncclUint64, ncclMax)), in place.
extern "C" int crdt_shard_allreduce_max_u64(crdt_comm *c, uint64_t *const *buf, size_t n) {
    if (!valid(c) || !buf) return CRDT_E_INVAL;
    if (n == 0) return CRDT_OK;
    for (size_t i = 0; i < c->m.size(); ++i)
        if (!buf[i]) return CRDT_E_INVAL;
    return c->x->allreduce(c, (void *const *)buf, n, XType::U64, XOp::Max);
}

extern "C" int crdt_shard_allreduce(crdt_comm *c, void *const *buf, size_t n, int type, int op) {
    if (!valid(c) || !buf) return CRDT_E_INVAL;
    XType t;
    switch (type) {
        case CRDT_SHARD_I64: t = XType::I64; break;
        case CRDT_SHARD_U64: t = XType::U64; break;
        case CRDT_SHARD_U32: t = XType::U32; break;
        case CRDT_SHARD_I32: t = XType::I32; break;
        default: return CRDT_E_INVAL;
    }
    XOp o;
    switch (op) {
        case CRDT_SHARD_SUM: o = XOp::Sum; break;
        case CRDT_SHARD_MAX: o = XOp::Max; break;
        default: return CRDT_E_INVAL;
    }
    if (n == 0) return CRDT_OK;
    for (size_t i = 0; i < c->m.size(); ++i)
        if (!buf[i]) return CRDT_E_INVAL;
    return c->x->allreduce(c, buf, n, t, o);
}

// Whole-population G-Counter / vector-clock join (config E1): member i folds
// its [rows[i] x nodes] row shard into out[i], then one all-reduce(max).
// Every member's out holds the global fold on return (enqueued; async).
extern "C" int crdt_shard_fold_max_u64(crdt_comm *c, const uint64_t *const *shard, const size_t *rows, size_t nodes,
                                       uint64_t *const *out) {
    if (!valid(c) || !shard || !rows || !out || nodes == 0) return CRDT_E_INVAL;
    for (size_t i = 0; i < c->m.size(); ++i) {
        int rc = crdt_gcounter_fold(c->m[i].ctx, shard[i], rows[i], nodes, out[i]);
        if (rc) return rc;
    }
    return crdt_shard_allreduce_max_u64(c, out, nodes);
}

namespace {

// The scratch head every keyed-set protocol keeps: word 0 = the member's own
// tuple count (device), words 1 .. R = every rank's (all-gathered).
size_t head_bytes(size_t R) { return Carve::round((R + 2) * 8); }

// Keyed-set all-gather-v from the counts in every member's scratch word 0:
// one all-gather of the counts, one read-back (member 0), then every field of
// every rank's tuples in ONE point-to-point group (send to every rank, receive
// from every rank at its offset) -- not one broadcast per root and field.
int allgather_v_head(crdt_comm *c, const crdt_tuples *local, const crdt_tuples *out, size_t cap, size_t *n_total) {
    const size_t M = c->m.size(), R = (size_t)c->nranks;
    std::vector<const void *> snd(M);
    std::vector<void *> rcv(M);
    for (size_t i = 0; i < M; ++i) {
        snd[i] = c->m[i].scratch;
        rcv[i] = (uint64_t *)c->m[i].scratch + 1;
    }
    int rc = c->x->allgather(c, snd.data(), rcv.data(), 8);
    if (rc) return rc;
    std::vector<uint64_t> cnt(R), off(R + 1, 0);
    rc = read_member0(c, (const uint64_t *)c->m[0].scratch + 1, cnt.data(), R);
    if (rc) return rc;
    for (size_t q = 0; q < R; ++q) off[q + 1] = off[q] + cnt[q];
    *n_total = off[R];
    if (off[R] > cap) return CRDT_E_RANGE;
    for (size_t i = 0; i < M; ++i) {
        const size_t g = (size_t)c->rank0 + i;
        if (off[R] && (!out[i].key || !out[i].ts || !out[i].rep || !out[i].tomb)) return CRDT_E_INVAL;
        if (cnt[g] && (!local[i].key || !local[i].ts || !local[i].rep || !local[i].tomb)) return CRDT_E_INVAL;
    }
    std::vector<XP2P> ops;
    const size_t esz[4] = {8, 8, 4, 1};
    for (size_t i = 0; i < M; ++i) {
        const size_t g = (size_t)c->rank0 + i;
        const void *fs[4] = {local[i].key, local[i].ts, local[i].rep, local[i].tomb};
        char *fd[4] = {(char *)out[i].key, (char *)out[i].ts, (char *)out[i].rep, (char *)out[i].tomb};
        for (size_t q = 0; q < R; ++q)
            for (int f = 0; f < 4; ++f) {
                if (cnt[g]) ops.push_back(XP2P{i, (int)q, true, fs[f], nullptr, cnt[g] * esz[f]});
                if (cnt[q]) ops.push_back(XP2P{i, (int)q, false, nullptr, fd[f] + off[q] * esz[f], cnt[q] * esz[f]});
            }
    }
    return c->x->p2p(c, ops);
}

}  // namespace

// Keyed-set all-gather-v: member i contributes local[i] (n_local[i] tuples on
// its device); every member's out[i] receives the concatenation in global
// rank order.  *n_total (host) = the gathered length.  Synchronises once (the
// counts are all-gathered and read back before the transfers are sized).
extern "C" int crdt_shard_set_allgather_v(crdt_comm *c, const crdt_tuples *local, const size_t *n_local,
                                          const crdt_tuples *out, size_t cap, size_t *n_total) {
    if (!valid(c) || !local || !n_local || !out || !n_total) return CRDT_E_INVAL;
    const size_t M = c->m.size(), R = (size_t)c->nranks;
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        int rc = scratch_reserve(mb, head_bytes(R));
        if (rc) return rc;
        rc = bind(mb.ctx);
        if (rc) return rc;
        uint64_t v = n_local[i];
        hipError_t e = hipMemcpyAsync(mb.scratch, &v, sizeof v, hipMemcpyHostToDevice, mb.ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(mb.ctx->stream);    // v is a stack value
        if (e != hipSuccess) return hip_fail(mb.ctx, e);
    }
    return allgather_v_head(c, local, out, cap, n_total);
}

namespace {

// Sharded LWW / OR-Set merge of inputs every member holds in full (a[i], b[i]
// on member i's device, identical contents).  Splitters: the nranks-quantiles
// of an evenly spaced sample of both key arrays -- computed from identical
// data, so every rank derives the same ones without an exchange.
int shard_set_merge(crdt_comm *c, bool lww, const crdt_tuples *a, size_t na, const crdt_tuples *b, size_t nb,
                    const crdt_tuples *out, size_t cap, size_t *n_out) {
    if (!valid(c) || !a || !b || !out || !n_out) return CRDT_E_INVAL;
    const size_t M = c->m.size(), R = (size_t)c->nranks;
    for (size_t i = 0; i < M; ++i) {
        if (na && !a[i].key) return CRDT_E_INVAL;
        if (nb && !b[i].key) return CRDT_E_INVAL;
    }
    // 1. splitters from member 0's copy
    std::vector<uint64_t> spl(R + 1, 0);
    spl[R] = kKeyEnd;
    {
        auto &mb = c->m[0];
        int rc = scratch_reserve(mb, 2 * kSamplesPerSide * sizeof(uint64_t));
        if (rc) return rc;
        rc = bind(mb.ctx);
        if (rc) return rc;
        uint64_t *smp = (uint64_t *)mb.scratch;
        const unsigned pa = na ? kSamplesPerSide : 0, pb = nb ? kSamplesPerSide : 0;
        if (pa) k_sample_keys<<<1, 256, 0, mb.ctx->stream>>>(a[0].key, na, pa, smp);
        if (pb) k_sample_keys<<<1, 256, 0, mb.ctx->stream>>>(b[0].key, nb, pb, smp + pa);
        rc = check_launch(mb.ctx);
        if (rc) return rc;
        std::vector<uint64_t> h(pa + pb);
        rc = read_member0(c, smp, h.data(), h.size());
        if (rc) return rc;
        std::sort(h.begin(), h.end());
        if (!h.empty())
            for (size_t q = 1; q < R; ++q) spl[q] = h[q * h.size() / R];
    }
    // 2. each member's key range [spl[g], spl[g+1]) of both inputs (lower_bound
    //    of the splitters on the member's own copy), merged on its device into
    //    its scratch
    std::vector<crdt_tuples> loc(M);
    std::vector<uint64_t> bounds(4 * M);
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        const size_t g = (size_t)c->rank0 + i;
        int rc = scratch_reserve(mb, 4096);
        if (rc) return rc;
        rc = bind(mb.ctx);
        if (rc) return rc;
        uint64_t *pr = (uint64_t *)mb.scratch, *lb = pr + 2;
        const uint64_t probes[2] = {spl[g], spl[g + 1]};
        hipError_t e = hipMemcpyAsync(pr, probes, sizeof probes, hipMemcpyHostToDevice, mb.ctx->stream);
        if (e != hipSuccess) return hip_fail(mb.ctx, e);
        uint64_t *hb = &bounds[4 * i];
        hb[0] = 0, hb[1] = na, hb[2] = 0, hb[3] = nb;
        if (na) rc = crdt_u64_lower_bound(mb.ctx, a[i].key, na, pr, 2, lb);
        if (!rc && nb) rc = crdt_u64_lower_bound(mb.ctx, b[i].key, nb, pr, 2, lb + 2);
        if (rc) return rc;
        uint64_t got[4];
        e = hipMemcpyAsync(got, lb, sizeof got, hipMemcpyDeviceToHost, mb.ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(mb.ctx->stream);
        if (e != hipSuccess) return hip_fail(mb.ctx, e);
        const bool top = g + 1 == R;                 // the last range runs to the end of the key space
        if (na) hb[0] = g ? got[0] : 0, hb[1] = top ? na : got[1];
        if (nb) hb[2] = g ? got[2] : 0, hb[3] = top ? nb : got[3];
    }
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        const uint64_t *hb = &bounds[4 * i];
        const size_t ma = hb[1] - hb[0], mb_n = hb[3] - hb[2], cap_i = ma + mb_n;
        // scratch: [head (word 0: the merged count) | key | ts | rep | tomb] of capacity cap_i
        const size_t need = head_bytes(R) + Carve::round(cap_i * 8) * 2 + Carve::round(cap_i * 4) +
                            Carve::round(cap_i) + 1024;
        int rc = scratch_reserve(mb, need);
        if (rc) return rc;
        Carve w(mb.scratch);
        uint64_t *count = w.take<uint64_t>(R + 2);
        loc[i].key = w.take<uint64_t>(cap_i);
        loc[i].ts = w.take<uint64_t>(cap_i);
        loc[i].rep = w.take<uint32_t>(cap_i);
        loc[i].tomb = w.take<uint8_t>(cap_i);
        crdt_tuples sa{a[i].key + hb[0], a[i].ts + hb[0], a[i].rep + hb[0], a[i].tomb + hb[0]};
        crdt_tuples sb{b[i].key + hb[2], b[i].ts + hb[2], b[i].rep + hb[2], b[i].tomb + hb[2]};
        if (!ma) sa = crdt_tuples{nullptr, nullptr, nullptr, nullptr};
        if (!mb_n) sb = crdt_tuples{nullptr, nullptr, nullptr, nullptr};
        rc = lww ? crdt_lww_merge(mb.ctx, &sa, ma, &sb, mb_n, &loc[i], count)
                 : crdt_orset_merge(mb.ctx, &sa, ma, &sb, mb_n, &loc[i], count);
        if (rc) return rc;
    }
    // 3. all-gather-v in rank order (the merged counts travel from the scratch heads)
    int rc = allgather_v_head(c, loc.data(), out, cap, n_out);
    if (rc) return rc;
    return check_devices(c);
}

}  // namespace

extern "C" int crdt_shard_lww_merge(crdt_comm *c, const crdt_tuples *a, size_t na, const crdt_tuples *b, size_t nb,
                                    const crdt_tuples *out, size_t cap, size_t *n_out) {
    return shard_set_merge(c, true, a, na, b, nb, out, cap, n_out);
}

extern "C" int crdt_shard_orset_merge(crdt_comm *c, const crdt_tuples *a, size_t na, const crdt_tuples *b, size_t nb,
                                      const crdt_tuples *out, size_t cap, size_t *n_out) {
    return shard_set_merge(c, false, a, na, b, nb, out, cap, n_out);
}

// ---------------------------------------------------------------- RefMerge by ts range (§8(e))
// (*Server).merge() (main.go:35-100) of one batch of replicas whose Diff /
// RemoteDiff logs are split by ts range over the ranks (global rank g holds
// the g-th range of every replica, ranks in ascending ts order).  The four
// steps of crdt_amd/shard.py's sharded_refmerge, on the communicator's
// transport and member streams, no host synchronisation:
//   1. crdt_refmerge_local_maxl, all-reduce(max, int64): the GLOBAL max(L) of
//      every replica (remote ts at or above it are dropped, main.go:49);
//   2. crdt_refmerge_batch_ex with that max: the member's slice of the new
//      Diff (slices concatenate in rank order) and its unreduced accumulators;
//   3. the key's max-ts holder across ranks: max of shard << 40 | rank
//      (crdt_refmerge_acc_rank), sum of the owner's string id, sum of the
//      wrapped sums (int64 two's complement: main.go:95) and of the parsable
//      counts;
//   4. crdt_refmerge_finalize: CurrentState, identical on every member.
// Integer reductions only: bit-exact with crdt_refmerge_batch of the
// unsharded batch for any rank count.
extern "C" int crdt_shard_refmerge(crdt_comm *c, const crdt_refmerge_in *in, const crdt_refmerge_out *out) {
    if (!valid(c) || !in || !out) return CRDT_E_INVAL;
    const size_t M = c->m.size();
    const uint32_t P = in[0].replicas, ns = in[0].n_slots;
    for (size_t i = 0; i < M; ++i)
        if (in[i].replicas != P || in[i].n_slots != ns) return CRDT_E_INVAL;   // one batch, one slot space
    if (P == 0) return CRDT_OK;
    if ((size_t)c->rank0 + M > (1u << 23)) return CRDT_E_RANGE;            // shard << 40 | rank packing
    struct Bufs {
        int64_t *maxl, *c, *cmax, *v;
        crdt_refmerge_acc acc;
    };
    std::vector<Bufs> bf(M);
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        const size_t need = Carve::round(P * 8) + Carve::round(ns * 8 + 8) * 5 + Carve::round(ns * 4 + 4) + 1024;
        int rc = scratch_reserve(mb, need);
        if (rc) return rc;
        Carve w(mb.scratch);
        bf[i].maxl = w.take<int64_t>(P);
        bf[i].acc.best = w.take<uint64_t>(ns + 1);
        bf[i].acc.sum = w.take<int64_t>(ns + 1);
        bf[i].acc.npar = w.take<uint32_t>(ns + 1);
        bf[i].c = w.take<int64_t>(ns + 1);
        bf[i].cmax = w.take<int64_t>(ns + 1);
        bf[i].v = w.take<int64_t>(ns + 1);
    }
    auto each = [&](auto fn) -> int {
        for (size_t i = 0; i < M; ++i) {
            int rc = bind(c->m[i].ctx);
            if (!rc) rc = fn(i, c->m[i].ctx);
            if (rc) return rc;
        }
        return CRDT_OK;
    };
    std::vector<void *> ptr(M);
    auto allreduce = [&](auto ptr_of, size_t n, XType t, XOp op) -> int {
        for (size_t i = 0; i < M; ++i) ptr[i] = ptr_of(i);
        return c->x->allreduce(c, ptr.data(), n, t, op);
    };
    // 1. the global max(L) per replica
    int rc = each([&](size_t i, crdt_ctx *x) { return crdt_refmerge_local_maxl(x, &in[i], bf[i].maxl); });
    if (!rc) rc = allreduce([&](size_t i) { return (void *)bf[i].maxl; }, P, XType::I64, XOp::Max);
    // 2. the local merges (new-Diff slices, unreduced accumulators)
    if (!rc) rc = each([&](size_t i, crdt_ctx *x) {
        return crdt_refmerge_batch_ex(x, &in[i], &out[i], bf[i].maxl, &bf[i].acc);
    });
    if (rc) return rc;
    if (ns == 0) return CRDT_OK;
    // 3. the accumulators reduced across ranks
    if (c->nranks > 1) {
        rc = each([&](size_t i, crdt_ctx *x) {
            int r = crdt_refmerge_acc_rank(x, &bf[i].acc, ns, (uint32_t)(c->rank0 + i), bf[i].c);
            if (r) return r;
            hipError_t e = hipMemcpyAsync(bf[i].cmax, bf[i].c, ns * 8, hipMemcpyDeviceToDevice, x->stream);
            return e == hipSuccess ? CRDT_OK : hip_fail(x, e);
        });
        if (!rc) rc = allreduce([&](size_t i) { return (void *)bf[i].cmax; }, ns, XType::I64, XOp::Max);
        if (!rc) rc = each([&](size_t i, crdt_ctx *x) {
            return crdt_refmerge_acc_owner_str(x, &bf[i].acc, ns, bf[i].c, bf[i].cmax, bf[i].v);
        });
        if (!rc) rc = allreduce([&](size_t i) { return (void *)bf[i].v; }, ns, XType::I64, XOp::Sum);
        if (!rc) rc = allreduce([&](size_t i) { return (void *)bf[i].acc.sum; }, ns, XType::I64, XOp::Sum);
        if (!rc) rc = allreduce([&](size_t i) { return (void *)bf[i].acc.npar; }, ns, XType::U32, XOp::Sum);
        if (!rc) rc = each([&](size_t i, crdt_ctx *x) {
            return crdt_refmerge_acc_set_best(x, &bf[i].acc, ns, bf[i].cmax, bf[i].v);
        });
        if (rc) return rc;
    }
    // 4. CurrentState on every member
    return each([&](size_t i, crdt_ctx *x) {
        return crdt_refmerge_finalize(x, &bf[i].acc, ns, in[i].str_bytes, in[i].str_off, in[i].n_str, &out[i]);
    });
}

// ---------------------------------------------------------------- all-to-all-v
// Member i sends send_counts[i * R + q] elements of elem_size bytes to global
// rank q, from its send buffer's segments in rank order, and receives
// recv_counts[i * R + p] elements from rank p into its recv buffer, segments
// in rank order (one point-to-point group, enqueued on the member streams).
extern "C" int crdt_shard_alltoallv(crdt_comm *c, const void *const *send, const size_t *send_counts,
                                    void *const *recv, const size_t *recv_counts, size_t elem_size) {
    if (!valid(c) || !send || !send_counts || !recv || !recv_counts || elem_size == 0) return CRDT_E_INVAL;
    const size_t M = c->m.size(), R = (size_t)c->nranks;
    std::vector<XP2P> ops;
    for (size_t i = 0; i < M; ++i) {
        size_t ns = 0, nr = 0;
        for (size_t q = 0; q < R; ++q) ns += send_counts[i * R + q], nr += recv_counts[i * R + q];
        if ((ns && !send[i]) || (nr && !recv[i])) return CRDT_E_INVAL;
        const char *sb = (const char *)send[i];
        char *rb = (char *)recv[i];
        size_t so = 0, ro = 0;
        for (size_t q = 0; q < R; ++q) {
            const size_t sn = send_counts[i * R + q] * elem_size, rn = recv_counts[i * R + q] * elem_size;
            if (sn) ops.push_back(XP2P{i, (int)q, true, sb + so, nullptr, sn});
            if (rn) ops.push_back(XP2P{i, (int)q, false, nullptr, rb + ro, rn});
            so += sn;
            ro += rn;
        }
    }
    return c->x->p2p(c, ops);
}

namespace {

// Splitters of a distributed key population from per-rank samples: block p
// of the gathered samples = [n_a, n_b, S keys of A, S keys of B] (a side
// with n > 0 sampled at i * n / S, each sample weighing n; an empty side's
// samples weigh 0).  Inner splitter q = the first sample key (in key order)
// at which the cumulative weight reaches q / R of the total.  Rank r owns
// keys [spl[r], spl[r+1]); crdt_amd/shard.py weighted_splitters is the same rule.
std::vector<uint64_t> weighted_splitters(const uint64_t *blocks, size_t R, size_t S) {
    // the samples of every non-empty side, walked in key order by a k-way
    // merge of the (sorted) sample lists: each crossing of q / R of the total
    // weight names splitter q.  Among equal keys the walk order does not
    // matter: a crossing inside a run of equal keys names that key.
    struct List {
        const uint64_t *k;
        uint64_t w;
        size_t i;
    };
    std::vector<List> ls;
    unsigned __int128 W = 0;
    for (size_t p = 0; p < R; ++p) {
        const uint64_t *b = blocks + p * (2 + 2 * S);
        for (int side = 0; side < 2; ++side)
            if (b[side] && S) {
                ls.push_back(List{b + 2 + side * S, b[side], 0});
                W += (unsigned __int128)S * b[side];
            }
    }
    std::vector<uint64_t> spl(R + 1, 0);
    spl[R] = kKeyEnd;
    if (W == 0) return spl;
    auto later = [&](int x, int y) { return ls[x].k[ls[x].i] > ls[y].k[ls[y].i]; };
    std::vector<int> h(ls.size());
    for (size_t x = 0; x < ls.size(); ++x) h[x] = (int)x;
    std::make_heap(h.begin(), h.end(), later);
    unsigned __int128 cum = 0;
    uint64_t last = 0;
    size_t q = 1;
    while (q < R && !h.empty()) {
        std::pop_heap(h.begin(), h.end(), later);
        List &l = ls[h.back()];
        last = l.k[l.i];
        cum += l.w;
        while (q < R && cum * R >= (unsigned __int128)q * W) spl[q++] = last;
        if (++l.i < S) std::push_heap(h.begin(), h.end(), later);
        else h.pop_back();
    }
    for (; q < R; ++q) spl[q] = last;                  // (not reached: the walk ends at cum = W)
    return spl;
}

__global__ void k_sample_block(const uint64_t *__restrict__ ka, size_t na, const uint64_t *__restrict__ kb, size_t nb,
                               unsigned S, uint64_t *__restrict__ blk) {
    const unsigned i = blockIdx.x * 256 + threadIdx.x;
    if (i == 0) {
        blk[0] = na;
        blk[1] = nb;
    }
    if (i < S) {
        blk[2 + i] = na ? ka[(size_t)((unsigned __int128)i * na / S)] : 0;
        blk[2 + S + i] = nb ? kb[(size_t)((unsigned __int128)i * nb / S)] : 0;
    }
}

// A member's row of the count matrix from the lower bounds of the R - 1
// inner splitters in its sorted keys: out = [A tuples to rank 0 .. R-1 | B
// tuples to rank 0 .. R-1] (cut q of a side = lb[q-1]; cut 0 = 0, cut R = n).
__global__ void k_cut_counts(const uint64_t *__restrict__ lb, unsigned R, size_t na, size_t nb,
                             uint64_t *__restrict__ out) {
    const unsigned q = blockIdx.x * 256 + threadIdx.x;
    if (q >= R) return;
    const uint64_t *la = lb, *lbb = lb + (R - 1);
    const uint64_t a0 = q ? la[q - 1] : 0, a1 = q + 1 < R ? la[q] : na;
    const uint64_t b0 = q ? lbb[q - 1] : 0, b1 = q + 1 < R ? lbb[q] : nb;
    out[q] = a1 - a0;
    out[R + q] = b1 - b0;
}

// A member's row of the count matrix in ONE launch (round 6): the R - 1
// inner splitters by value (no host-to-device copy), one wave per 64-ary
// lower-bound search of a side's sorted keys, then the cuts' differences.
constexpr unsigned kCutMaxR = 64;
struct Splitters {
    uint64_t v[kCutMaxR - 1];
};
__global__ __launch_bounds__(1024) void k_member_cuts(const uint64_t *__restrict__ ka, size_t na,
                                                      const uint64_t *__restrict__ kb, size_t nb, Splitters sp,
                                                      unsigned R, uint64_t *__restrict__ row) {
    __shared__ uint64_t s_lb[2][kCutMaxR];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    for (unsigned j = (unsigned)wv; j < 2 * (R - 1); j += (unsigned)nwv) {
        const int side = j >= R - 1;
        const unsigned q = side ? j - (R - 1) : j;
        const uint64_t *k = side ? kb : ka;
        const uint64_t pr = sp.v[q];
        size_t lo = 0, hi = side ? nb : na;           // first index with k >= pr lies in [lo, hi]
        while (lo < hi) {
            const size_t span = hi - lo;
            const size_t x = lo + span * (size_t)lane / 64;
            const uint64_t ge = __ballot(k[x] >= pr);
            if (ge == 0) {
                lo += span * 63 / 64 + 1;
            } else {
                const int t = __ffsll((long long)ge) - 1;
                hi = lo + span * (size_t)t / 64;
                if (t > 0) lo += span * (size_t)(t - 1) / 64 + 1;
            }
        }
        if (lane == 0) s_lb[side][q] = lo;
    }
    __syncthreads();
    for (unsigned q = threadIdx.x; q < R; q += blockDim.x) {
        const uint64_t a0 = q ? s_lb[0][q - 1] : 0, a1 = q + 1 < R ? s_lb[0][q] : na;
        const uint64_t b0 = q ? s_lb[1][q - 1] : 0, b1 = q + 1 < R ? s_lb[1][q] : nb;
        row[q] = a1 - a0;
        row[R + q] = b1 - b0;
    }
}

// Host-side phase timing of the distributed set merge (diagnostic build,
// "shard.host_timing" = 1): microseconds since the call started, per phase,
// to stderr -- where the host waits or works while the GPU idles.
struct PhaseClock {
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    char buf[512];
    int len = 0;
    void mark(const char *what) {
        if (!g_shard_host_timing) return;
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        len += snprintf(buf + len, sizeof buf - (size_t)len, " %s %.0f", what, us);
        if (len >= (int)sizeof buf) len = (int)sizeof buf - 1;
    }
    ~PhaseClock() {
        if (g_shard_host_timing && len) fprintf(stderr, "[shard] us:%s\n", buf);
    }
};

int shard_set_merge_local(crdt_comm *c, bool lww, const crdt_tuples *a, const size_t *na, const crdt_tuples *b,
                          const size_t *nb, const crdt_tuples *out, size_t cap, size_t *n_out,
                          uint64_t *const *n_dev, int gather) {
    if (!valid(c) || !a || !na || !b || !nb || !out || (!n_out && !n_dev)) return CRDT_E_INVAL;
    if (n_dev && gather) return CRDT_E_INVAL;
    const size_t M = c->m.size(), R = (size_t)c->nranks, S = kSamplesPerSide;
    for (size_t i = 0; i < M; ++i) {
        if ((na[i] && !a[i].key) || (nb[i] && !b[i].key)) return CRDT_E_INVAL;
        if (n_dev && !n_dev[i]) return CRDT_E_INVAL;
    }
    auto set_merge = [&](crdt_ctx *x, const crdt_tuples &A, size_t n_a, const crdt_tuples &B, size_t n_b,
                         const crdt_tuples &O, uint64_t *count) {
        return lww ? crdt_lww_merge(x, &A, n_a, &B, n_b, const_cast<crdt_tuples *>(&O), count)
                   : crdt_orset_merge(x, &A, n_a, &B, n_b, const_cast<crdt_tuples *>(&O), count);
    };
    if (R == 1 && !g_shard_exchange_always && cap >= na[0] + nb[0]) {   // one rank owns every key: no exchange
        auto &mb = c->m[0];
        int rc = scratch_reserve(mb, head_bytes(R));
        if (rc) return rc;
        uint64_t *count = n_dev ? n_dev[0] : (uint64_t *)mb.scratch;
        rc = set_merge(mb.ctx, a[0], na[0], b[0], nb[0], out[0], count);
        if (rc || n_dev) return rc;                      // (counts stay on the device: no synchronisation)
        uint64_t h = 0;
        rc = read_member0(c, count, &h, 1);
        if (rc) return rc;
        n_out[0] = h;
        return check_devices(c);
    }
    // control block after the head: [samples R x blk | count matrix R x 2R | probes R | bounds 2R]
    const size_t blk = 2 + 2 * S;
    struct Ctrl {
        uint64_t *smp, *cnt, *prb, *lb;
    };
    const size_t ctrl_bytes = head_bytes(R) + Carve::round(R * blk * 8) + Carve::round(2 * R * R * 8) +
                              Carve::round(R * 8) + Carve::round(2 * R * 8) + 1024;
    auto carve_ctrl = [&](crdt_comm::Member &mb, Ctrl *k) {
        Carve w(mb.scratch);
        (void)w.take<uint64_t>(R + 2);                   // the head
        k->smp = w.take<uint64_t>(R * blk);
        k->cnt = w.take<uint64_t>(2 * R * R);
        k->prb = w.take<uint64_t>(R);
        k->lb = w.take<uint64_t>(2 * R);
        return w.used;
    };
    std::vector<Ctrl> ct(M);
    for (size_t i = 0; i < M; ++i) {
        int rc = scratch_reserve(c->m[i], ctrl_bytes);
        if (rc) return rc;
        carve_ctrl(c->m[i], &ct[i]);
    }
    PhaseClock pc;
    // 1. samples + sizes, all-gathered; every rank derives the same splitters (read-back 1)
    std::vector<const void *> snd(M);
    std::vector<void *> rcv(M);
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        int rc = bind(mb.ctx);
        if (rc) return rc;
        uint64_t *mine = ct[i].smp + (c->rank0 + i) * blk;
        k_sample_block<<<(unsigned)((S + 255) / 256), 256, 0, mb.ctx->stream>>>(a[i].key, na[i], b[i].key, nb[i],
                                                                               (unsigned)S, mine);
        rc = check_launch(mb.ctx);
        if (rc) return rc;
        snd[i] = mine;
        rcv[i] = ct[i].smp;
    }
    int rc = c->x->allgather(c, snd.data(), rcv.data(), blk * 8);
    if (rc) return rc;
    pc.mark("ag1");
    std::vector<uint64_t> h_smp(R * blk);
    rc = read_member0(c, ct[0].smp, h_smp.data(), R * blk);
    if (rc) return rc;
    pc.mark("rb1");
    const std::vector<uint64_t> spl = weighted_splitters(h_smp.data(), R, S);
    pc.mark("spl");
    // 2. each member's cuts (device lower_bound of the inner splitters) -> its
    //    row of the count matrix on the device; the matrix all-gathered (read-back 2)
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        rc = bind(mb.ctx);
        if (rc) return rc;
        uint64_t *row = ct[i].cnt + (c->rank0 + i) * 2 * R;
        if (R <= kCutMaxR) {                             // splitters by value, one launch
            Splitters sp{};
            for (size_t q = 1; q < R; ++q) sp.v[q - 1] = spl[q];
            const unsigned th = (unsigned)std::min<size_t>(1024, std::max<size_t>(64, 64 * 2 * (R - 1)));
            k_member_cuts<<<1, th, 0, mb.ctx->stream>>>(a[i].key, na[i], b[i].key, nb[i], sp, (unsigned)R, row);
        } else {
            hipError_t e = hipMemcpyAsync(ct[i].prb, spl.data() + 1, (R - 1) * 8, hipMemcpyHostToDevice,
                                          mb.ctx->stream);
            if (e != hipSuccess) return hip_fail(mb.ctx, e);
            rc = crdt_u64_lower_bound(mb.ctx, a[i].key, na[i], ct[i].prb, R - 1, ct[i].lb);
            if (!rc) rc = crdt_u64_lower_bound(mb.ctx, b[i].key, nb[i], ct[i].prb, R - 1, ct[i].lb + (R - 1));
            if (rc) return rc;
            k_cut_counts<<<(unsigned)((R + 255) / 256), 256, 0, mb.ctx->stream>>>(ct[i].lb, (unsigned)R, na[i], nb[i],
                                                                                 row);
        }
        rc = check_launch(mb.ctx);
        if (rc) return rc;
        snd[i] = row;
        rcv[i] = ct[i].cnt;
    }
    pc.mark("cuts");
    rc = c->x->allgather(c, snd.data(), rcv.data(), 2 * R * 8);
    if (rc) return rc;
    pc.mark("ag2");
    std::vector<uint64_t> mat(2 * R * R);               // row p = rank p's [A counts | B counts] by destination
    rc = read_member0(c, ct[0].cnt, mat.data(), mat.size());
    if (rc) return rc;
    pc.mark("rb2");
    std::vector<size_t> tot_a(M, 0), tot_b(M, 0);
    for (size_t i = 0; i < M; ++i) {
        const size_t g = (size_t)c->rank0 + i;
        size_t sa = 0, sb = 0;
        for (size_t q = 0; q < R; ++q) sa += mat[g * 2 * R + q], sb += mat[g * 2 * R + R + q];
        if (sa != na[i] || sb != nb[i]) return CRDT_E_COMM;    // the matrix must describe the member's own sides
        for (size_t p = 0; p < R; ++p) tot_a[i] += mat[p * 2 * R + g], tot_b[i] += mat[p * 2 * R + R + g];
    }
    // 3. per member two tuple arenas of n = received tuples after the control
    //    block (the scratch is re-carved: nothing in it is needed any more)
    std::vector<crdt_tuples> ar0(M), ar1(M);
    std::vector<bool> direct(M);
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        const size_t n = tot_a[i] + tot_b[i];
        direct[i] = !gather && cap >= n;                 // the final merge writes straight into out[i]
        if (n_dev && !direct[i]) return CRDT_E_RANGE;
        const size_t ab = Carve::round(n * 8 + 8) * 2 + Carve::round(n * 4 + 4) + Carve::round(n + 1);
        rc = scratch_reserve(mb, ctrl_bytes + 2 * ab + 2048);
        if (rc) return rc;
        Carve w(mb.scratch);
        w.used = carve_ctrl(mb, &ct[i]);
        for (crdt_tuples *t : {&ar0[i], &ar1[i]}) {
            t->key = w.take<uint64_t>(n + 1);
            t->ts = w.take<uint64_t>(n + 1);
            t->rep = w.take<uint32_t>(n + 1);
            t->tomb = w.take<uint8_t>(n + 1);
        }
    }
    pc.mark("arenas");
    // 4. the exchange: every field of both sides to its key-range owner, ONE
    //    point-to-point group; arena 0 receives A's runs then B's, rank order
    {
        std::vector<XP2P> ops;
        const size_t esz[4] = {8, 8, 4, 1};
        for (size_t i = 0; i < M; ++i) {
            const size_t g = (size_t)c->rank0 + i;
            size_t so[2] = {0, 0}, ro[2] = {0, tot_a[i]};
            for (size_t q = 0; q < R; ++q)
                for (int side = 0; side < 2; ++side) {
                    const crdt_tuples &src = side ? b[i] : a[i];
                    const char *fs[4] = {(const char *)src.key, (const char *)src.ts, (const char *)src.rep,
                                         (const char *)src.tomb};
                    char *fd[4] = {(char *)ar0[i].key, (char *)ar0[i].ts, (char *)ar0[i].rep, (char *)ar0[i].tomb};
                    const size_t sn = mat[g * 2 * R + side * R + q], rn = mat[q * 2 * R + side * R + g];
                    for (int f = 0; f < 4; ++f) {
                        if (sn) ops.push_back(XP2P{i, (int)q, true, fs[f] + so[side] * esz[f], nullptr, sn * esz[f]});
                        if (rn) ops.push_back(XP2P{i, (int)q, false, nullptr, fd[f] + ro[side] * esz[f], rn * esz[f]});
                    }
                    so[side] += sn;
                    ro[side] += rn;
                }
        }
        rc = c->x->p2p(c, ops);
        if (rc) return rc;
    }
    pc.mark("xchg");
    // 5. per member: each side's R runs merged stably in rank order (lower rank
    //    left) by a tree of crdt_tuples_merge levels -- every length known on
    //    the host, so no read-back -- then ONE set merge of the two sides.
    //    Both sides have R runs, so they finish in the same arena.
    std::vector<crdt_tuples> fin(M);
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        rc = bind(mb.ctx);
        if (rc) return rc;
        struct Run {
            size_t off, n;
        };
        std::vector<Run> ru[2];
        size_t o = 0;
        for (int side = 0; side < 2; ++side)
            for (size_t p = 0; p < R; ++p) {
                const size_t n = mat[p * 2 * R + side * R + (size_t)c->rank0 + i];
                ru[side].push_back(Run{o, n});
                o += n;
            }
        auto view = [&](int arena, size_t off) {
            const crdt_tuples &t = arena ? ar1[i] : ar0[i];
            return crdt_tuples{t.key + off, t.ts + off, t.rep + off, t.tomb + off};
        };
        int cur = 0;
        while (ru[0].size() > 1) {                       // one level of both sides: one batched launch pair
            std::vector<MergePairArg> lvl;
            for (int side = 0; side < 2; ++side) {
                std::vector<Run> nx;
                for (size_t k = 0; k < ru[side].size(); k += 2) {
                    const Run x = ru[side][k], y = k + 1 < ru[side].size() ? ru[side][k + 1] : Run{x.off + x.n, 0};
                    lvl.push_back(MergePairArg{view(cur, x.off), x.n, view(cur, y.off), y.n, view(1 - cur, x.off)});
                    nx.push_back(Run{x.off, x.n + y.n});
                }
                ru[side].swap(nx);
            }
            rc = tuples_merge_stable_batch(mb.ctx, lvl);
            if (rc) return rc;
            cur = 1 - cur;
        }
        uint64_t *count = n_dev ? n_dev[i] : (uint64_t *)mb.scratch;   // (the head's word 0)
        fin[i] = direct[i] ? out[i] : view(1 - cur, 0);
        crdt_tuples A = view(cur, 0), B = view(cur, tot_a[i]);
        rc = set_merge(mb.ctx, A, tot_a[i], B, tot_b[i], fin[i], count);
        if (rc) return rc;
    }
    pc.mark("merges");
    if (n_dev) return CRDT_OK;                           // enqueued; counts on the device
    // 6. the whole merged state on every member, or each member's own range
    if (gather) {
        size_t tot = 0;
        rc = allgather_v_head(c, fin.data(), out, cap, &tot);
        if (rc) return rc;
        pc.mark("gather");
        for (size_t i = 0; i < M; ++i) n_out[i] = tot;
        rc = check_devices(c);
        pc.mark("done");
        return rc;
    }
    for (size_t i = 0; i < M; ++i) {                   // every member's count read in flight at once
        auto &mb = c->m[i];
        rc = bind(mb.ctx);
        if (!rc) rc = ctx_read_begin(mb.ctx, mb.scratch, 8);
        if (rc) return rc;
    }
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        rc = bind(mb.ctx);
        const void *hw = nullptr;
        if (!rc) rc = ctx_read_end(mb.ctx, &hw);
        if (rc) return rc;
        const uint64_t h = *(const uint64_t *)hw;
        n_out[i] = h;
        hipError_t e = hipSuccess;
        if (direct[i] || !h) continue;
        if (h > cap) return CRDT_E_RANGE;
        e = hipMemcpyAsync(out[i].key, fin[i].key, h * 8, hipMemcpyDeviceToDevice, mb.ctx->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(out[i].ts, fin[i].ts, h * 8, hipMemcpyDeviceToDevice, mb.ctx->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(out[i].rep, fin[i].rep, h * 4, hipMemcpyDeviceToDevice, mb.ctx->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(out[i].tomb, fin[i].tomb, h, hipMemcpyDeviceToDevice, mb.ctx->stream);
        if (e != hipSuccess) return hip_fail(mb.ctx, e);
    }
    return check_devices(c);
}

}  // namespace

// Keyed-set merge of a DISTRIBUTED population: member i
// holds only its own tuples a[i] (na[i]) and b[i] (nb[i]), each sorted by
// (key, ts, rep).  The population's A is the stable merge of every rank's A
// in rank order (likewise B); the result is crdt_lww_merge / crdt_orset_merge
// of those -- computed by key-range owners: weighted sample splitters (one
// all-gather), the count matrix (one all-gather), every rank's tuples sent to
// their owner (one point-to-point group), the owner's rank-order stable
// merges of the received runs and one set merge.  gather != 0: every
// member's out[i] receives the whole merged state and n_out[i] its length;
// gather == 0: out[i] / n_out[i] = the member's own key range of it (ranges
// ascend with rank).  Synchronises.
extern "C" int crdt_shard_lww_merge_local(crdt_comm *c, const crdt_tuples *a, const size_t *na, const crdt_tuples *b,
                                          const size_t *nb, const crdt_tuples *out, size_t cap, size_t *n_out,
                                          int gather) {
    return shard_set_merge_local(c, true, a, na, b, nb, out, cap, n_out, nullptr, gather);
}

extern "C" int crdt_shard_orset_merge_local(crdt_comm *c, const crdt_tuples *a, const size_t *na,
                                            const crdt_tuples *b, const size_t *nb, const crdt_tuples *out,
                                            size_t cap, size_t *n_out, int gather) {
    return shard_set_merge_local(c, false, a, na, b, nb, out, cap, n_out, nullptr, gather);
}

// The same without the trailing synchronisation: each member's own key range
// (gather == 0) into out[i], its length written to n_out_dev[i] (a device
// word on the member's GPU) on the member stream.  Planning still reads back
// the samples and the count matrix when nranks > 1; with one rank nothing is
// read back.  CRDT_E_RANGE if cap is below the member's received tuples.
extern "C" int crdt_shard_lww_merge_local_dev(crdt_comm *c, const crdt_tuples *a, const size_t *na,
                                              const crdt_tuples *b, const size_t *nb, const crdt_tuples *out,
                                              size_t cap, uint64_t *const *n_out_dev) {
    return shard_set_merge_local(c, true, a, na, b, nb, out, cap, nullptr, n_out_dev, 0);
}

extern "C" int crdt_shard_orset_merge_local_dev(crdt_comm *c, const crdt_tuples *a, const size_t *na,
                                                const crdt_tuples *b, const size_t *nb, const crdt_tuples *out,
                                                size_t cap, uint64_t *const *n_out_dev) {
    return shard_set_merge_local(c, false, a, na, b, nb, out, cap, nullptr, n_out_dev, 0);
}
