// shard.hip -- replica-sharded joins over RCCL (SURVEY §8(a) a9, §8(b) crdt_shard_*, §8(e)).
//
// The reference has no collective: its replicas exchange whole logs by HTTP
// pull gossip (main.go:226-258).  Here a replica population is sharded over
// the GPUs of one node and the cross-shard join is one RCCL collective over
// xGMI:
//   * counters / clocks: every member folds its contiguous row shard
//     (crdt_gcounter_fold), then ONE ncclAllReduce(ncclUint64, ncclMax) of the
//     `nodes`-long fold -- RCCL's unsigned 64-bit max is exactly the join, so
//     no order map is needed on this path;
//   * divergent full-state copies (config E2): ncclAllReduce(ncclUint64,
//     ncclMax) in place;
//   * keyed sets: members own disjoint ordered key ranges, merge them locally
//     and an all-gather-v (counts by ncclAllGather, then one grouped
//     ncclBroadcast per root and field) concatenates the outputs in rank order,
//     which is already the globally sorted merged state (a key's LWW / OR-Set
//     output depends only on that key's tuples);
//   * keyed sets of a DISTRIBUTED population (every rank holds only its own
//     tuples, crdt_shard_*_merge_local): sampled splitters (one ncclAllGather),
//     each rank's tuples sent to their key-range owner (grouped ncclSend /
//     ncclRecv, an all-to-all-v), the owner's merge of the received runs,
//     then the all-gather-v above;
//   * RefMerge of one batch whose logs are split by ts range over the ranks
//     (crdt_shard_refmerge): all-reduce(max) of max(L), the local merge, then
//     integer all-reduces of the replay accumulators (main.go:35-100).
// A communicator has one or more LOCAL members (device + crdt_ctx + ncclComm):
// crdt_shard_comm_create drives every listed GPU from one process
// (ncclCommInitAll, grouped calls); crdt_shard_comm_init_rank makes one member
// per process (ncclCommInitRank; torchrun-style one process per GPU).
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <vector>

#include "common.hpp"

static_assert(sizeof(ncclUniqueId) == CRDT_SHARD_ID_BYTES, "RCCL unique id size");

struct crdt_comm {
    struct Member {
        int device = 0;
        crdt_ctx *ctx = nullptr;
        bool own_ctx = false;
        ncclComm_t nccl = nullptr;
        void *scratch = nullptr;      // per-member device scratch (set-merge slices, counts)
        size_t scratch_bytes = 0;
    };
    int nranks = 0;                   // ranks over all processes
    int rank0 = 0;                    // global rank of local member 0
    int last_nccl_error = 0;
    std::vector<Member> m;
};

namespace crdt {
namespace {

int nccl_fail(crdt_comm *c, ncclResult_t r) {
    if (c) c->last_nccl_error = (int)r;
    return CRDT_E_COMM;
}

// Grow a member's scratch to `bytes` (the member's stream is drained first).
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

int check_devices(crdt_comm *c) {
    for (auto &mb : c->m) {
        uint32_t flags = 0;
        int rc = crdt_ctx_device_status(mb.ctx, &flags, 1);
        if (rc) return rc;
        if (flags) return CRDT_E_DEVICE;
    }
    return CRDT_OK;
}

bool valid(const crdt_comm *c) { return c && !c->m.empty(); }

// out[i] = key[i * n / per], i < per (evenly spaced sample of a sorted key array).
__global__ void k_sample_keys(const uint64_t *__restrict__ key, size_t n, unsigned per, uint64_t *__restrict__ out) {
    const unsigned i = blockIdx.x * 256 + threadIdx.x;
    if (i < per) out[i] = key[(size_t)((unsigned __int128)i * n / per)];
}

constexpr unsigned kSamplesPerSide = 256;
constexpr uint64_t kKeyEnd = ~0ULL;       // splitter sentinel: "to the end of the key space"

template <class T> ncclDataType_t nccl_type();
template <> ncclDataType_t nccl_type<uint64_t>() { return ncclUint64; }
template <> ncclDataType_t nccl_type<uint32_t>() { return ncclUint32; }
template <> ncclDataType_t nccl_type<uint8_t>() { return ncclUint8; }

}  // namespace
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

extern "C" int crdt_shard_comm_create(const int *devices, int n, crdt_comm **out) {
    if (!out) return CRDT_E_INVAL;
    *out = nullptr;
    if (!devices || n <= 0) return CRDT_E_INVAL;
    crdt_comm *c = new (std::nothrow) crdt_comm();
    if (!c) return CRDT_E_NOMEM;
    c->nranks = n;
    c->m.resize(n);
    int rc = CRDT_OK;
    for (int i = 0; i < n && rc == CRDT_OK; ++i) {
        for (int j = 0; j < i; ++j)
            if (devices[j] == devices[i]) rc = CRDT_E_INVAL;      // RCCL: one rank per GPU
        if (rc) break;
        void *s = nullptr;
        rc = crdt_stream_create(devices[i], &s);
        if (rc) break;
        rc = crdt_ctx_create(devices[i], s, &c->m[i].ctx);
        if (rc) {
            (void)crdt_stream_destroy(s);
            break;
        }
        c->m[i].ctx->own_stream = true;                        // destroyed with the context
        c->m[i].own_ctx = true;
        c->m[i].device = devices[i];
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

extern "C" int crdt_shard_comm_init_rank(crdt_ctx *ctx, const void *id, int nranks, int rank, crdt_comm **out) {
    if (!out) return CRDT_E_INVAL;
    *out = nullptr;
    if (!ctx || !id || nranks <= 0 || rank < 0 || rank >= nranks) return CRDT_E_INVAL;
    int rc = bind(ctx);
    if (rc) return rc;
    crdt_comm *c = new (std::nothrow) crdt_comm();
    if (!c) return CRDT_E_NOMEM;
    c->nranks = nranks;
    c->rank0 = rank;
    c->m.resize(1);
    c->m[0].device = ctx->device;
    c->m[0].ctx = ctx;                      // borrowed: the caller's context and stream
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
// every rank's buf: ncclAllReduce(ncclUint64, ncclMax), in place.
extern "C" int crdt_shard_allreduce_max_u64(crdt_comm *c, uint64_t *const *buf, size_t n) {
    if (!valid(c) || !buf) return CRDT_E_INVAL;
    if (n == 0) return CRDT_OK;
    for (size_t i = 0; i < c->m.size(); ++i)
        if (!buf[i]) return CRDT_E_INVAL;
    ncclResult_t r = ncclGroupStart();
    for (size_t i = 0; i < c->m.size() && r == ncclSuccess; ++i)
        r = ncclAllReduce(buf[i], buf[i], n, ncclUint64, ncclMax, c->m[i].nccl, c->m[i].ctx->stream);
    ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess) return nccl_fail(c, r);
    if (r2 != ncclSuccess) return nccl_fail(c, r2);
    return CRDT_OK;
}

extern "C" int crdt_shard_allreduce(crdt_comm *c, void *const *buf, size_t n, int type, int op) {
    if (!valid(c) || !buf) return CRDT_E_INVAL;
    ncclDataType_t t;
    switch (type) {
        case CRDT_SHARD_I64: t = ncclInt64; break;
        case CRDT_SHARD_U64: t = ncclUint64; break;
        case CRDT_SHARD_U32: t = ncclUint32; break;
        case CRDT_SHARD_I32: t = ncclInt32; break;
        default: return CRDT_E_INVAL;
    }
    ncclRedOp_t o;
    switch (op) {
        case CRDT_SHARD_SUM: o = ncclSum; break;
        case CRDT_SHARD_MAX: o = ncclMax; break;
        default: return CRDT_E_INVAL;
    }
    if (n == 0) return CRDT_OK;
    for (size_t i = 0; i < c->m.size(); ++i)
        if (!buf[i]) return CRDT_E_INVAL;
    ncclResult_t r = ncclGroupStart();
    for (size_t i = 0; i < c->m.size() && r == ncclSuccess; ++i)
        r = ncclAllReduce(buf[i], buf[i], n, t, o, c->m[i].nccl, c->m[i].ctx->stream);
    ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess) return nccl_fail(c, r);
    if (r2 != ncclSuccess) return nccl_fail(c, r2);
    return CRDT_OK;
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

// Keyed-set all-gather-v: member i contributes local[i] (n_local[i] tuples on
// its device); every member's out[i] receives the concatenation in global
// rank order.  *n_total (host) = the gathered length.  Synchronises once (the
// counts travel by ncclAllGather and are read back before the broadcasts).
extern "C" int crdt_shard_set_allgather_v(crdt_comm *c, const crdt_tuples *local, const size_t *n_local,
                                          const crdt_tuples *out, size_t cap, size_t *n_total) {
    if (!valid(c) || !local || !n_local || !out || !n_total) return CRDT_E_INVAL;
    const size_t M = c->m.size(), R = (size_t)c->nranks;
    // counts: member scratch = [my count | R gathered counts]
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        int rc = scratch_reserve(mb, (R + 1) * sizeof(uint64_t));
        if (rc) return rc;
        rc = bind(mb.ctx);
        if (rc) return rc;
        uint64_t v = n_local[i];
        hipError_t e = hipMemcpyAsync(mb.scratch, &v, sizeof v, hipMemcpyHostToDevice, mb.ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(mb.ctx->stream);    // v is a stack value
        if (e != hipSuccess) return hip_fail(mb.ctx, e);
    }
    ncclResult_t r = ncclGroupStart();
    for (size_t i = 0; i < M && r == ncclSuccess; ++i) {
        uint64_t *s = (uint64_t *)c->m[i].scratch;
        r = ncclAllGather(s, s + 1, 1, ncclUint64, c->m[i].nccl, c->m[i].ctx->stream);
    }
    ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess) return nccl_fail(c, r);
    if (r2 != ncclSuccess) return nccl_fail(c, r2);
    std::vector<uint64_t> cnt(R), off(R + 1, 0);
    {
        auto &mb = c->m[0];
        int rc = bind(mb.ctx);
        if (rc) return rc;
        hipError_t e = hipMemcpyAsync(cnt.data(), (uint64_t *)mb.scratch + 1, R * sizeof(uint64_t),
                                      hipMemcpyDeviceToHost, mb.ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(mb.ctx->stream);
        if (e != hipSuccess) return hip_fail(mb.ctx, e);
    }
    for (size_t q = 0; q < R; ++q) off[q + 1] = off[q] + cnt[q];
    *n_total = off[R];
    if (off[R] > cap) return CRDT_E_RANGE;
    for (size_t i = 0; i < M; ++i) {
        if (cnt[c->rank0 + i] != n_local[i]) return CRDT_E_COMM;
        if (off[R] && (!out[i].key || !out[i].ts || !out[i].rep || !out[i].tomb)) return CRDT_E_INVAL;
        if (n_local[i] && (!local[i].key || !local[i].ts || !local[i].rep || !local[i].tomb)) return CRDT_E_INVAL;
    }
    r = ncclGroupStart();
    for (size_t q = 0; q < R && r == ncclSuccess; ++q) {
        if (cnt[q] == 0) continue;
        for (size_t i = 0; i < M && r == ncclSuccess; ++i) {
            const bool root = (size_t)c->rank0 + i == q;
            const crdt_tuples &src = root ? local[i] : out[i];   // sendbuff is read on the root only
            const crdt_tuples &dst = out[i];
            ncclComm_t cm = c->m[i].nccl;
            hipStream_t st = c->m[i].ctx->stream;
            const size_t n = cnt[q], o = off[q];
            r = ncclBroadcast(src.key, dst.key + o, n, ncclUint64, (int)q, cm, st);
            if (r == ncclSuccess) r = ncclBroadcast(src.ts, dst.ts + o, n, ncclUint64, (int)q, cm, st);
            if (r == ncclSuccess) r = ncclBroadcast(src.rep, dst.rep + o, n, ncclUint32, (int)q, cm, st);
            if (r == ncclSuccess) r = ncclBroadcast(src.tomb, dst.tomb + o, n, ncclUint8, (int)q, cm, st);
        }
    }
    r2 = ncclGroupEnd();
    if (r != ncclSuccess) return nccl_fail(c, r);
    if (r2 != ncclSuccess) return nccl_fail(c, r2);
    return CRDT_OK;
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
        if (!h.empty()) {
            hipError_t e = hipMemcpyAsync(h.data(), smp, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost,
                                          mb.ctx->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(mb.ctx->stream);
            if (e != hipSuccess) return hip_fail(mb.ctx, e);
            std::sort(h.begin(), h.end());
            for (size_t q = 1; q < R; ++q) spl[q] = h[q * h.size() / R];
        }
    }
    // 2. each member's key range [spl[g], spl[g+1]) of both inputs (lower_bound
    //    of the splitters on the member's own copy), merged on its device into
    //    its scratch
    std::vector<crdt_tuples> loc(M);
    std::vector<size_t> nloc(M, 0);
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
        // scratch: [count | key | ts | rep | tomb] of capacity cap_i
        const size_t need = Carve::round(8) + Carve::round(cap_i * 8) * 2 + Carve::round(cap_i * 4) +
                            Carve::round(cap_i) + 1024;
        int rc = scratch_reserve(mb, need);
        if (rc) return rc;
        Carve w(mb.scratch);
        uint64_t *count = w.take<uint64_t>(1);
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
    // 3. local counts (the device status read synchronises each member)
    int rc = check_devices(c);
    if (rc) return rc;
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        uint64_t v = 0;
        hipError_t e = hipMemcpyAsync(&v, mb.scratch, sizeof v, hipMemcpyDeviceToHost, mb.ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(mb.ctx->stream);
        if (e != hipSuccess) return hip_fail(mb.ctx, e);
        nloc[i] = v;
    }
    // 4. all-gather-v in rank order
    return crdt_shard_set_allgather_v(c, loc.data(), nloc.data(), out, cap, n_out);
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
// steps of crdt_amd/shard.py's sharded_refmerge, on the library's own RCCL
// communicator and member streams, no host synchronisation:
//   1. crdt_refmerge_local_maxl, ncclAllReduce(ncclInt64, ncclMax): the GLOBAL
//      max(L) of every replica (remote ts at or above it are dropped, main.go:49);
//   2. crdt_refmerge_batch_ex with that max: the member's slice of the new
//      Diff (slices concatenate in rank order) and its unreduced accumulators;
//   3. the key's max-ts holder across ranks: ncclMax of shard << 40 | rank
//      (crdt_refmerge_acc_rank), ncclSum of the owner's string id, ncclSum of
//      the wrapped sums (int64 two's complement: main.go:95) and of the
//      parsable counts;
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
    auto allreduce = [&](auto ptr_of, size_t n, ncclDataType_t t, ncclRedOp_t op) -> int {
        ncclResult_t r = ncclGroupStart();
        for (size_t i = 0; i < M && r == ncclSuccess; ++i)
            r = ncclAllReduce(ptr_of(i), ptr_of(i), n, t, op, c->m[i].nccl, c->m[i].ctx->stream);
        ncclResult_t r2 = ncclGroupEnd();
        if (r != ncclSuccess) return nccl_fail(c, r);
        if (r2 != ncclSuccess) return nccl_fail(c, r2);
        return CRDT_OK;
    };
    // 1. the global max(L) per replica
    int rc = each([&](size_t i, crdt_ctx *x) { return crdt_refmerge_local_maxl(x, &in[i], bf[i].maxl); });
    if (!rc) rc = allreduce([&](size_t i) { return (void *)bf[i].maxl; }, P, ncclInt64, ncclMax);
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
        if (!rc) rc = allreduce([&](size_t i) { return (void *)bf[i].cmax; }, ns, ncclInt64, ncclMax);
        if (!rc) rc = each([&](size_t i, crdt_ctx *x) {
            return crdt_refmerge_acc_owner_str(x, &bf[i].acc, ns, bf[i].c, bf[i].cmax, bf[i].v);
        });
        if (!rc) rc = allreduce([&](size_t i) { return (void *)bf[i].v; }, ns, ncclInt64, ncclSum);
        if (!rc) rc = allreduce([&](size_t i) { return (void *)bf[i].acc.sum; }, ns, ncclInt64, ncclSum);
        if (!rc) rc = allreduce([&](size_t i) { return (void *)bf[i].acc.npar; }, ns, ncclUint32, ncclSum);
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
// in rank order (grouped ncclSend / ncclRecv, enqueued on the member streams).
extern "C" int crdt_shard_alltoallv(crdt_comm *c, const void *const *send, const size_t *send_counts,
                                    void *const *recv, const size_t *recv_counts, size_t elem_size) {
    if (!valid(c) || !send || !send_counts || !recv || !recv_counts || elem_size == 0) return CRDT_E_INVAL;
    const size_t M = c->m.size(), R = (size_t)c->nranks;
    for (size_t i = 0; i < M; ++i) {
        size_t ns = 0, nr = 0;
        for (size_t q = 0; q < R; ++q) ns += send_counts[i * R + q], nr += recv_counts[i * R + q];
        if ((ns && !send[i]) || (nr && !recv[i])) return CRDT_E_INVAL;
    }
    ncclResult_t r = ncclGroupStart();
    for (size_t i = 0; i < M && r == ncclSuccess; ++i) {
        const char *sb = (const char *)send[i];
        char *rb = (char *)recv[i];
        size_t so = 0, ro = 0;
        for (size_t q = 0; q < R && r == ncclSuccess; ++q) {
            const size_t sn = send_counts[i * R + q] * elem_size, rn = recv_counts[i * R + q] * elem_size;
            if (sn) r = ncclSend(sb + so, sn, ncclUint8, (int)q, c->m[i].nccl, c->m[i].ctx->stream);
            if (r == ncclSuccess && rn) r = ncclRecv(rb + ro, rn, ncclUint8, (int)q, c->m[i].nccl, c->m[i].ctx->stream);
            so += sn;
            ro += rn;
        }
    }
    ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess) return nccl_fail(c, r);
    if (r2 != ncclSuccess) return nccl_fail(c, r2);
    return CRDT_OK;
}

namespace {

// Splitters of a distributed key population from per-rank samples: block p
// of the gathered samples = [n_a, n_b, S keys of A, S keys of B] (a side
// with n > 0 sampled at i * n / S, each sample weighing n; an empty side's
// samples weigh 0).  Inner splitter q = the first sample key (in key order)
// at which the cumulative weight reaches q / R of the total.  Rank r owns
// keys [spl[r], spl[r+1]); crdt_amd/shard.py weighted_splitters is the same rule.
std::vector<uint64_t> weighted_splitters(const uint64_t *blocks, size_t R, size_t S) {
    std::vector<std::pair<uint64_t, uint64_t>> e;       // (key, weight)
    e.reserve(2 * S * R);
    for (size_t p = 0; p < R; ++p) {
        const uint64_t *b = blocks + p * (2 + 2 * S);
        for (int side = 0; side < 2; ++side)
            if (b[side])
                for (size_t i = 0; i < S; ++i) e.emplace_back(b[2 + side * S + i], b[side]);
    }
    std::sort(e.begin(), e.end(), [](const auto &x, const auto &y) { return x.first < y.first; });
    unsigned __int128 W = 0;
    for (auto &x : e) W += x.second;
    std::vector<uint64_t> spl(R + 1, 0);
    spl[R] = kKeyEnd;
    unsigned __int128 cum = 0;
    size_t k = 0;
    for (size_t q = 1; q < R; ++q) {
        const unsigned __int128 target = (unsigned __int128)q * W;
        while (k < e.size() && (cum + e[k].second) * R < target) cum += e[k++].second;
        spl[q] = W == 0 ? 0 : (k < e.size() ? e[k].first : e.back().first);
    }
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

struct Run {
    int arena;           // 0 / 1
    size_t off, n;
};

int shard_set_merge_local(crdt_comm *c, bool lww, const crdt_tuples *a, const size_t *na, const crdt_tuples *b,
                          const size_t *nb, const crdt_tuples *out, size_t cap, size_t *n_out, int gather) {
    if (!valid(c) || !a || !na || !b || !nb || !out || !n_out) return CRDT_E_INVAL;
    const size_t M = c->m.size(), R = (size_t)c->nranks, S = kSamplesPerSide;
    for (size_t i = 0; i < M; ++i)
        if ((na[i] && !a[i].key) || (nb[i] && !b[i].key)) return CRDT_E_INVAL;
    if (R == 1 && !g_shard_exchange_always && cap >= na[0] + nb[0]) {   // one rank owns every key: no exchange
        auto &mb = c->m[0];
        int rc = scratch_reserve(mb, 64);
        if (rc) return rc;
        uint64_t *count = (uint64_t *)mb.scratch;
        rc = lww ? crdt_lww_merge(mb.ctx, &a[0], na[0], &b[0], nb[0], const_cast<crdt_tuples *>(&out[0]), count)
                 : crdt_orset_merge(mb.ctx, &a[0], na[0], &b[0], nb[0], const_cast<crdt_tuples *>(&out[0]), count);
        if (rc) return rc;
        uint64_t h = 0;
        hipError_t e = hipMemcpyAsync(&h, count, 8, hipMemcpyDeviceToHost, mb.ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(mb.ctx->stream);
        if (e != hipSuccess) return hip_fail(mb.ctx, e);
        n_out[0] = h;
        return check_devices(c);
    }
    // scratch layout: [ctrl: samples R x (2 + 2S) | counts 2R x R | bounds] then two tuple arenas
    const size_t blk = 2 + 2 * S;
    const size_t ctrl = Carve::round((R + 2) * 8) + Carve::round(R * blk * 8) + Carve::round(2 * R * R * 8) +
                        Carve::round(4 * (R + 1) * 8) + Carve::round(4 * R * 8 + 8) + 4096;
    for (size_t i = 0; i < M; ++i) {
        int rc = scratch_reserve(c->m[i], ctrl);
        if (rc) return rc;
    }
    auto carve_ctrl = [&](crdt_comm::Member &mb, uint64_t **smp, uint64_t **cnt, uint64_t **bnd, uint64_t **mc) {
        Carve w(mb.scratch);
        (void)w.take<uint64_t>(R + 2);                   // (crdt_shard_set_allgather_v's counts)
        *smp = w.take<uint64_t>(R * blk);
        *cnt = w.take<uint64_t>(2 * R * R);
        *bnd = w.take<uint64_t>(4 * (R + 1));
        *mc = w.take<uint64_t>(4 * R + 1);
        return w.used;
    };
    // 1. samples + sizes, all-gathered; every rank derives the same splitters
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        uint64_t *smp, *cnt, *bnd, *mc;
        carve_ctrl(mb, &smp, &cnt, &bnd, &mc);
        int rc = bind(mb.ctx);
        if (rc) return rc;
        k_sample_block<<<(unsigned)((S + 255) / 256), 256, 0, mb.ctx->stream>>>(a[i].key, na[i], b[i].key, nb[i],
                                                                               (unsigned)S, smp + (c->rank0 + i) * blk);
        rc = check_launch(mb.ctx);
        if (rc) return rc;
    }
    ncclResult_t r = ncclGroupStart();
    for (size_t i = 0; i < M && r == ncclSuccess; ++i) {
        auto &mb = c->m[i];
        uint64_t *smp, *cnt, *bnd, *mc;
        carve_ctrl(mb, &smp, &cnt, &bnd, &mc);
        uint64_t *mine = smp + (c->rank0 + i) * blk;
        r = ncclAllGather(mine, smp, blk, ncclUint64, mb.nccl, mb.ctx->stream);
    }
    ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess) return nccl_fail(c, r);
    if (r2 != ncclSuccess) return nccl_fail(c, r2);
    std::vector<uint64_t> h_smp(R * blk);
    {
        auto &mb = c->m[0];
        uint64_t *smp, *cnt, *bnd, *mc;
        carve_ctrl(mb, &smp, &cnt, &bnd, &mc);
        int rc = bind(mb.ctx);
        if (rc) return rc;
        hipError_t e = hipMemcpyAsync(h_smp.data(), smp, R * blk * 8, hipMemcpyDeviceToHost, mb.ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(mb.ctx->stream);
        if (e != hipSuccess) return hip_fail(mb.ctx, e);
    }
    const std::vector<uint64_t> spl = weighted_splitters(h_smp.data(), R, S);
    // 2. each member's send ranges: lower_bound of the inner splitters in its keys
    std::vector<size_t> sa(M * R), sb(M * R), ra(M * R), rb(M * R);
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        uint64_t *smp, *cnt, *bnd, *mc;
        carve_ctrl(mb, &smp, &cnt, &bnd, &mc);
        int rc = bind(mb.ctx);
        if (rc) return rc;
        std::vector<uint64_t> hb(2 * (R + 1), 0);
        if (R > 1) {
            hipError_t e = hipMemcpyAsync(bnd, spl.data() + 1, (R - 1) * 8, hipMemcpyHostToDevice, mb.ctx->stream);
            if (e != hipSuccess) return hip_fail(mb.ctx, e);
            if (na[i]) rc = crdt_u64_lower_bound(mb.ctx, a[i].key, na[i], bnd, R - 1, bnd + R);
            if (!rc && nb[i]) rc = crdt_u64_lower_bound(mb.ctx, b[i].key, nb[i], bnd, R - 1, bnd + 2 * R);
            if (rc) return rc;
            e = hipMemcpyAsync(hb.data(), bnd + R, 2 * R * 8, hipMemcpyDeviceToHost, mb.ctx->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(mb.ctx->stream);
            if (e != hipSuccess) return hip_fail(mb.ctx, e);
        }
        // cuts of A: 0, lb(spl[1]) .. lb(spl[R-1]), na (lower_bound of 0 is 0, of the end na)
        std::vector<uint64_t> cutA(R + 1), cutB(R + 1);
        cutA[0] = cutB[0] = 0;
        for (size_t q = 1; q < R; ++q) cutA[q] = na[i] ? hb[q - 1] : 0, cutB[q] = nb[i] ? hb[R + q - 1] : 0;
        cutA[R] = na[i];
        cutB[R] = nb[i];
        for (size_t q = 0; q < R; ++q) {
            sa[i * R + q] = cutA[q + 1] - cutA[q];
            sb[i * R + q] = cutB[q + 1] - cutB[q];
        }
    }
    // 3. the count matrix, all-gathered: block p = rank p's [send A counts | send B counts]
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        uint64_t *smp, *cnt, *bnd, *mc;
        carve_ctrl(mb, &smp, &cnt, &bnd, &mc);
        int rc = bind(mb.ctx);
        if (rc) return rc;
        std::vector<uint64_t> h(2 * R);
        for (size_t q = 0; q < R; ++q) h[q] = sa[i * R + q], h[R + q] = sb[i * R + q];
        hipError_t e = hipMemcpyAsync(cnt + (c->rank0 + i) * 2 * R, h.data(), 2 * R * 8, hipMemcpyHostToDevice,
                                      mb.ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(mb.ctx->stream);     // h is a local
        if (e != hipSuccess) return hip_fail(mb.ctx, e);
    }
    r = ncclGroupStart();
    for (size_t i = 0; i < M && r == ncclSuccess; ++i) {
        auto &mb = c->m[i];
        uint64_t *smp, *cnt, *bnd, *mc;
        carve_ctrl(mb, &smp, &cnt, &bnd, &mc);
        uint64_t *mine = cnt + (c->rank0 + i) * 2 * R;
        r = ncclAllGather(mine, cnt, 2 * R, ncclUint64, mb.nccl, mb.ctx->stream);
    }
    r2 = ncclGroupEnd();
    if (r != ncclSuccess) return nccl_fail(c, r);
    if (r2 != ncclSuccess) return nccl_fail(c, r2);
    std::vector<size_t> tot_a(M, 0), tot_b(M, 0);
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        uint64_t *smp, *cnt, *bnd, *mc;
        carve_ctrl(mb, &smp, &cnt, &bnd, &mc);
        int rc = bind(mb.ctx);
        if (rc) return rc;
        std::vector<uint64_t> h(2 * R * R);
        hipError_t e = hipMemcpyAsync(h.data(), cnt, 2 * R * R * 8, hipMemcpyDeviceToHost, mb.ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(mb.ctx->stream);
        if (e != hipSuccess) return hip_fail(mb.ctx, e);
        const size_t g = (size_t)c->rank0 + i;
        for (size_t p = 0; p < R; ++p) {
            ra[i * R + p] = h[p * 2 * R + g];
            rb[i * R + p] = h[p * 2 * R + R + g];
            tot_a[i] += ra[i * R + p];
            tot_b[i] += rb[i * R + p];
        }
    }
    // 4. the exchange into arena 0 (A's runs, then B's, in rank order), field by field
    std::vector<crdt_tuples> ar0(M), ar1(M);
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        const size_t n = tot_a[i] + tot_b[i] + 1;
        const size_t need = ctrl + 2 * (Carve::round(n * 8) * 2 + Carve::round(n * 4) + Carve::round(n)) + 4096;
        int rc = scratch_reserve(mb, need);
        if (rc) return rc;
        uint64_t *smp, *cnt, *bnd, *mc;
        Carve w(mb.scratch);
        w.used = carve_ctrl(mb, &smp, &cnt, &bnd, &mc);
        for (crdt_tuples *t : {&ar0[i], &ar1[i]}) {
            t->key = w.take<uint64_t>(n);
            t->ts = w.take<uint64_t>(n);
            t->rep = w.take<uint32_t>(n);
            t->tomb = w.take<uint8_t>(n);
        }
    }
    {
        std::vector<const void *> snd(M);
        std::vector<void *> rcv(M);
        const size_t esz[4] = {8, 8, 4, 1};
        for (int side = 0; side < 2; ++side)
            for (int f = 0; f < 4; ++f) {
                for (size_t i = 0; i < M; ++i) {
                    const crdt_tuples &src = side ? b[i] : a[i];
                    const void *fs[4] = {src.key, src.ts, src.rep, src.tomb};
                    void *fd[4] = {ar0[i].key, ar0[i].ts, ar0[i].rep, ar0[i].tomb};
                    snd[i] = fs[f];
                    rcv[i] = (char *)fd[f] + (side ? tot_a[i] * esz[f] : 0);
                }
                int rc = crdt_shard_alltoallv(c, snd.data(), side ? sb.data() : sa.data(), rcv.data(),
                                              side ? rb.data() : ra.data(), esz[f]);
                if (rc) return rc;
            }
    }
    // 5. per member, a tree of merges over the received runs: A's runs in
    //    rank order pairwise (lower rank left: the stable rank-order merge),
    //    B's likewise, then merge(A, B); levels alternate between the arenas
    std::vector<size_t> final_n(M, 0);
    std::vector<crdt_tuples> fin(M);
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        int rc = bind(mb.ctx);
        if (rc) return rc;
        uint64_t *smp, *cnt, *bnd, *mc;
        carve_ctrl(mb, &smp, &cnt, &bnd, &mc);
        std::vector<Run> ruA, ruB;
        size_t o = 0;
        for (size_t p = 0; p < R; ++p) ruA.push_back(Run{0, o, ra[i * R + p]}), o += ra[i * R + p];
        for (size_t p = 0; p < R; ++p) ruB.push_back(Run{0, o, rb[i * R + p]}), o += rb[i * R + p];
        auto view = [&](const Run &x) {
            const crdt_tuples &ar = x.arena ? ar1[i] : ar0[i];
            return crdt_tuples{ar.key + x.off, ar.ts + x.off, ar.rep + x.off, ar.tomb + x.off};
        };
        auto merge = [&](const Run &x, const Run &y, int dst, uint64_t *count) -> int {
            crdt_tuples tx = view(x), ty = view(y);
            const crdt_tuples &ad = dst ? ar1[i] : ar0[i];
            crdt_tuples to{ad.key + x.off, ad.ts + x.off, ad.rep + x.off, ad.tomb + x.off};   // (x, y adjacent)
            return lww ? crdt_lww_merge(mb.ctx, &tx, x.n, &ty, y.n, &to, count)
                       : crdt_orset_merge(mb.ctx, &tx, x.n, &ty, y.n, &to, count);
        };
        int level_arena = 0;
        bool final_done = false;
        while (!final_done) {
            // one level: pairs of A runs, pairs of B runs; the last level merges A with B
            std::vector<std::pair<Run, Run>> jobs;
            std::vector<int> job_side;
            const bool last = ruA.size() == 1 && ruB.size() == 1;
            if (last) {
                jobs.emplace_back(ruA[0], ruB[0]);
                job_side.push_back(2);
            } else {
                for (int side = 0; side < 2; ++side) {
                    auto &ru = side ? ruB : ruA;
                    for (size_t k = 0; k < ru.size(); k += 2) {
                        Run y = k + 1 < ru.size() ? ru[k + 1] : Run{ru[k].arena, ru[k].off + ru[k].n, 0};
                        jobs.emplace_back(ru[k], y);
                        job_side.push_back(side);
                    }
                }
            }
            const int dst = 1 - level_arena;
            for (size_t j = 0; j < jobs.size(); ++j) {
                rc = merge(jobs[j].first, jobs[j].second, dst, mc + j);
                if (rc) return rc;
            }
            std::vector<uint64_t> hn(jobs.size());
            hipError_t e = hipMemcpyAsync(hn.data(), mc, jobs.size() * 8, hipMemcpyDeviceToHost, mb.ctx->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(mb.ctx->stream);
            if (e != hipSuccess) return hip_fail(mb.ctx, e);
            std::vector<Run> na_, nb_;
            for (size_t j = 0; j < jobs.size(); ++j) {
                const Run nr{dst, jobs[j].first.off, hn[j]};
                if (job_side[j] == 2) {
                    fin[i] = view(nr);
                    final_n[i] = hn[j];
                    final_done = true;
                } else {
                    (job_side[j] ? nb_ : na_).push_back(nr);
                }
            }
            if (!final_done) {
                ruA.swap(na_);
                ruB.swap(nb_);
            }
            level_arena = dst;
        }
    }
    int rc = check_devices(c);
    if (rc) return rc;
    // 6. the whole merged state on every member, or each member's own range
    if (gather) {
        size_t tot = 0;
        rc = crdt_shard_set_allgather_v(c, fin.data(), final_n.data(), out, cap, &tot);
        if (rc) return rc;
        for (size_t i = 0; i < M; ++i) n_out[i] = tot;
        return CRDT_OK;
    }
    for (size_t i = 0; i < M; ++i) {
        auto &mb = c->m[i];
        n_out[i] = final_n[i];
        if (final_n[i] > cap) return CRDT_E_RANGE;
        if (!final_n[i]) continue;
        rc = bind(mb.ctx);
        if (rc) return rc;
        const size_t n = final_n[i];
        hipError_t e = hipMemcpyAsync(out[i].key, fin[i].key, n * 8, hipMemcpyDeviceToDevice, mb.ctx->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(out[i].ts, fin[i].ts, n * 8, hipMemcpyDeviceToDevice, mb.ctx->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(out[i].rep, fin[i].rep, n * 4, hipMemcpyDeviceToDevice, mb.ctx->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(out[i].tomb, fin[i].tomb, n, hipMemcpyDeviceToDevice, mb.ctx->stream);
        if (e != hipSuccess) return hip_fail(mb.ctx, e);
    }
    return CRDT_OK;
}

}  // namespace

// Keyed-set merge of a DISTRIBUTED population: member i
// holds only its own tuples a[i] (na[i]) and b[i] (nb[i]), each sorted by
// (key, ts, rep).  The population's A is the stable merge of every rank's A
// in rank order (likewise B); the result is crdt_lww_merge / crdt_orset_merge
// of those -- computed by key-range owners: weighted sample splitters (one
// all-gather), every rank's tuples sent to their owner (all-to-all-v), the
// owner merges the received runs (rank-order pairwise merges, then A with
// B).  gather != 0: every member's out[i] receives the whole merged state and
// n_out[i] its length; gather == 0: out[i] / n_out[i] = the member's own key
// range of it (ranges ascend with rank).  Synchronises.
extern "C" int crdt_shard_lww_merge_local(crdt_comm *c, const crdt_tuples *a, const size_t *na, const crdt_tuples *b,
                                          const size_t *nb, const crdt_tuples *out, size_t cap, size_t *n_out,
                                          int gather) {
    return shard_set_merge_local(c, true, a, na, b, nb, out, cap, n_out, gather);
}

extern "C" int crdt_shard_orset_merge_local(crdt_comm *c, const crdt_tuples *a, const size_t *na,
                                            const crdt_tuples *b, const size_t *nb, const crdt_tuples *out,
                                            size_t cap, size_t *n_out, int gather) {
    return shard_set_merge_local(c, false, a, na, b, nb, out, cap, n_out, gather);
}
