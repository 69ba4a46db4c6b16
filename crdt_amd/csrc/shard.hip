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
//     output depends only on that key's tuples).
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
