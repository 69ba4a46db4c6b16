// population.hip -- anti-entropy rounds of a device-resident replica
// population behind the C-ABI (crdt_population_*).
//
// The reference runs one gossip goroutine per Server (main.go:226-261): each
// round it picks a friend (main.go:230), GETs the friend's whole Diff
// (main.go:159), decodes it into RemoteDiff (main.go:245-256) and merges
// (main.go:257); a failed GET skips the round (main.go:234-239).  Here P
// replicas' Diffs live in HBM in the crdt_refmerge_in layout and one call runs
// a synchronous round for all of them (one legal schedule of the reference's
// asynchronous goroutines):
//   * crdt_population_round: every peer on this population.  The merge reads
//     each peer's Diff where it lies (crdt_refmerge_batch_pull: R = an entry
//     range of the population's own arrays, the pulled key slots re-based by
//     a per-replica delta) and writes the next Diffs with their kv pairs; the
//     per-replica arrays are computed on the host from the entry / pair
//     counts it keeps and uploaded in one copy; one read-back at the end
//     refreshes the counts.
//   * crdt_population_round_sharded: replicas partitioned over a
//     communicator's ranks (crdt_shard_range).  Every rank derives from the
//     round's global draw which Diffs every rank pulls, the per-replica counts
//     are all-gathered (one collective, one read-back), each rank packs the
//     Diffs of its replicas that others pull and ONE point-to-point group moves
//     them to their pullers (entries, per-entry pair counts, pairs -- the
//     pairs straight into the puller's kv arena behind its own); the merge
//     then reads the received Diffs in place like the local round.
// Dead peers (-1) skip the round: no merge for that replica -- its Diff stays
// (an empty pull inserts nothing) and its CurrentState is put back after the
// batched merge rebuilt it (main.go:76).  A device-side failure leaves the
// population as it was (outputs go to spare buffers, swapped in on success).
//
// Key slots: local replica i's key k is slot i * K + k.
#include <string.h>

#include <algorithm>
#include <functional>
#include <new>
#include <vector>

#include "common.hpp"

struct crdt_population {
    struct Diff {
        uint64_t *off = nullptr;      // [P + 1]
        int64_t *ts = nullptr;        // [cap_e]
        uint8_t *origin = nullptr;
        int64_t *src = nullptr;
        uint64_t *kv_off = nullptr;   // [cap_e + 1]
        uint32_t *kv_key = nullptr;   // [cap_kv]: the Diff's pairs, room behind them
        uint32_t *kv_val = nullptr;
        size_t cap_e = 0, cap_kv = 0;
    };
    crdt_ctx *ctx = nullptr;
    uint32_t P = 0, K = 0;
    uint64_t first = 0;
    Diff d[2];
    int cur = 0;
    size_t n_e = 0, n_kv = 0;                  // the current Diffs' entries / kv pairs
    std::vector<uint64_t> cnt, kvcnt;          // per replica (host)
    std::vector<uint64_t> pcnt, pkvcnt;        // ... of the Diffs before the last round (crdt_population_undo)
    size_t p_n_e = 0, p_n_kv = 0;
    bool can_undo = false;
    // every entry of the current Diffs holds exactly one kv pair (the
    // reference's load generator writes one key per command, main.go:282):
    // rounds then size the kv output from entry counts alone
    // (refmerge_batch_pull_one_pair).  Exact or false: set at creation from
    // the host arrays, kept by local rounds and by wire rounds whose decode
    // counted no other entry, cleared by multi-pair commands and sharded
    // rounds.
    bool one_pair = false, p_one_pair = false;
    uint8_t *str_bytes = nullptr;
    uint64_t *str_off = nullptr;
    uint64_t n_str = 0;
    // after the first wire round: the value table the pulls were interned
    // into IS the string arena (its first n_str strings checked equal to the
    // population's own, which are then freed); refreshed before every use
    crdt_strtab *vtab = nullptr;
    uint8_t *st_kind[2] = {nullptr, nullptr};  // CurrentState, double-buffered with the Diffs
    uint32_t *st_str[2] = {nullptr, nullptr};
    int64_t *st_sum[2] = {nullptr, nullptr};
    void *pin = nullptr;                       // pinned staging (uploads, the end-of-round read-back; coherent)
    void *pin_d = nullptr;                     // ... its device address (kernels read / write it directly)
    size_t pin_bytes = 0;
    uint64_t *hflag = nullptr, *hflag_d = nullptr;   // the round's completion word (coherent host memory)
    uint64_t seq = 0;                          // ... the value the current round's last kernel writes
    void *dsm = nullptr;                       // device staging of the per-replica arrays
    size_t dsm_bytes = 0;
    void *xb = nullptr;                        // sharded rounds: send and import buffers
    size_t xb_bytes = 0;
    void *dscr = nullptr;                      // wire rounds: the device decode's own scratch (the merge
    size_t dscr_bytes = 0;                     //   runs behind its claim pass in ctx->ws)
};

namespace crdt {
namespace {

int dev_free(crdt_ctx *ctx, void **p) {
    if (*p) {
        hipError_t e = hipFree(*p);
        *p = nullptr;
        if (e != hipSuccess) return hip_fail(ctx, e);
    }
    return CRDT_OK;
}

// (re)allocate *p to hold `bytes` (contents lost; the stream is drained first)
int dev_grow(crdt_ctx *ctx, void **p, size_t *cap, size_t bytes) {
    if (bytes <= *cap && *p) return CRDT_OK;
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
    int rc = dev_free(ctx, p);
    if (rc) return rc;
    *cap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
    e = hipMalloc(p, want);
    if (e != hipSuccess) {
        *p = nullptr;
        return hip_fail(ctx, e);
    }
    *cap = want;
    return CRDT_OK;
}

int pin_grow(crdt_population *pop, size_t bytes) {
    if (bytes <= pop->pin_bytes) return CRDT_OK;
    hipError_t e = hipStreamSynchronize(pop->ctx->stream);
    if (e != hipSuccess) return hip_fail(pop->ctx, e);
    if (pop->pin) (void)hipHostFree(pop->pin);
    pop->pin = pop->pin_d = nullptr;
    pop->pin_bytes = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
    // coherent (fine-grained): the round's staging kernel reads it and the
    // bounds kernel writes it directly, no copy-engine transfers
    e = hipHostMalloc(&pop->pin, want, hipHostMallocCoherent | hipHostMallocMapped);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&pop->pin_d, pop->pin, 0);
    if (e != hipSuccess) {
        if (pop->pin) (void)hipHostFree(pop->pin);
        pop->pin = pop->pin_d = nullptr;
        return hip_fail(pop->ctx, e);
    }
    pop->pin_bytes = want;
    if (!pop->hflag) {
        void *f = nullptr, *fd = nullptr;
        e = hipHostMalloc(&f, 64, hipHostMallocCoherent | hipHostMallocMapped);
        if (e == hipSuccess) e = hipHostGetDevicePointer(&fd, f, 0);
        if (e != hipSuccess) {
            if (f) (void)hipHostFree(f);
            return hip_fail(pop->ctx, e);
        }
        pop->hflag = (uint64_t *)f;
        pop->hflag_d = (uint64_t *)fd;
        *(volatile uint64_t *)pop->hflag = 0;
    }
    return CRDT_OK;
}

template <class T>
int alloc(crdt_ctx *ctx, T **p, size_t n) {
    hipError_t e = hipMalloc((void **)p, std::max<size_t>(n, 1) * sizeof(T));
    if (e != hipSuccess) {
        *p = nullptr;
        return hip_fail(ctx, e);
    }
    return CRDT_OK;
}

void diff_free(crdt_population::Diff &d) {
    for (void *p : {(void *)d.off, (void *)d.ts, (void *)d.origin, (void *)d.src, (void *)d.kv_off, (void *)d.kv_key,
                    (void *)d.kv_val})
        if (p) (void)hipFree(p);
    d = crdt_population::Diff{};
}

// Diff d with room for cap_e entries and cap_kv pairs (contents kept when
// keep != 0: the current Diff growing its kv arena for a sharded import).
int diff_reserve(crdt_population *pop, crdt_population::Diff &d, size_t cap_e, size_t cap_kv, bool keep) {
    crdt_ctx *ctx = pop->ctx;
    int rc = CRDT_OK;
    if (!d.off) rc = alloc(ctx, &d.off, pop->P + 1);
    if (!rc && (cap_e > d.cap_e || !d.ts)) {
        if (keep && d.ts) return CRDT_E_INVAL;           // (only the kv arena grows in place)
        hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e);
        for (void *p : {(void *)d.ts, (void *)d.origin, (void *)d.src, (void *)d.kv_off})
            if (p) (void)hipFree(p);
        d.ts = nullptr, d.origin = nullptr, d.src = nullptr, d.kv_off = nullptr, d.cap_e = 0;
        const size_t c = cap_e + cap_e / 4 + 1024;
        rc = alloc(ctx, &d.ts, c);
        if (!rc) rc = alloc(ctx, &d.origin, c);
        if (!rc) rc = alloc(ctx, &d.src, c);
        if (!rc) rc = alloc(ctx, &d.kv_off, c + 1);
        if (!rc) d.cap_e = c;
    }
    if (!rc && (cap_kv > d.cap_kv || !d.kv_key)) {
        hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e);
        const size_t c = 2 * cap_kv + 1024;               // room behind the pairs for a round's pulls
        uint32_t *k = nullptr, *v = nullptr;
        rc = alloc(ctx, &k, c);
        if (!rc) rc = alloc(ctx, &v, c);
        if (!rc && keep && pop->n_kv) {
            e = hipMemcpyAsync(k, d.kv_key, pop->n_kv * 4, hipMemcpyDeviceToDevice, ctx->stream);
            if (e == hipSuccess) e = hipMemcpyAsync(v, d.kv_val, pop->n_kv * 4, hipMemcpyDeviceToDevice, ctx->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
            if (e != hipSuccess) rc = hip_fail(ctx, e);
        }
        if (rc) {
            if (k) (void)hipFree(k);
            if (v) (void)hipFree(v);
            return rc;
        }
        if (d.kv_key) (void)hipFree(d.kv_key);
        if (d.kv_val) (void)hipFree(d.kv_val);
        d.kv_key = k, d.kv_val = v, d.cap_kv = c;
    }
    return rc;
}

// the value arena of a population that adopted a table (the table may have
// grown or moved since the last call)
void pop_arena(crdt_population *pop) {
    if (!pop->vtab) return;
    uint64_t nb = 0;
    const uint8_t *b = nullptr;
    const uint64_t *o = nullptr;
    (void)crdt_strtab_info(pop->vtab, &pop->n_str, &nb, &b, &o);
    pop->str_bytes = const_cast<uint8_t *>(b);           // (borrowed: freed by the table)
    pop->str_off = const_cast<uint64_t *>(o);
}

// CurrentState of the replicas whose peer was dead: put back after the batched merge rebuilt it
__global__ void k_pop_keep_state(const uint8_t *__restrict__ skip, uint32_t K, uint64_t n_slots,
                                 const uint8_t *__restrict__ ok, const uint32_t *__restrict__ os,
                                 const int64_t *__restrict__ ov, uint8_t *__restrict__ nk, uint32_t *__restrict__ ns,
                                 int64_t *__restrict__ nv) {
    for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < n_slots; s += (uint64_t)gridDim.x * 256)
        if (skip[s / K]) {
            nk[s] = ok[s];
            ns[s] = os[s];
            nv[s] = ov[s];
        }
}

// The end-of-round read-back: out[p] = off[p], out[P + 1 + p] = kv_off[off[p]]
// (p <= P), out[2P + 2] = the device status word (the flags a pass raised).
__global__ void k_pop_bounds(const uint64_t *__restrict__ off, const uint64_t *__restrict__ kv_off, uint32_t P,
                             const uint32_t *__restrict__ status, uint64_t *__restrict__ out) {
    for (uint32_t p = blockIdx.x * 256 + threadIdx.x; p <= P; p += gridDim.x * 256) {
        const uint64_t o = off[p];
        out[p] = o;
        out[P + 1 + p] = kv_off[o];
        if (p == 0) out[2 * P + 2] = *status;
    }
}


// pop.direct (default 1): the round's per-replica arrays come from the
// coherent pinned staging by this kernel (no copy-engine upload, no separate
// status copy), and the end-of-round bounds go straight into it with a
// completion word the host polls (no copy-engine read-back, no interrupt
// wake-up).  Measured in DESIGN.md §5.8.
__global__ void k_pop_stage(const uint64_t *__restrict__ src, uint64_t *__restrict__ dst, size_t nw,
                            const uint32_t *__restrict__ status, uint64_t *__restrict__ snap) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nw; i += (size_t)gridDim.x * 256) dst[i] = src[i];
    if (blockIdx.x == 0 && threadIdx.x == 0) *snap = *status;
}

// as k_pop_bounds, one workgroup, into host memory; then the completion word
// (system-scope release: the bounds are visible to the host before it)
__global__ __launch_bounds__(1024) void k_pop_bounds_host(const uint64_t *__restrict__ off,
                                                         const uint64_t *__restrict__ kv_off, uint32_t P,
                                                         const uint32_t *__restrict__ status,
                                                         const uint64_t *__restrict__ snap, uint64_t *__restrict__ out,
                                                         uint64_t *__restrict__ flag, uint64_t seq) {
    for (uint32_t p = threadIdx.x; p <= P; p += 1024) {
        const uint64_t o = off[p];
        out[p] = o;
        out[P + 1 + p] = kv_off[o];
    }
    if (threadIdx.x == 0) {
        out[2 * P + 2] = *status;
        out[2 * P + 3] = *snap;
    }
    // every writing wave releases its own stores at system scope before the
    // barrier: thread 0's release below covers only its own wave
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Per-replica arrays of one round's merge, one carve in both the device
// staging and the pinned staging: r_off P | r_end P | bounds 2P + 4 (u64) |
// slot delta P (u32) | skip P (u8).  bounds: the next Diffs' entry offsets
// (P + 1), kv offsets at the replica bounds (P + 1), the status word after
// the round's passes and (slot 2P + 3) as it was before them.
struct RoundArrays {
    uint64_t *r_off, *r_end, *bounds;
    uint32_t *sd;
    uint8_t *skip;
};
size_t round_bytes(uint32_t P) {
    return Carve::round(P * 8) * 2 + Carve::round((2 * P + 4) * 8) + Carve::round(P * 4) + Carve::round(P) + 1024;
}
RoundArrays carve_round(void *base, uint32_t P) {
    Carve w(base);
    RoundArrays a;
    a.r_off = w.take<uint64_t>(P);
    a.r_end = w.take<uint64_t>(P);
    a.bounds = w.take<uint64_t>(2 * P + 4);
    a.sd = w.take<uint32_t>(P);
    a.skip = w.take<uint8_t>(P);
    return a;
}

struct HostRound {
    std::vector<uint64_t> r_off, r_end;
    std::vector<uint32_t> sd;
    std::vector<uint8_t> skip;
    size_t n_r = 0, n_rkv = 0;                 // pulled entries / pairs over all replicas (with repeats)
    bool any_skip = false;
    explicit HostRound(uint32_t P) : r_off(P, 0), r_end(P, 0), sd(P, 0), skip(P, 0) {}
};

// The round's per-replica arrays: staged in pinned memory, one upload; the
// status word snapshot taken behind it (flags raised before this round are
// not this round's).
int upload_round(crdt_population *pop, const HostRound &h, RoundArrays *a) {
    const uint32_t P = pop->P;
    const size_t rb = round_bytes(P);
    int rc = dev_grow(pop->ctx, &pop->dsm, &pop->dsm_bytes, rb);
    if (!rc) rc = pin_grow(pop, rb);
    if (rc) return rc;
    *a = carve_round(pop->dsm, P);
    const RoundArrays hp = carve_round(pop->pin, P);
    if (P) {
        memcpy(hp.r_off, h.r_off.data(), P * 8);
        memcpy(hp.r_end, h.r_end.data(), P * 8);
        memcpy(hp.sd, h.sd.data(), P * 4);
        memcpy(hp.skip, h.skip.data(), P);
    }
    const size_t upto = (size_t)((char *)(hp.skip + P) - (char *)pop->pin);
    if (g_pop_direct) {
        const size_t nw = (upto + 7) / 8;                // (the carve's slack covers the rounding)
        k_pop_stage<<<grid_for(nw, 256, 64), 256, 0, pop->ctx->stream>>>((const uint64_t *)pop->pin_d,
                                                                          (uint64_t *)pop->dsm, nw,
                                                                          pop->ctx->dev_status, a->bounds + 2 * P + 3);
        return check_launch(pop->ctx);
    }
    hipError_t e = hipMemcpyAsync(pop->dsm, pop->pin, upto, hipMemcpyHostToDevice, pop->ctx->stream);
    // (8 bytes from the 256-byte status allocation: only the low word is compared)
    if (e == hipSuccess)
        e = hipMemcpyAsync(a->bounds + 2 * P + 3, pop->ctx->dev_status, 8, hipMemcpyDeviceToDevice, pop->ctx->stream);
    return e == hipSuccess ? CRDT_OK : hip_fail(pop->ctx, e);
}

// Enqueue the round's merge: R = [r_off, r_end) ranges of r_ts / r_kv, the
// pairs in the current Diff's kv arena (n_arena pairs: the Diff's own, plus
// any imported behind them); the next Diffs and CurrentState into the spare
// buffers; the read-back of their bounds into the pinned staging (async).
int pop_merge(crdt_population *pop, const RoundArrays &a, const HostRound &h, const int64_t *r_ts,
              const uint64_t *r_kv, size_t n_arena, bool one_pair = false) {
    crdt_ctx *ctx = pop->ctx;
    const uint32_t P = pop->P;
    if (P == 0) return CRDT_OK;                          // (a rank that holds no replica merges nothing)
    pop_arena(pop);
    pop->can_undo = false;                               // the spare buffers (the undo snapshot) are rewritten below
    auto &nd = pop->d[1 - pop->cur];
    int rc = diff_reserve(pop, nd, pop->n_e + h.n_r, pop->n_kv + h.n_rkv, false);
    if (rc) return rc;
    auto &cd = pop->d[pop->cur];
    const int so = pop->cur, sn = 1 - pop->cur;
    crdt_refmerge_in in{};
    in.replicas = P;
    in.n_slots = (uint32_t)((uint64_t)P * pop->K);
    in.n_l = pop->n_e;
    in.n_r = h.n_r;
    in.n_kv = n_arena;
    in.n_str = pop->n_str;
    in.l_off = cd.off;
    in.l_ts = cd.ts;
    in.l_origin = cd.origin;
    in.l_kv = cd.kv_off;
    in.r_off = a.r_off;
    in.r_ts = r_ts;
    in.r_kv = r_kv;
    in.kv_key = cd.kv_key;
    in.kv_val = cd.kv_val;
    in.str_bytes = pop->str_bytes;
    in.str_off = pop->str_off;
    const crdt_refmerge_out out{nd.off, nd.ts, nd.origin, nd.src, pop->st_kind[sn], pop->st_str[sn],
                                pop->st_sum[sn]};
    const crdt_refmerge_pull pull{a.r_end, a.sd};
    const crdt_refmerge_kv_out kv{nd.kv_off, nd.kv_key, nd.kv_val, nd.cap_kv};
    rc = one_pair ? refmerge_batch_pull_one_pair(ctx, &in, &out, &pull, &kv)
                  : crdt_refmerge_batch_pull(ctx, &in, &out, &pull, &kv);
    if (rc) return rc;
    const uint64_t ns = (uint64_t)P * pop->K;
    if (h.any_skip && ns)
        k_pop_keep_state<<<grid_for(ns, 256, (unsigned)ctx->num_cus * 4), 256, 0, ctx->stream>>>(
            a.skip, pop->K, ns, pop->st_kind[so], pop->st_str[so], pop->st_sum[so], pop->st_kind[sn],
            pop->st_str[sn], pop->st_sum[sn]);
    if (g_pop_direct) {
        pop->seq += 1;
        k_pop_bounds_host<<<1, 1024, 0, ctx->stream>>>(nd.off, nd.kv_off, P, ctx->dev_status, a.bounds + 2 * P + 3,
                                                       carve_round(pop->pin_d, P).bounds, pop->hflag_d, pop->seq);
        return check_launch(ctx);
    }
    k_pop_bounds<<<grid_for(P + 1, 256, 64), 256, 0, ctx->stream>>>(nd.off, nd.kv_off, P, ctx->dev_status,
                                                                      a.bounds);
    rc = check_launch(ctx);
    if (rc) return rc;
    uint64_t *hb = carve_round(pop->pin, P).bounds;
    hipError_t e = hipMemcpyAsync(hb, a.bounds, (2 * P + 4) * 8, hipMemcpyDeviceToHost, ctx->stream);
    return e == hipSuccess ? CRDT_OK : hip_fail(ctx, e);
}

// After the stream has drained: the next Diffs / CurrentState are swapped in
// and the host counts refreshed from the read-back -- unless a pass of this
// round raised a device flag, which leaves the population as it was.
// (split in two so that a sharded round can check every member before it
// swaps any in: all or nothing across the communicator's members)
int pop_commit_check(crdt_population *pop) {
    const uint32_t P = pop->P;
    if (g_pop_direct && P) {
        // poll the completion word; the stream's own state ends the wait when
        // the round's kernels did not all run (a launch or device error)
        const volatile uint64_t *f = pop->hflag;
        while (*f != pop->seq) {
            const hipError_t q = hipStreamQuery(pop->ctx->stream);
            if (q == hipErrorNotReady) continue;
            if (*f == pop->seq) break;
            return hip_fail(pop->ctx, q == hipSuccess ? hipErrorUnknown : q);
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
    } else {
        hipError_t e = hipStreamSynchronize(pop->ctx->stream);
        if (e != hipSuccess) return hip_fail(pop->ctx, e);
    }
    if (P == 0) return CRDT_OK;
    const uint64_t *hb = carve_round(pop->pin, P).bounds;
    const uint32_t after = (uint32_t)hb[2 * P + 2], before = (uint32_t)hb[2 * P + 3];
    return (after & ~before) ? CRDT_E_DEVICE : CRDT_OK;
}

void pop_commit_apply(crdt_population *pop) {
    const uint32_t P = pop->P;
    if (P == 0) return;
    const uint64_t *hb = carve_round(pop->pin, P).bounds;
    pop->pcnt.swap(pop->cnt);
    pop->pkvcnt.swap(pop->kvcnt);
    pop->cnt.resize(P);
    pop->kvcnt.resize(P);
    pop->p_n_e = pop->n_e;
    pop->p_n_kv = pop->n_kv;
    pop->p_one_pair = pop->one_pair;
    pop->can_undo = true;
    for (uint32_t p = 0; p < P; ++p) {
        pop->cnt[p] = hb[p + 1] - hb[p];
        pop->kvcnt[p] = hb[P + 2 + p] - hb[P + 1 + p];
    }
    pop->n_e = hb[P];
    pop->n_kv = hb[2 * P + 1];
    pop->cur = 1 - pop->cur;
}

int pop_commit(crdt_population *pop) {
    const int rc = pop_commit_check(pop);
    if (rc == CRDT_OK) pop_commit_apply(pop);
    return rc;
}

bool pop_valid(const crdt_population *p) { return p && p->ctx && p->d[p->cur].off; }


// host prefix of a count vector
std::vector<uint64_t> prefix(const std::vector<uint64_t> &c) {
    std::vector<uint64_t> o(c.size() + 1, 0);
    for (size_t i = 0; i < c.size(); ++i) o[i + 1] = o[i] + c[i];
    return o;
}

}  // namespace
}  // namespace crdt

using namespace crdt;

extern "C" int crdt_population_create(crdt_ctx *ctx, const crdt_population_init *h, crdt_population **out) {
    if (!out) return CRDT_E_INVAL;
    *out = nullptr;
    int rc = bind(ctx);
    if (rc) return rc;
    if (!h || !h->l_off || h->keys_per_replica == 0 || !h->str_off) return CRDT_E_INVAL;
    const uint32_t P = h->replicas;
    if ((uint64_t)P * h->keys_per_replica > 0xffffffffULL) return CRDT_E_RANGE;
    const uint64_t n_e = h->l_off[P];
    if (h->l_off[0] != 0 || (n_e && (!h->l_ts || !h->l_origin)) || !h->l_kv || h->l_kv[0] != 0) return CRDT_E_INVAL;
    for (uint32_t p = 0; p < P; ++p)
        if (h->l_off[p + 1] < h->l_off[p]) return CRDT_E_INVAL;
    const uint64_t n_kv = h->l_kv[n_e];
    if (n_kv && (!h->kv_key || !h->kv_val)) return CRDT_E_INVAL;
    if (h->n_str && !h->str_bytes) return CRDT_E_INVAL;
    crdt_population *pop = new (std::nothrow) crdt_population();
    if (!pop) return CRDT_E_NOMEM;
    pop->ctx = ctx;
    pop->P = P;
    pop->K = h->keys_per_replica;
    pop->first = h->first;
    pop->cnt.resize(P);
    pop->kvcnt.resize(P);
    for (uint32_t p = 0; p < P; ++p) {
        pop->cnt[p] = h->l_off[p + 1] - h->l_off[p];
        pop->kvcnt[p] = h->l_kv[h->l_off[p + 1]] - h->l_kv[h->l_off[p]];
    }
    pop->n_e = n_e;
    pop->n_kv = n_kv;
    pop->n_str = h->n_str;
    pop->one_pair = true;
    for (uint64_t e = 0; e < n_e && pop->one_pair; ++e) pop->one_pair = h->l_kv[e + 1] - h->l_kv[e] == 1;
    auto &d = pop->d[0];
    rc = diff_reserve(pop, d, n_e, n_kv, false);
    const uint64_t ns = (uint64_t)P * pop->K, nbytes = h->str_off[h->n_str];
    for (int b = 0; b < 2 && !rc; ++b) {
        rc = alloc(ctx, &pop->st_kind[b], ns);
        if (!rc) rc = alloc(ctx, &pop->st_str[b], ns);
        if (!rc) rc = alloc(ctx, &pop->st_sum[b], ns);
    }
    if (!rc) rc = alloc(ctx, &pop->str_bytes, nbytes);
    if (!rc) rc = alloc(ctx, &pop->str_off, h->n_str + 1);
    hipError_t e = hipSuccess;
    auto up = [&](void *dst, const void *src, size_t bytes) {
        if (e == hipSuccess && bytes) e = hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice);
    };
    if (!rc) {
        up(d.off, h->l_off, (P + 1) * 8);
        up(d.ts, h->l_ts, n_e * 8);
        up(d.origin, h->l_origin, n_e);
        up(d.kv_off, h->l_kv, (n_e + 1) * 8);
        up(d.kv_key, h->kv_key, n_kv * 4);
        up(d.kv_val, h->kv_val, n_kv * 4);
        up(pop->str_bytes, h->str_bytes, nbytes);
        up(pop->str_off, h->str_off, (h->n_str + 1) * 8);
        // CurrentState of NewServer with an empty initialState (main.go:102-105): every slot absent
        if (e == hipSuccess && ns) e = hipMemset(pop->st_kind[0], 0, ns);
        if (e == hipSuccess && ns) e = hipMemset(pop->st_str[0], 0, ns * 4);
        if (e == hipSuccess && ns) e = hipMemset(pop->st_sum[0], 0, ns * 8);
        if (e != hipSuccess) rc = hip_fail(ctx, e);
    }
    if (rc) {
        (void)crdt_population_destroy(pop);
        return rc;
    }
    *out = pop;
    return CRDT_OK;
}

extern "C" int crdt_population_destroy(crdt_population *pop) {
    if (!pop) return CRDT_OK;
    if (pop->ctx) {
        (void)bind(pop->ctx);
        (void)hipStreamSynchronize(pop->ctx->stream);
    }
    diff_free(pop->d[0]);
    diff_free(pop->d[1]);
    for (int b = 0; b < 2; ++b)
        for (void *p : {(void *)pop->st_kind[b], (void *)pop->st_str[b], (void *)pop->st_sum[b]})
            if (p) (void)hipFree(p);
    if (!pop->vtab)
        for (void *p : {(void *)pop->str_bytes, (void *)pop->str_off})
            if (p) (void)hipFree(p);
    for (void *p : {pop->dsm, pop->xb, pop->dscr})
        if (p) (void)hipFree(p);
    if (pop->pin) (void)hipHostFree(pop->pin);
    if (pop->hflag) (void)hipHostFree(pop->hflag);
    delete pop;
    return CRDT_OK;
}

// POST /data on every replica at once (AddCommand, main.go:173-215) through
// crdt_local_apply: the commands (host arrays, arrival order per replica) in
// one upload, the next Diffs and CurrentState into the spare buffers (the
// state copied first: the apply updates it in place), the new Diffs' kv
// pairs gathered from the old Diffs' and the commands' (by src, the entry
// count read on the device), one read-back of the bounds, the status word
// and every command's HTTP status.  More than kLaMax commands for one
// replica run as several chunks, each the next kLaMax of every replica's.
namespace crdt {
namespace {
constexpr uint64_t kLaMax = 4096;        // crdt_local_apply: commands per replica per call

int pop_apply_chunk(crdt_population *pop, const crdt_population_cmds &c, const std::vector<uint64_t> &idx,
                    const std::vector<uint64_t> &sub_off, uint16_t *status) {
    crdt_ctx *ctx = pop->ctx;
    const uint32_t P = pop->P;
    const size_t n_c = idx.size();
    // the chunk's commands, packed: c_off P+1 | c_ts n_c | c_kv n_c+1 (u64), kv_key | kv_val (u32)
    std::vector<uint64_t> kv_off(n_c + 1, 0);
    for (size_t j = 0; j < n_c; ++j) kv_off[j + 1] = kv_off[j] + (c.c_kv[idx[j] + 1] - c.c_kv[idx[j]]);
    const size_t n_kvc = kv_off[n_c];
    const size_t bytes = Carve::round((P + 1) * 8) + Carve::round(n_c * 8 + 8) + Carve::round((n_c + 1) * 8) +
                         Carve::round(n_kvc * 4 + 4) * 2 + Carve::round(n_c * 2 + 2) + round_bytes(P) + 1024;
    int rc = dev_grow(ctx, &pop->xb, &pop->xb_bytes, bytes);
    if (!rc) rc = pin_grow(pop, bytes);
    if (rc) return rc;
    Carve w(pop->xb), hw(pop->pin);
    uint64_t *d_off = w.take<uint64_t>(P + 1), *h_off = hw.take<uint64_t>(P + 1);
    int64_t *d_ts = w.take<int64_t>(n_c + 1), *h_ts = hw.take<int64_t>(n_c + 1);
    uint64_t *d_kv = w.take<uint64_t>(n_c + 1), *h_kv = hw.take<uint64_t>(n_c + 1);
    uint32_t *d_key = w.take<uint32_t>(n_kvc + 1), *h_key = hw.take<uint32_t>(n_kvc + 1);
    uint32_t *d_val = w.take<uint32_t>(n_kvc + 1), *h_val = hw.take<uint32_t>(n_kvc + 1);
    uint16_t *d_st = w.take<uint16_t>(n_c + 1), *h_st = hw.take<uint16_t>(n_c + 1);
    uint64_t *d_bounds = w.take<uint64_t>(2 * P + 4), *h_bounds = hw.take<uint64_t>(2 * P + 4);
    std::copy(sub_off.begin(), sub_off.end(), h_off);
    std::copy(kv_off.begin(), kv_off.end(), h_kv);
    for (size_t j = 0; j < n_c; ++j) {
        h_ts[j] = c.c_ts[idx[j]];
        const uint64_t a = c.c_kv[idx[j]], b = c.c_kv[idx[j] + 1];
        std::copy(c.kv_key + a, c.kv_key + b, h_key + kv_off[j]);
        std::copy(c.kv_val + a, c.kv_val + b, h_val + kv_off[j]);
    }
    const size_t upto = (size_t)((char *)(h_val + n_kvc + 1) - (char *)pop->pin);
    hipError_t e = hipMemcpyAsync(pop->xb, pop->pin, upto, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(d_bounds + 2 * P + 3, ctx->dev_status, 8, hipMemcpyDeviceToDevice, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
    pop->can_undo = false;                               // (undo is a round's; the spare buffers are rewritten below)
    auto &nd = pop->d[1 - pop->cur];
    rc = diff_reserve(pop, nd, pop->n_e + n_c, pop->n_kv + n_kvc, false);
    if (rc) return rc;
    auto &cd = pop->d[pop->cur];
    const int so = pop->cur, sn = 1 - pop->cur;
    const uint64_t ns = (uint64_t)P * pop->K;
    if (ns) {
        e = hipMemcpyAsync(pop->st_kind[sn], pop->st_kind[so], ns, hipMemcpyDeviceToDevice, ctx->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(pop->st_str[sn], pop->st_str[so], ns * 4, hipMemcpyDeviceToDevice, ctx->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(pop->st_sum[sn], pop->st_sum[so], ns * 8, hipMemcpyDeviceToDevice, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e);
    }
    crdt_local_in in{};
    in.replicas = P;
    in.n_slots = (uint32_t)ns;
    in.n_l = pop->n_e;
    in.n_c = n_c;
    in.n_kv = n_kvc;
    in.n_str = pop->n_str;
    in.l_off = cd.off;
    in.l_ts = cd.ts;
    in.l_origin = cd.origin;
    in.c_off = d_off;
    in.c_ts = d_ts;
    in.c_kv = d_kv;
    in.kv_key = d_key;
    in.kv_val = d_val;
    in.str_bytes = pop->str_bytes;
    in.str_off = pop->str_off;
    const crdt_local_out out{nd.off, nd.ts, nd.origin, nd.src, d_st, pop->st_kind[sn], pop->st_str[sn], pop->st_sum[sn]};
    rc = crdt_local_apply(ctx, &in, &out);
    if (rc) return rc;
    // the new Diffs' kv pairs: an entry's from the old Diff (src >= 0) or its command (src < 0)
    rc = seg_gather2_dev_count(ctx, pop->n_e + n_c, nd.off + P, nd.src, cd.kv_off, d_kv, nd.kv_off, cd.kv_key, d_key,
                               nd.kv_key, cd.kv_val, d_val, nd.kv_val);
    if (rc) return rc;
    k_pop_bounds<<<grid_for(P + 1, 256, 64), 256, 0, ctx->stream>>>(nd.off, nd.kv_off, P, ctx->dev_status, d_bounds);
    rc = check_launch(ctx);
    if (rc) return rc;
    e = hipMemcpyAsync(h_bounds, d_bounds, (2 * P + 4) * 8, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && n_c) e = hipMemcpyAsync(h_st, d_st, n_c * 2, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
    const uint32_t after = (uint32_t)h_bounds[2 * P + 2], before = (uint32_t)h_bounds[2 * P + 3];
    if (after & ~before) return CRDT_E_DEVICE;           // nothing swapped in
    for (size_t j = 0; j < n_c; ++j) status[idx[j]] = h_st[j];
    for (uint32_t p = 0; p < P; ++p) {
        pop->cnt[p] = h_bounds[p + 1] - h_bounds[p];
        pop->kvcnt[p] = h_bounds[P + 2 + p] - h_bounds[P + 1 + p];
    }
    pop->n_e = h_bounds[P];
    pop->n_kv = h_bounds[2 * P + 1];
    pop->cur = 1 - pop->cur;
    pop->can_undo = false;                               // (undo is a round's)
    return CRDT_OK;
}

}  // namespace
}  // namespace crdt

extern "C" int crdt_population_add_commands(crdt_population *pop, const crdt_population_cmds *c, uint16_t *status) {
    if (!pop_valid(pop) || !c || !c->c_off) return CRDT_E_INVAL;
    int rc = bind(pop->ctx);
    if (rc) return rc;
    pop_arena(pop);
    const uint32_t P = pop->P;
    if (c->c_off[0] != 0) return CRDT_E_INVAL;
    for (uint32_t p = 0; p < P; ++p)
        if (c->c_off[p + 1] < c->c_off[p]) return CRDT_E_INVAL;
    const uint64_t n_c = c->c_off[P];
    if (n_c == 0) return CRDT_OK;
    if (!c->c_ts || !c->c_kv || !status || c->c_kv[0] != 0) return CRDT_E_INVAL;
    for (uint64_t j = 0; j < n_c; ++j)
        if (c->c_kv[j + 1] < c->c_kv[j]) return CRDT_E_INVAL;
    if (c->c_kv[n_c] && (!c->kv_key || !c->kv_val)) return CRDT_E_INVAL;
    for (uint64_t q = 0; q < c->c_kv[n_c]; ++q)          // slots of the replica's own range (checked per command below)
        if (c->kv_val[q] >= pop->n_str) return CRDT_E_INVAL;
    for (uint32_t p = 0; p < P; ++p)
        for (uint64_t j = c->c_off[p]; j < c->c_off[p + 1]; ++j)
            for (uint64_t q = c->c_kv[j]; q < c->c_kv[j + 1]; ++q)
                if (c->kv_key[q] < (uint64_t)p * pop->K || c->kv_key[q] >= (uint64_t)(p + 1) * pop->K)
                    return CRDT_E_INVAL;
    for (uint64_t j = 0; j < n_c && pop->one_pair; ++j)   // (cleared before any chunk lands)
        if (c->c_kv[j + 1] - c->c_kv[j] != 1) pop->one_pair = false;
    std::fill(status, status + n_c, (uint16_t)0);        // 0 = not applied (a failing chunk leaves its own and later ones at 0)
    uint64_t most = 0;
    for (uint32_t p = 0; p < P; ++p) most = std::max(most, c->c_off[p + 1] - c->c_off[p]);
    for (uint64_t r = 0; r * kLaMax < most; ++r) {       // chunk r: the commands r*kLaMax .. of every replica
        std::vector<uint64_t> idx, sub_off(P + 1, 0);
        for (uint32_t p = 0; p < P; ++p) {
            const uint64_t a = std::min(c->c_off[p] + r * kLaMax, c->c_off[p + 1]);
            const uint64_t b = std::min(a + kLaMax, c->c_off[p + 1]);
            for (uint64_t j = a; j < b; ++j) idx.push_back(j);
            sub_off[p + 1] = idx.size();
        }
        rc = pop_apply_chunk(pop, *c, idx, sub_off, status);
        if (rc) return rc;
    }
    return CRDT_OK;
}

// Undo the last round: the Diffs and CurrentState as they were before it
// (still in the spare buffers; valid once, until the next round).
extern "C" int crdt_population_undo(crdt_population *pop) {
    if (!pop_valid(pop)) return CRDT_E_INVAL;
    if (!pop->can_undo) return CRDT_E_INVAL;
    int rc = bind(pop->ctx);
    if (rc) return rc;
    // (no synchronisation: the swap is host bookkeeping, and every later use of
    // either buffer set is ordered behind the round on the population's stream)
    pop->cnt.swap(pop->pcnt);
    pop->kvcnt.swap(pop->pkvcnt);
    pop->n_e = pop->p_n_e;
    pop->n_kv = pop->p_n_kv;
    pop->one_pair = pop->p_one_pair;
    pop->cur = 1 - pop->cur;
    pop->can_undo = false;
    return CRDT_OK;
}

extern "C" int crdt_population_info(const crdt_population *pop, uint32_t *replicas, size_t *n_entries,
                                    size_t *n_kv) {
    if (!pop_valid(pop) || !replicas || !n_entries || !n_kv) return CRDT_E_INVAL;
    *replicas = pop->P;
    *n_entries = pop->n_e;
    *n_kv = pop->n_kv;
    return CRDT_OK;
}

extern "C" int crdt_population_read(crdt_population *pop, uint64_t *l_off, int64_t *ts, uint8_t *origin,
                                    uint64_t *l_kv, uint32_t *kv_key, uint32_t *kv_val, uint8_t *st_kind,
                                    uint32_t *st_str, int64_t *st_sum) {
    if (!pop_valid(pop)) return CRDT_E_INVAL;
    int rc = bind(pop->ctx);
    if (rc) return rc;
    const auto &d = pop->d[pop->cur];
    const int s = pop->cur;
    const uint64_t ns = (uint64_t)pop->P * pop->K;
    hipError_t e = hipStreamSynchronize(pop->ctx->stream);
    auto down = [&](void *dst, const void *src, size_t bytes) {
        if (e == hipSuccess && dst && bytes) e = hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
    };
    down(l_off, d.off, (pop->P + 1) * 8);
    down(ts, d.ts, pop->n_e * 8);
    down(origin, d.origin, pop->n_e);
    down(l_kv, d.kv_off, (pop->n_e + 1) * 8);
    down(kv_key, d.kv_key, pop->n_kv * 4);
    down(kv_val, d.kv_val, pop->n_kv * 4);
    down(st_kind, pop->st_kind[s], ns);
    down(st_str, pop->st_str[s], ns * 4);
    down(st_sum, pop->st_sum[s], ns * 8);
    return e == hipSuccess ? CRDT_OK : hip_fail(pop->ctx, e);
}

// One synchronous round, every peer on this population: local replica i
// pulls the Diff of global replica peers[i] (peers[i] == first + i: a
// self-pull, merge() runs and rebuilds CurrentState; -1: a dead peer, the
// round is skipped for i).
extern "C" int crdt_population_round(crdt_population *pop, const int64_t *peers) {
    if (!pop_valid(pop) || (!peers && pop->P)) return CRDT_E_INVAL;
    int rc = bind(pop->ctx);
    if (rc) return rc;
    const uint32_t P = pop->P;
    if (P == 0) return CRDT_OK;
    const std::vector<uint64_t> l_off = prefix(pop->cnt);
    HostRound h(P);
    for (uint32_t i = 0; i < P; ++i) {
        const int64_t q = peers[i];
        if (q < 0) {                                     // dead: an empty pull, state kept
            h.r_off[i] = h.r_end[i] = l_off[i];
            h.skip[i] = 1;
            h.any_skip = true;
            continue;
        }
        if ((uint64_t)q < pop->first || (uint64_t)q - pop->first >= P) return CRDT_E_INVAL;   // not on this population
        const uint32_t lq = (uint32_t)((uint64_t)q - pop->first);
        h.r_off[i] = l_off[lq];
        h.r_end[i] = l_off[lq + 1];
        h.sd[i] = (uint32_t)(((int64_t)i - (int64_t)lq) * (int64_t)pop->K);
        h.n_r += pop->cnt[lq];
        h.n_rkv += pop->kvcnt[lq];
    }
    RoundArrays a;
    rc = upload_round(pop, h, &a);
    const auto &cd = pop->d[pop->cur];
    if (!rc) rc = pop_merge(pop, a, h, cd.ts, cd.kv_off, pop->n_kv, pop->one_pair);   // (pulls: this population's own Diffs)
    if (rc) return rc;
    return pop_commit(pop);                              // (one_pair kept: entries of one-pair Diffs)
}

// One synchronous round whose pulls arrive on the wire (main.go:226-258 with
// the Gossip body of main.go:159 in its binary form): body i =
// bodies[body_off[i], body_off[i+1]) in device memory is local replica i's
// pulled Diff; an empty body is a failed GET (the round skipped for i,
// main.go:234-239).  The bodies are decoded on the device against the
// context's string tables (keys: key id k of replica i -> slot i*K + k, ids
// below K; vals: the value ids, whose arena becomes the population's), their
// pairs behind the current Diff's in its kv arena, then merged as in
// crdt_population_round.  A body the device decode does not take (malformed,
// a nil map, unsorted, a key id >= K) fails the call with CRDT_E_UNSORTED and
// its status in body_status[i] (host, P words; 0 = taken): nothing is merged.
// The first wire round checks that vals holds the population's strings at
// their ids (intern them first) and adopts its arena.  Synchronises.
extern "C" int crdt_population_round_wire(crdt_population *pop, crdt_strtab *keys, crdt_strtab *vals,
                                          const uint8_t *bodies, const uint64_t *body_off, uint32_t *body_status) {
    if (!pop_valid(pop) || !keys || !vals || !body_status || (!body_off && pop->P)) return CRDT_E_INVAL;
    int rc = bind(pop->ctx);
    if (rc) return rc;
    const uint32_t P = pop->P;
    if (P == 0) return CRDT_OK;
    crdt_ctx *ctx = pop->ctx;
    if (!bodies && body_off[P] > body_off[0]) return CRDT_E_INVAL;
    if (pop->vtab && pop->vtab != vals) return CRDT_E_INVAL;
    if (!pop->vtab) {                                    // adopt vals' arena: its first n_str strings must agree
        uint64_t nv = 0, nbv = 0;
        (void)crdt_strtab_info(vals, &nv, &nbv, nullptr, nullptr);
        if (nv < pop->n_str) return CRDT_E_INVAL;
        std::vector<uint64_t> off(pop->n_str + 1);
        hipError_t e = hipMemcpy(off.data(), pop->str_off, off.size() * 8, hipMemcpyDeviceToHost);
        std::vector<uint8_t> bytes(off.back() - off[0]);
        if (e == hipSuccess && !bytes.empty())
            e = hipMemcpy(bytes.data(), pop->str_bytes + off[0], bytes.size(), hipMemcpyDeviceToHost);
        if (e != hipSuccess) return hip_fail(ctx, e);
        for (uint64_t i = 0; i < pop->n_str; ++i) {
            const char *q = nullptr;
            size_t qn = 0;
            if (crdt_strtab_get(vals, i, &q, &qn) != CRDT_OK || qn != off[i + 1] - off[i] ||
                (qn && memcmp(q, bytes.data() + (off[i] - off[0]), qn) != 0))
                return CRDT_E_INVAL;
        }
    }
    std::vector<uint64_t> at(P), len(P);
    for (uint32_t i = 0; i < P; ++i) {
        if (body_off[i + 1] < body_off[i]) return CRDT_E_INVAL;
        at[i] = body_off[i];
        len[i] = body_off[i + 1] - body_off[i];
    }
    // sizes from the headers: the decode's entries per body, pairs in total
    std::vector<uint8_t> hdr(32 * (size_t)P);
    rc = gossip_headers(ctx, P, bodies, at.data(), len.data(), hdr.data());
    if (rc) return rc;
    HostRound h(P);
    std::vector<uint32_t> sbase(P);
    uint64_t n_e = 0, n_p = 0;
    for (uint32_t i = 0; i < P; ++i) {
        uint64_t ne = 0, np = 0, nby = 0;
        if (len[i] >= 32 && memcmp(&hdr[32 * i], "CRDTSOA1", 8) == 0) {
            memcpy(&ne, &hdr[32 * i + 8], 8);
            memcpy(&np, &hdr[32 * i + 16], 8);
            memcpy(&nby, &hdr[32 * i + 24], 8);
            if (ne > len[i] / 12 || np > len[i] / 8 || nby > len[i] || 32 + ne * 12 + np * 8 + nby != len[i])
                ne = np = 0;                             // (malformed: the decode flags it)
        }
        h.r_off[i] = n_e;
        h.r_end[i] = n_e + ne;
        sbase[i] = (uint32_t)((uint64_t)i * pop->K);
        if (len[i] == 0) {                               // a failed GET: no merge for i
            h.skip[i] = 1;
            h.any_skip = true;
        }
        n_e += ne;
        n_p += np;
    }
    if (n_e >= 0xFFFFFFFFull) return CRDT_E_RANGE;
    h.n_r = n_e;
    h.n_rkv = n_p;
    // the pulled pairs go behind the current Diff's own in its kv arena; the
    // decoded entries into the exchange buffers
    auto &cd = pop->d[pop->cur];
    rc = diff_reserve(pop, cd, pop->n_e, pop->n_kv + n_p, true);
    const size_t xb = Carve::round((P + 1) * 8) + Carve::round(n_e * 8 + 8) + Carve::round((n_e + 1) * 8) + 1024;
    if (!rc) rc = dev_grow(ctx, &pop->xb, &pop->xb_bytes, xb);
    if (rc) return rc;
    Carve w(pop->xb);
    uint64_t *r_off = w.take<uint64_t>(P + 1);
    int64_t *r_ts = w.take<int64_t>(n_e + 1);
    uint64_t *r_kv = w.take<uint64_t>(n_e + 1);
    const crdt_gossip_decoded go{r_off, r_ts, r_kv, cd.kv_key, cd.kv_val};
    uint64_t multi = 1;
    // The merge is enqueued by the decode right behind its claim pass
    // (pop.wire_early, default 1): the pulled strings are nearly always
    // interned already, so the host does not wait for the claims before the
    // merge starts.  Its guesses -- the one-pair passes when the population
    // is one-pair, the ids as the claim pass left them -- are checked after
    // the decode; a wrong one (new strings, a multi-pair pull) runs the merge
    // again.  Either way it writes only the spare buffers: a refused body
    // still leaves the population as it was (with nothing to undo).
    const bool guess_one = pop->one_pair;
    RoundArrays a;
    bool merged = false;
    const std::function<int()> run_merge = [&]() -> int {
        int r = upload_round(pop, h, &a);
        if (!r) {                                        // (R just written by the decode: crdt_ctx::rm_nt)
            ctx->rm_nt = false;
            r = pop_merge(pop, a, h, r_ts, r_kv, pop->n_kv + n_p, guess_one);
            ctx->rm_nt = true;
        }
        merged = r == CRDT_OK;
        return r;
    };
    bool stale = false;
    const size_t need = gossip_decode_scratch_bytes(P, n_e, n_p);
    // Not on a population's first wire round (no vtab yet): the early merge
    // would fold with the population's own arena and n_str, while vals may
    // already hold strings past them (a refused earlier round interned them,
    // or vals is shared), and a pulled id in [n_str, vals->n) would skip the
    // replay fold without the rerun below noticing.
    const bool early = g_pop_wire_early && pop->vtab &&
                       dev_grow(ctx, &pop->dscr, &pop->dscr_bytes, need) == CRDT_OK;
    rc = gossip_decode_at(ctx, P, bodies, at.data(), len.data(), pop->K, pop->n_kv, sbase.data(), hdr.data(), keys,
                          vals, &go, body_status, early ? &run_merge : nullptr, early ? pop->dscr : nullptr,
                          early ? pop->dscr_bytes : 0, &stale, &multi);
    if (rc) return rc;
    for (uint32_t i = 0; i < P; ++i)
        if (body_status[i] && len[i]) return CRDT_E_UNSORTED;   // (nothing committed: the population is unchanged)
    if (!pop->vtab) {                                    // the arena is vals' from now on
        (void)dev_free(ctx, (void **)&pop->str_bytes);
        (void)dev_free(ctx, (void **)&pop->str_off);
        pop->vtab = vals;
    }
    // one pair per pulled entry too (counted by the decode): the one-pair passes
    const bool one = pop->one_pair && multi == 0;
    if (!merged || stale || one != guess_one) {
        rc = upload_round(pop, h, &a);
        if (!rc) {
            ctx->rm_nt = false;
            rc = pop_merge(pop, a, h, r_ts, r_kv, pop->n_kv + n_p, one);
            ctx->rm_nt = true;
        }
        if (rc) return rc;
    }
    rc = pop_commit(pop);
    if (!rc) pop->one_pair = one;
    return rc;
}

// One synchronous round over a communicator: member i's population holds
// global replicas crdt_shard_range(total, nranks, rank0 + i); peers_all[r]
// is global replica r's draw (global ids, -1 = dead peer), identical on every
// rank.  Each rank receives exactly the Diffs its replicas pull (main.go:226-
// 258 over xGMI): count all-gather, one point-to-point group, the merge.
// Synchronises.
extern "C" int crdt_population_round_sharded(crdt_comm *c, crdt_population *const *pops, const int64_t *peers_all,
                                             uint64_t total) {
    const size_t M = comm_members(c);
    if (M == 0 || !pops || (!peers_all && total)) return CRDT_E_INVAL;
    const int R = comm_nranks(c), g0 = comm_rank0(c);
    std::vector<uint64_t> f(R + 1);
    for (int r = 0; r < R; ++r) {
        uint64_t b, e;
        int rc = crdt_shard_range(total, R, r, &b, &e);
        if (rc) return rc;
        f[r] = b;
        f[r + 1] = e;
    }
    uint64_t maxP = 0;
    for (int r = 0; r < R; ++r) maxP = std::max(maxP, f[r + 1] - f[r]);
    for (size_t i = 0; i < M; ++i) {
        const crdt_population *p = pops[i];
        const int g = g0 + (int)i;
        if (!pop_valid(p) || p->ctx != comm_member_ctx(c, i) || p->first != f[g] || p->P != f[g + 1] - f[g])
            return CRDT_E_INVAL;
    }
    for (uint64_t r = 0; r < total; ++r)
        if (peers_all[r] >= (int64_t)total) return CRDT_E_INVAL;
    auto owner = [&](uint64_t q) { return (int)(std::upper_bound(f.begin(), f.end(), q) - f.begin()) - 1; };
    // 1. every replica's entry / pair counts, all-gathered: block r = [cnt (maxP) | kvcnt (maxP)]
    const size_t blk = 2 * maxP;
    std::vector<const void *> snd(M);
    std::vector<void *> rcv(M);
    for (size_t i = 0; i < M; ++i) {
        crdt_population *p = pops[i];
        int rc = bind(p->ctx);
        if (!rc) rc = dev_grow(p->ctx, &p->xb, &p->xb_bytes, (R * blk + 1) * 8);
        if (!rc) rc = pin_grow(p, std::max(round_bytes(p->P), (R * blk + 1) * 8));
        if (rc) return rc;
        uint64_t *hp = (uint64_t *)p->pin;
        for (uint64_t k = 0; k < blk; ++k) hp[k] = 0;
        for (uint32_t k = 0; k < p->P; ++k) hp[k] = p->cnt[k], hp[maxP + k] = p->kvcnt[k];
        uint64_t *mine = (uint64_t *)p->xb + (size_t)(g0 + i) * blk;
        hipError_t e = hipMemcpyAsync(mine, hp, blk * 8, hipMemcpyHostToDevice, p->ctx->stream);
        if (e != hipSuccess) return hip_fail(p->ctx, e);
        snd[i] = mine;
        rcv[i] = p->xb;
    }
    int rc = comm_allgather(c, snd.data(), rcv.data(), blk * 8);
    if (rc) return rc;
    std::vector<uint64_t> allc(total), allk(total);
    {
        crdt_population *p = pops[0];
        rc = bind(p->ctx);
        if (rc) return rc;
        std::vector<uint64_t> h(R * blk);
        hipError_t e = hipMemcpyAsync(h.data(), p->xb, R * blk * 8, hipMemcpyDeviceToHost, p->ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(p->ctx->stream);
        if (e != hipSuccess) return hip_fail(p->ctx, e);
        for (int r = 0; r < R; ++r)
            for (uint64_t k = 0; k < f[r + 1] - f[r]; ++k) {
                allc[f[r] + k] = h[r * blk + k];
                allk[f[r] + k] = h[r * blk + maxP + k];
            }
    }
    // 2. the pull plan, identical on every rank: need[r] = the sorted distinct
    //    live peers rank r's replicas pull
    std::vector<std::vector<uint64_t>> need(R);
    for (int r = 0; r < R; ++r) {
        for (uint64_t q = f[r]; q < f[r + 1]; ++q)
            if (peers_all[q] >= 0) need[r].push_back((uint64_t)peers_all[q]);
        std::sort(need[r].begin(), need[r].end());
        need[r].erase(std::unique(need[r].begin(), need[r].end()), need[r].end());
    }
    // 3. per member: pack the Diffs others pull, size the import, build the
    //    round's per-replica arrays; then ONE point-to-point group
    struct Plan {
        std::vector<uint64_t> se, sk, re, rk;            // per rank: entries / pairs sent, received
        uint64_t E_out = 0, K_out = 0, E_in = 0, K_in = 0;
        int64_t *s_ts, *i_ts;
        uint32_t *s_kc, *s_key, *s_val, *i_kc;
        uint64_t *i_kv;
        HostRound h;
        explicit Plan(uint32_t P) : h(P) {}
    };
    std::vector<Plan> pl;
    pl.reserve(M);
    std::vector<XP2P> ops;
    for (size_t i = 0; i < M; ++i) {
        crdt_population *p = pops[i];
        crdt_ctx *ctx = p->ctx;
        const int g = g0 + (int)i;
        pl.emplace_back(p->P);
        Plan &x = pl.back();
        x.se.assign(R, 0), x.sk.assign(R, 0), x.re.assign(R, 0), x.rk.assign(R, 0);
        std::vector<int64_t> codes;                      // local replicas sent, in destination order
        std::vector<uint64_t> de{0}, dk{0};              // their entry / pair offsets in the send block
        for (int r = 0; r < R; ++r)
            for (uint64_t q : need[r])
                if (q >= f[g] && q < f[g + 1]) {
                    codes.push_back((int64_t)(q - f[g]));
                    x.se[r] += allc[q];
                    x.sk[r] += allk[q];
                    de.push_back(de.back() + allc[q]);
                    dk.push_back(dk.back() + allk[q]);
                }
        x.E_out = de.back(), x.K_out = dk.back();
        std::vector<uint64_t> imp_off{0};                // the import block: need[g] in order (= rank order)
        for (uint64_t q : need[g]) {
            x.re[owner(q)] += allc[q];
            x.rk[owner(q)] += allk[q];
            imp_off.push_back(imp_off.back() + allc[q]);
        }
        x.E_in = imp_off.back();
        for (int r = 0; r < R; ++r) x.K_in += x.rk[r];
        // the round's R ranges into the import block
        for (uint32_t k = 0; k < p->P; ++k) {
            const int64_t q = peers_all[f[g] + k];
            if (q < 0) {
                x.h.skip[k] = 1;
                x.h.any_skip = true;
                continue;
            }
            const size_t idx = (size_t)(std::lower_bound(need[g].begin(), need[g].end(), (uint64_t)q) - need[g].begin());
            x.h.r_off[k] = imp_off[idx];
            x.h.r_end[k] = imp_off[idx + 1];
            const int64_t lq = q - (int64_t)f[owner((uint64_t)q)];
            x.h.sd[k] = (uint32_t)(((int64_t)k - lq) * (int64_t)p->K);
            x.h.n_r += allc[q];
            x.h.n_rkv += allk[q];
        }
        // the import's pairs go behind the Diff's own in its kv arena
        rc = bind(ctx);
        if (!rc) rc = diff_reserve(p, p->d[p->cur], 0, p->n_kv + x.K_in, true);
        if (rc) return rc;
        // device buffers: codes | de | dk | a_kr (P + 1) | kc of every entry | send ts kc key val | import ts kc kv
        const size_t ns_ = codes.size();
        const size_t need_b = Carve::round(ns_ * 8 + 8) + Carve::round((ns_ + 1) * 8) * 2 + Carve::round((p->P + 1) * 8) +
                              Carve::round(p->n_e * 4 + 4) + Carve::round(x.E_out * 8 + 8) + Carve::round(x.E_out * 4 + 4) +
                              Carve::round(x.K_out * 4 + 4) * 2 + Carve::round(x.E_in * 8 + 8) +
                              Carve::round(x.E_in * 4 + 4) + Carve::round((x.E_in + 1) * 8) + 4096;
        const size_t host_b = Carve::round(ns_ * 8 + 8) + Carve::round((ns_ + 1) * 8) * 2 + Carve::round((p->P + 1) * 8);
        rc = dev_grow(ctx, &p->xb, &p->xb_bytes, need_b);
        if (!rc) rc = pin_grow(p, std::max(host_b, round_bytes(p->P)));
        if (rc) return rc;
        Carve w(p->xb), hw(p->pin);
        int64_t *d_codes = w.take<int64_t>(ns_ + 1);
        uint64_t *d_de = w.take<uint64_t>(ns_ + 1), *d_dk = w.take<uint64_t>(ns_ + 1);
        uint64_t *d_akr = w.take<uint64_t>(p->P + 1);
        uint32_t *d_kc = w.take<uint32_t>(p->n_e + 1);
        x.s_ts = w.take<int64_t>(x.E_out + 1);
        x.s_kc = w.take<uint32_t>(x.E_out + 1);
        x.s_key = w.take<uint32_t>(x.K_out + 1);
        x.s_val = w.take<uint32_t>(x.K_out + 1);
        x.i_ts = w.take<int64_t>(x.E_in + 1);
        x.i_kc = w.take<uint32_t>(x.E_in + 1);
        x.i_kv = w.take<uint64_t>(x.E_in + 1);
        int64_t *h_codes = hw.take<int64_t>(ns_ + 1);
        uint64_t *h_de = hw.take<uint64_t>(ns_ + 1), *h_dk = hw.take<uint64_t>(ns_ + 1);
        uint64_t *h_akr = hw.take<uint64_t>(p->P + 1);
        std::copy(codes.begin(), codes.end(), h_codes);
        std::copy(de.begin(), de.end(), h_de);
        std::copy(dk.begin(), dk.end(), h_dk);
        h_akr[0] = 0;
        for (uint32_t k = 0; k < p->P; ++k) h_akr[k + 1] = h_akr[k] + p->kvcnt[k];
        hipError_t e = hipMemcpyAsync(p->xb, p->pin, hw.used, hipMemcpyHostToDevice, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);      // (the pinned staging is reused below)
        if (e != hipSuccess) return hip_fail(ctx, e);
        const auto &cd = p->d[p->cur];
        rc = crdt_offsets_to_counts(ctx, cd.kv_off, p->n_e, d_kc);
        if (!rc && ns_) rc = crdt_seg_copy(ctx, ns_, d_codes, cd.off, nullptr, d_de, 8, cd.ts, nullptr, x.s_ts, nullptr, 1);
        if (!rc && ns_) rc = crdt_seg_copy(ctx, ns_, d_codes, cd.off, nullptr, d_de, 4, d_kc, nullptr, x.s_kc, nullptr, 1);
        if (!rc && ns_ && x.K_out)
            rc = crdt_seg_copy2(ctx, ns_, d_codes, d_akr, nullptr, d_dk, 4, cd.kv_key, nullptr, x.s_key, nullptr,
                                cd.kv_val, nullptr, x.s_val, 1);
        if (rc) return rc;
        uint64_t so_e = 0, so_k = 0, ro_e = 0, ro_k = 0;
        for (int r = 0; r < R; ++r) {
            if (x.se[r]) {
                ops.push_back(XP2P{i, r, true, x.s_ts + so_e, nullptr, x.se[r] * 8});
                ops.push_back(XP2P{i, r, true, x.s_kc + so_e, nullptr, x.se[r] * 4});
            }
            if (x.sk[r]) {
                ops.push_back(XP2P{i, r, true, x.s_key + so_k, nullptr, x.sk[r] * 4});
                ops.push_back(XP2P{i, r, true, x.s_val + so_k, nullptr, x.sk[r] * 4});
            }
            if (x.re[r]) {
                ops.push_back(XP2P{i, r, false, nullptr, x.i_ts + ro_e, x.re[r] * 8});
                ops.push_back(XP2P{i, r, false, nullptr, x.i_kc + ro_e, x.re[r] * 4});
            }
            if (x.rk[r]) {
                ops.push_back(XP2P{i, r, false, nullptr, cd.kv_key + p->n_kv + ro_k, x.rk[r] * 4});
                ops.push_back(XP2P{i, r, false, nullptr, cd.kv_val + p->n_kv + ro_k, x.rk[r] * 4});
            }
            so_e += x.se[r], so_k += x.sk[r], ro_e += x.re[r], ro_k += x.rk[r];
        }
    }
    rc = comm_p2p(c, ops);
    if (rc) return rc;
    // 4. per member: the import's kv offsets (behind the Diff's pairs), then
    //    the merge reading the received Diffs in place
    for (size_t i = 0; i < M; ++i) {
        crdt_population *p = pops[i];
        Plan &x = pl[i];
        rc = bind(p->ctx);
        if (!rc) rc = crdt_counts_to_offsets(p->ctx, x.i_kc, x.E_in, p->n_kv, x.i_kv);
        RoundArrays a;
        if (!rc) rc = upload_round(p, x.h, &a);
        if (!rc) rc = pop_merge(p, a, x.h, x.i_ts, x.i_kv, p->n_kv + x.K_in);
        if (rc) return rc;
    }
    for (size_t i = 0; i < M; ++i) {                    // every member checked before any is swapped in
        const int rc_i = pop_commit_check(pops[i]);
        if (rc_i && !rc) rc = rc_i;
    }
    if (rc) return rc;
    for (size_t i = 0; i < M; ++i) {
        pop_commit_apply(pops[i]);
        pops[i]->one_pair = false;                       // (entries from other ranks' Diffs: not checked)
    }
    return CRDT_OK;
}
