// refmerge.hip -- bit-exact batched (*Server).merge() of the reference
// (/root/reference/main.go:35-100), many replicas per launch.
//
// Closed form implemented (derivation in DESIGN.md "RefMerge"):
//  Walk (main.go:45-73): Diff' = L u {r in R : r not in L, r < max(L)}.
//    r is inserted iff lower_bound(L, r) < |L| and L[lb] != r: an equal ts
//    keeps the local entry (main.go:54-65); remote ts above max(L) are never
//    reached by the two-pointer loop (main.go:49) and are dropped.
//  Replay (main.go:75-98): CurrentState rebuilt from empty over the
//    remote-origin entries of Diff' (local *Command values fail the
//    map[string]string assertion, main.go:80), descending ts.  Per key:
//      base = value of the max-ts entry holding the key;
//      if Atoi(base) fails or no other holder's value parses -> base verbatim
//      else Itoa(sum of every parsable value), int64 wrap (main.go:95).
//    The sum is order-independent (mod 2^64), which is what lets the fold run
//    as parallel atomics instead of the reference's serial descending loop.
//
// Kernels: atoi over the string arena; walk flags (binary search per R
// entry); device scan of the flags; L and R scatters into the new Diff;
// per-replica replay over the new Diff with LDS accumulators (k_replay).
// (Workgroup-per-replica and chunk-parallel walk/scatter variants measured
// no faster: every variant is bound by chains of dependent global loads.)
#include <algorithm>

#include "scan.hpp"

namespace crdt {

// Go 1.18 strconv.Atoi (64-bit): ^[+-]?[0-9]+$ within int64, leading zeros ok.
__device__ __forceinline__ bool go_atoi(const uint8_t *s, uint64_t len, int64_t *out) {
    if (len == 0) return false;
    uint64_t i = 0;
    bool neg = false;
    if (s[0] == '+' || s[0] == '-') {
        neg = s[0] == '-';
        i = 1;
        if (len == 1) return false;
    }
    uint64_t acc = 0;
    for (; i < len; ++i) {
        const unsigned d = (unsigned)s[i] - (unsigned)'0';
        if (d > 9) return false;
        if (acc > (0xFFFFFFFFFFFFFFFFULL - d) / 10) return false;   // ParseUint range error
        acc = acc * 10 + d;
    }
    if (!neg && acc >= 0x8000000000000000ULL) return false;        // ParseInt range error
    if (neg && acc > 0x8000000000000000ULL) return false;
    *out = neg ? (int64_t)(0 - acc) : (int64_t)acc;
    return true;
}

__global__ void k_atoi(const uint8_t *__restrict__ bytes, const uint64_t *__restrict__ off, uint64_t n,
                       uint8_t *__restrict__ ok, int64_t *__restrict__ val) {
    for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < n; s += (uint64_t)gridDim.x * 256) {
        int64_t v = 0;
        const bool good = go_atoi(bytes + off[s], off[s + 1] - off[s], &v);
        ok[s] = good;
        val[s] = good ? v : 0;
    }
}

// Replica owning global entry g: largest p with off[p] <= g.
__device__ __forceinline__ uint32_t owner(const uint64_t *off, uint32_t replicas, uint64_t g) {
    uint32_t lo = 0, hi = replicas;          // off[0] <= g < off[replicas]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (off[mid] <= g) lo = mid;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ uint64_t lower_bound_i64(const int64_t *v, uint64_t lo, uint64_t hi, int64_t x) {
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (v[mid] < x) lo = mid + 1;        // signed order: Int64Comparator (main.go:106)
        else hi = mid;
    }
    return lo;
}

__global__ void k_walk_flags(crdt_refmerge_in in, uint32_t *__restrict__ flag, uint64_t *__restrict__ rpos) {
    for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < in.n_r; g += (uint64_t)gridDim.x * 256) {
        const uint32_t p = owner(in.r_off, in.replicas, g);
        const uint64_t lb = in.l_off[p], le = in.l_off[p + 1];
        const int64_t r = in.r_ts[g];
        const uint64_t pos = lower_bound_i64(in.l_ts, lb, le, r);
        flag[g] = (pos < le && in.l_ts[pos] != r) ? 1u : 0u;
        rpos[g] = pos - lb;
    }
}

__global__ void k_out_off(crdt_refmerge_in in, const uint64_t *__restrict__ ib, uint64_t *__restrict__ out_off) {
    for (uint32_t p = blockIdx.x * 256 + threadIdx.x; p <= in.replicas; p += gridDim.x * 256)
        out_off[p] = in.l_off[p] + ib[in.r_off[p]];
}

__global__ void k_scatter_l(crdt_refmerge_in in, const uint64_t *__restrict__ ib, crdt_refmerge_out out) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < in.n_l; i += (uint64_t)gridDim.x * 256) {
        const uint32_t p = owner(in.l_off, in.replicas, i);
        const uint64_t rb = in.r_off[p], re = in.r_off[p + 1];
        const uint64_t lbr = lower_bound_i64(in.r_ts, rb, re, in.l_ts[i]);
        const uint64_t o = out.off[p] + (i - in.l_off[p]) + (ib[lbr] - ib[rb]);
        out.ts[o] = in.l_ts[i];
        out.origin[o] = in.l_origin[i];
        out.src[o] = (int64_t)i;
    }
}

__global__ void k_scatter_r(crdt_refmerge_in in, const uint32_t *__restrict__ flag,
                            const uint64_t *__restrict__ rpos, const uint64_t *__restrict__ ib,
                            crdt_refmerge_out out) {
    for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < in.n_r; g += (uint64_t)gridDim.x * 256) {
        if (!flag[g]) continue;
        const uint32_t p = owner(in.r_off, in.replicas, g);
        const uint64_t o = out.off[p] + rpos[g] + (ib[g] - ib[in.r_off[p]]);
        out.ts[o] = in.r_ts[g];
        out.origin[o] = 0;
        out.src[o] = -(int64_t)g - 1;
    }
}

// ---------------------------------------------------------------- replay
// One workgroup per replica, over the replica's NEW Diff (already written by
// the scatters, ascending ts): an entry's position o in it orders the
// entries by ts, so the base holder of a key (its max-ts entry) is the one
// with the largest (o << 32 | string id) -- a single 64-bit max, reduced in
// the same pass as the sums and counts.  The per-key accumulators live in an
// LDS hash table (slots of different replicas are disjoint, so the workgroup
// owns every slot it touches: no global atomics); a replica with more
// distinct keys than the table holds is redone by the same workgroup through
// its slice of slot-indexed global accumulators.  (Four contended global
// atomics per key plus a second base pass took 4x longer; chunk-parallel
// workgroups with a table flush were 1.4x slower than this.)
constexpr int RT = 1024;                  // LDS table entries per workgroup
constexpr uint32_t kEmpty = 0xFFFFFFFFu;

struct SlotAcc {                          // global fallback, indexed by slot
    unsigned long long *best;
    unsigned *nent;
    unsigned long long *sum;
    unsigned *npar;
};

__global__ void k_slot_clear(crdt_refmerge_out out, SlotAcc acc, uint32_t n) {
    for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s < n; s += gridDim.x * 256) {
        out.st_kind[s] = 0;               // untouched slot: key absent from CurrentState
        out.st_str[s] = 0;
        out.st_sum[s] = 0;
        acc.best[s] = 0;
        acc.nent[s] = 0;
        acc.sum[s] = 0;
        acc.npar[s] = 0;
    }
}

// kv range of new-Diff entry o, clamped to the arena
__device__ __forceinline__ void entry_kv(const crdt_refmerge_in &in, const crdt_refmerge_out &out, uint64_t o,
                                         uint64_t *kb, uint64_t *ke) {
    const int64_t src = out.src[o];
    if (src >= 0) {
        *kb = in.l_kv[src];
        *ke = in.l_kv[src + 1];
    } else {
        const uint64_t g = (uint64_t)(-(src + 1));
        *kb = in.r_kv[g];
        *ke = in.r_kv[g + 1];
    }
    if (*ke > in.n_kv) *ke = in.n_kv;     // malformed ranges never read out of bounds
}

// Per-key closed form (main.go:82-96): verbatim base unless the base parses
// AND another holder's value parses; then Itoa(sum) with int64 wrap.
__device__ __forceinline__ void slot_final(const crdt_refmerge_out &out, const uint8_t *ok, uint32_t slot,
                                           unsigned long long best, unsigned npar, unsigned long long sum) {
    const uint32_t str = (uint32_t)best;
    const bool sum_form = ok[str] && npar >= 2;
    out.st_kind[slot] = sum_form ? 2 : 1;
    out.st_str[slot] = str;
    out.st_sum[slot] = sum_form ? (int64_t)sum : 0;
}

__global__ __launch_bounds__(256) void k_replay(crdt_refmerge_in in, const uint8_t *__restrict__ ok,
                                                const int64_t *__restrict__ val, crdt_refmerge_out out,
                                                SlotAcc acc) {
    __shared__ uint32_t t_slot[RT];
    __shared__ unsigned long long t_best[RT];
    __shared__ unsigned long long t_sum[RT];
    __shared__ uint32_t t_nent[RT], t_npar[RT];
    __shared__ int s_over;
    const int tid = threadIdx.x;
    for (uint32_t p = blockIdx.x; p < in.replicas; p += gridDim.x) {
        for (int h = tid; h < RT; h += 256) {
            t_slot[h] = kEmpty;
            t_best[h] = 0;
            t_sum[h] = 0;
            t_nent[h] = 0;
            t_npar[h] = 0;
        }
        if (tid == 0) s_over = 0;
        __syncthreads();
        const uint64_t ob = out.off[p], oe = out.off[p + 1];
        for (uint64_t o = ob + tid; o < oe; o += 256) {
            if (out.origin[o]) continue;                 // *Command: skipped (main.go:80)
            uint64_t kb, ke;
            entry_kv(in, out, o, &kb, &ke);
            const unsigned long long pos = (unsigned long long)(o - ob) << 32;
            for (uint64_t q = kb; q < ke; ++q) {
                const uint32_t slot = in.kv_key[q], v = in.kv_val[q];
                if (slot >= in.n_slots || v >= in.n_str) continue;
                uint32_t h = (slot * 2654435761u) >> 22;   // 10-bit hash
                int idx = -1;
                for (int probe = 0; probe < 32; ++probe, h = (h + 1) & (RT - 1)) {
                    const uint32_t c = atomicCAS(&t_slot[h], kEmpty, slot);
                    if (c == kEmpty || c == slot) {
                        idx = (int)h;
                        break;
                    }
                }
                if (idx < 0) {
                    s_over = 1;
                    continue;
                }
                atomicMax(&t_best[idx], pos | v);
                atomicAdd(&t_nent[idx], 1u);
                if (ok[v]) {
                    atomicAdd(&t_sum[idx], (unsigned long long)val[v]);   // mod 2^64 (main.go:95)
                    atomicAdd(&t_npar[idx], 1u);
                }
            }
        }
        __syncthreads();
        if (!s_over) {
            for (int h = tid; h < RT; h += 256)
                if (t_slot[h] != kEmpty) slot_final(out, ok, t_slot[h], t_best[h], t_npar[h], t_sum[h]);
        } else {
            // too many distinct keys for the table: this replica again through
            // its own (disjoint) slice of the global accumulators
            for (uint64_t o = ob + tid; o < oe; o += 256) {
                if (out.origin[o]) continue;
                uint64_t kb, ke;
                entry_kv(in, out, o, &kb, &ke);
                const unsigned long long pos = (unsigned long long)(o - ob) << 32;
                for (uint64_t q = kb; q < ke; ++q) {
                    const uint32_t slot = in.kv_key[q], v = in.kv_val[q];
                    if (slot >= in.n_slots || v >= in.n_str) continue;
                    atomicMax(&acc.best[slot], pos | v);
                    atomicAdd(&acc.nent[slot], 1u);
                    if (ok[v]) {
                        atomicAdd(&acc.sum[slot], (unsigned long long)val[v]);
                        atomicAdd(&acc.npar[slot], 1u);
                    }
                }
            }
            __threadfence();
            __syncthreads();
            for (uint64_t o = ob + tid; o < oe; o += 256) {
                if (out.origin[o]) continue;
                uint64_t kb, ke;
                entry_kv(in, out, o, &kb, &ke);
                for (uint64_t q = kb; q < ke; ++q) {
                    const uint32_t slot = in.kv_key[q], v = in.kv_val[q];
                    if (slot >= in.n_slots || v >= in.n_str) continue;
                    slot_final(out, ok, slot,
                               __hip_atomic_load(&acc.best[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                               __hip_atomic_load(&acc.npar[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                               __hip_atomic_load(&acc.sum[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                }
            }
        }
        __syncthreads();                                 // table reused by the next replica
    }
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_atoi_batch(crdt_ctx *ctx, const uint8_t *bytes, const uint64_t *off, uint64_t n_str,
                               uint8_t *ok, int64_t *val) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (n_str == 0) return CRDT_OK;
    if (!bytes || !off || !ok || !val) return CRDT_E_INVAL;
    k_atoi<<<grid_for(n_str, 256, (unsigned)ctx->num_cus * 8), 256, 0, ctx->stream>>>(bytes, off, n_str, ok, val);
    return check_launch(ctx);
}

extern "C" int crdt_refmerge_batch(crdt_ctx *ctx, const crdt_refmerge_in *inp, const crdt_refmerge_out *outp) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!inp || !outp) return CRDT_E_INVAL;
    const crdt_refmerge_in in = *inp;
    const crdt_refmerge_out out = *outp;
    if (in.replicas == 0) return CRDT_OK;
    if (!in.l_off || !in.r_off || !out.off) return CRDT_E_INVAL;
    if (in.n_l && (!in.l_ts || !in.l_origin)) return CRDT_E_INVAL;
    if (!in.l_kv || !in.r_kv) return CRDT_E_INVAL;
    if (in.n_r && !in.r_ts) return CRDT_E_INVAL;
    if (in.n_kv && (!in.kv_key || !in.kv_val)) return CRDT_E_INVAL;
    if (in.n_l + in.n_r && (!out.ts || !out.origin || !out.src)) return CRDT_E_INVAL;
    if (in.n_slots && (!out.st_kind || !out.st_str || !out.st_sum)) return CRDT_E_INVAL;
    if (in.n_str && (!in.str_bytes || !in.str_off)) return CRDT_E_INVAL;
    if (in.n_kv && !in.n_str) return CRDT_E_INVAL;

    const size_t nr = in.n_r, ns = in.n_slots, nstr = in.n_str;
    const size_t need = Carve::round((nr + 1) * 4) + Carve::round(nr * 8 + 8) + Carve::round((nr + 1) * 8) +
                        scan_tmp_bytes(nr) + Carve::round(nstr + 1) + Carve::round(nstr * 8 + 8) +
                        Carve::round(ns * 8 + 8) * 2 + Carve::round(ns * 4 + 4) * 2 + 4096;
    rc = ws_reserve(ctx, need);
    if (rc) return rc;
    Carve w(ctx->ws);
    uint32_t *flag = w.take<uint32_t>(nr + 1);
    uint64_t *rpos = w.take<uint64_t>(nr + 1);
    uint64_t *ib = w.take<uint64_t>(nr + 1);
    void *tmp = w.take<char>(scan_tmp_bytes(nr));
    uint8_t *ok = w.take<uint8_t>(nstr + 1);
    int64_t *val = w.take<int64_t>(nstr + 1);
    SlotAcc acc;
    acc.best = w.take<unsigned long long>(ns + 1);
    acc.sum = w.take<unsigned long long>(ns + 1);
    acc.nent = w.take<unsigned>(ns + 1);
    acc.npar = w.take<unsigned>(ns + 1);

    const hipStream_t s = ctx->stream;
    const unsigned cap = (unsigned)ctx->num_cus * 8;
    if (nstr) k_atoi<<<grid_for(nstr, 256, cap), 256, 0, s>>>(in.str_bytes, in.str_off, nstr, ok, val);
    if (nr) k_walk_flags<<<grid_for(nr, 256, cap), 256, 0, s>>>(in, flag, rpos);
    rc = check_launch(ctx);
    if (rc) return rc;
    rc = exclusive_scan_u32(ctx, flag, ib, nr, tmp);
    if (rc) return rc;
    k_out_off<<<grid_for((size_t)in.replicas + 1, 256, cap), 256, 0, s>>>(in, ib, out.off);
    if (in.n_l) k_scatter_l<<<grid_for(in.n_l, 256, cap), 256, 0, s>>>(in, ib, out);
    if (nr) k_scatter_r<<<grid_for(nr, 256, cap), 256, 0, s>>>(in, flag, rpos, ib, out);
    if (ns) {
        k_slot_clear<<<grid_for(ns, 256, cap), 256, 0, s>>>(out, acc, (uint32_t)ns);
        if (in.n_l + nr) k_replay<<<std::min<unsigned>(in.replicas, (unsigned)ctx->num_cus * 4), 256, 0, s>>>(
            in, ok, val, out, acc);
    }
    return check_launch(ctx);
}
