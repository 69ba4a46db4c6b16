// local.hip -- batched local apply: AddCommand (main.go:173-215) for many
// replicas in one device call.
//
// Per replica p, commands j = c_off[p] .. c_off[p+1] in ARRIVAL order, each
// a (ts, pairs) write.  The reference handler, per command:
//   Diff.Put(ts, &data)                                   main.go:187
//     -- a *Command at ts; an equal ts REPLACES the entry (treemap Put), so
//        of several same-ms commands the last one stays in the Diff;
//   for key, value := range data                          main.go:188-207
//     key absent  -> CurrentState[key] = value; RETURN 200  (main.go:189-193)
//     else Atoi(current), Atoi(value) (either fails: RETURN 500, :195-204),
//          CurrentState[key] = Itoa(current + value)        (:205-206, wraps)
//   200                                                   main.go:207-208
// Go's map order is random; pairs are applied in the order given (callers
// pass them in key order for parity with crdt_server_add_command -- one of
// Go's legal executions).
//
// Device passes:
//   k_la_plan  (workgroup per replica): the replica's commands sorted by
//              (ts, arrival) in LDS, the last of each equal-ts run kept, each
//              kept command's lower_bound in the replica's Diff (lb) and
//              whether it replaces an entry there (eq); new Diff length;
//   scan of the lengths -> out.off;
//   k_la_write (workgroup per replica): the new Diff = the Diff with the
//              kept commands inserted / substituted.  Diff entry i lands at
//              i + #{kept c: lb_c <= i} - #{kept c: eq_c, lb_c < i}; kept
//              command c (rank c in ts order) at lb_c + c - #{eq before c};
//   k_la_state (thread per replica): the CurrentState apply, sequential over
//              the replica's commands in arrival order (each step depends on
//              the state the previous one left), HTTP status per command.
#include "scan.hpp"

namespace crdt {
namespace {

constexpr int LB = 256;                 // threads per replica workgroup
constexpr uint32_t kMaxCmd = 4096;      // commands per replica per call (LDS sort)
constexpr uint32_t kSkip = 0xFFFFFFFFu; // kcnt sentinel: the replica exceeded a limit, nothing of it is applied

struct alignas(16) LaOk {               // Go Atoi of one arena string
    int64_t val;
    int64_t ok;
};

__device__ __forceinline__ bool go_atoi_dev(const uint8_t *s, uint64_t len, int64_t *out) {
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
        if (d > 9 || acc > (0xFFFFFFFFFFFFFFFFULL - d) / 10) return false;
        acc = acc * 10 + d;
    }
    if ((!neg && acc >= 0x8000000000000000ULL) || (neg && acc > 0x8000000000000000ULL)) return false;
    *out = neg ? (int64_t)(0 - acc) : (int64_t)acc;
    return true;
}

__global__ void k_la_atoi(const uint8_t *__restrict__ bytes, const uint64_t *__restrict__ off, uint64_t n,
                          LaOk *__restrict__ ok) {
    for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < n; s += (uint64_t)gridDim.x * 256) {
        int64_t v = 0;
        const bool g = go_atoi_dev(bytes + off[s], off[s + 1] - off[s], &v);
        ok[s] = LaOk{g ? v : 0, g ? 1 : 0};
    }
}

// exclusive block scan of one value per thread (LB threads)
__device__ __forceinline__ uint32_t block_scan(uint32_t v, uint32_t *s_w, uint32_t *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    __syncthreads();
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (int k = 0; k < LB / 64; ++k) {
        base += k < w ? s_w[k] : 0;
        tot += s_w[k];
    }
    *total = tot;
    return base + x - v;
}

__device__ __forceinline__ uint64_t lower_bound_g(const int64_t *a, uint64_t n, int64_t x) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Sort the replica's commands by (ts, arrival) in LDS; keep the last of each
// equal-ts run; lb / eq of each kept command against the Diff.
__global__ __launch_bounds__(LB) void k_la_plan(crdt_local_in in, uint32_t *__restrict__ k_lb,
                                                uint32_t *__restrict__ k_j, uint8_t *__restrict__ k_eq,
                                                uint32_t *__restrict__ kcnt, uint32_t *__restrict__ cnt,
                                                uint32_t *__restrict__ err) {
    __shared__ int64_t s_ts[kMaxCmd];
    __shared__ uint32_t s_j[kMaxCmd];
    __shared__ uint32_t s_w[LB / 64];
    const uint32_t p = blockIdx.x;
    const uint64_t lb0 = in.l_off[p], nl = in.l_off[p + 1] - lb0;
    const uint64_t c0 = in.c_off[p], m64 = in.c_off[p + 1] - c0;
    if (m64 > kMaxCmd || nl + m64 >= 0xFFFFFFFFull) {    // the caller splits such batches
        if (threadIdx.x == 0) {
            atomicOr(err, CRDT_DEV_RANGE);
            cnt[p] = 0;
            kcnt[p] = kSkip;                             // k_la_write / k_la_state leave this replica alone
        }
        return;
    }
    const uint32_t m = (uint32_t)m64;
    uint32_t M = 64;
    while (M < m) M <<= 1;
    for (uint32_t i = threadIdx.x; i < M; i += LB) {
        s_ts[i] = i < m ? in.c_ts[c0 + i] : INT64_MAX;
        s_j[i] = i < m ? i : 0xFFFFFFFFu;                // padding sorts last
    }
    __syncthreads();
    for (uint32_t k = 2; k <= M; k <<= 1)                // bitonic sort by (ts, j)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < M; i += LB) {
                const uint32_t q = i ^ j;
                if (q > i) {
                    const bool up = (i & k) == 0;
                    const int64_t ta = s_ts[i], tb = s_ts[q];
                    const uint32_t ja = s_j[i], jb = s_j[q];
                    const bool gt = ta > tb || (ta == tb && ja > jb);
                    if (gt == up) {
                        s_ts[i] = tb, s_ts[q] = ta;
                        s_j[i] = jb, s_j[q] = ja;
                    }
                }
            }
            __syncthreads();
        }
    // keep the last command of each equal-ts run (treemap Put replaces)
    uint32_t base = 0, my_eq = 0;
    for (uint32_t i0 = 0; i0 < m; i0 += LB) {
        const uint32_t i = i0 + threadIdx.x;
        const bool keep = i < m && (i + 1 == m || s_ts[i] != s_ts[i + 1]);
        uint32_t tot;
        const uint32_t r = block_scan(keep ? 1u : 0u, s_w, &tot);
        if (keep) {
            const int64_t ts = s_ts[i];
            const uint64_t lb = lower_bound_g(in.l_ts + lb0, nl, ts);
            const bool eq = lb < nl && in.l_ts[lb0 + lb] == ts;
            const uint64_t o = c0 + base + r;
            k_lb[o] = (uint32_t)lb;
            k_j[o] = s_j[i];
            k_eq[o] = eq ? 1 : 0;
            my_eq += eq ? 1u : 0u;
        }
        base += tot;
    }
    const uint32_t kept_total = base;
    uint32_t eq_total;
    (void)block_scan(my_eq, s_w, &eq_total);
    if (threadIdx.x == 0) {
        kcnt[p] = kept_total;
        cnt[p] = (uint32_t)(nl + kept_total - eq_total);
    }
}

// upper_bound / lower_bound over the kept list's lb (ascending) in LDS
__device__ __forceinline__ uint32_t ub_u32(const uint32_t *a, uint32_t n, uint32_t x) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] <= x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ uint32_t lb_u32(const uint32_t *a, uint32_t n, uint32_t x) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(LB) void k_la_write(crdt_local_in in, const uint32_t *__restrict__ k_lb,
                                                 const uint32_t *__restrict__ k_j, const uint8_t *__restrict__ k_eq,
                                                 const uint32_t *__restrict__ kcnt, crdt_local_out out) {
    __shared__ uint32_t s_lb[kMaxCmd];
    __shared__ uint32_t s_ep[kMaxCmd + 1];               // eq prefix: s_ep[c] = #eq among kept [0, c)
    __shared__ uint32_t s_w[LB / 64];
    const uint32_t p = blockIdx.x;
    const uint64_t lb0 = in.l_off[p], nl = in.l_off[p + 1] - lb0;
    const uint64_t c0 = in.c_off[p];
    const uint32_t k = kcnt[p];
    if (k > kMaxCmd) return;                             // kSkip: an empty range, nothing may land in it
    const uint64_t ob = out.off[p];
    uint32_t base = 0;
    for (uint32_t i0 = 0; i0 < k; i0 += LB) {            // (k <= kMaxCmd)
        const uint32_t c = i0 + threadIdx.x;
        const uint32_t e = c < k ? k_eq[c0 + c] : 0;
        if (c < k) s_lb[c] = k_lb[c0 + c];
        uint32_t tot;
        const uint32_t r = block_scan(e, s_w, &tot);
        if (c < k) s_ep[c] = base + r;
        base += tot;
    }
    if (threadIdx.x == 0) s_ep[k] = base;
    __syncthreads();
    for (uint32_t c = threadIdx.x; c < k; c += LB) {     // the kept commands
        const uint64_t pos = ob + s_lb[c] + c - s_ep[c];
        const uint64_t j = c0 + k_j[c0 + c];
        out.ts[pos] = in.c_ts[j];
        out.origin[pos] = 1;                             // a *Command (main.go:187)
        out.src[pos] = -(int64_t)j - 1;
    }
    for (uint64_t i = threadIdx.x; i < nl; i += LB) {    // the Diff's entries, shifted
        const uint32_t ii = (uint32_t)i;
        const uint32_t a = ub_u32(s_lb, k, ii);          // kept commands before entry i
        if (a && s_lb[a - 1] == ii && k_eq[c0 + a - 1]) continue;   // replaced by a same-ts command
        const uint32_t d = s_ep[lb_u32(s_lb, k, ii)];    // replaced entries before i
        const uint64_t pos = ob + i + a - d;
        out.ts[pos] = in.l_ts[lb0 + i];
        out.origin[pos] = in.l_origin[lb0 + i];
        out.src[pos] = (int64_t)(lb0 + i);
    }
}

// CurrentState apply (main.go:188-207), sequential per replica.
__global__ void k_la_state(crdt_local_in in, const LaOk *__restrict__ okv, const uint32_t *__restrict__ kcnt,
                           crdt_local_out out) {
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    if (p >= in.replicas) return;
    if (kcnt[p] == kSkip) {                              // over the limit: the state is left as it was, so a
        for (uint64_t j = in.c_off[p]; j < in.c_off[p + 1]; ++j) out.status[j] = 0;   // split retry applies once
        return;
    }
    for (uint64_t j = in.c_off[p]; j < in.c_off[p + 1]; ++j) {
        uint16_t status = 200;
        for (uint64_t q = in.c_kv[j]; q < in.c_kv[j + 1]; ++q) {
            const uint32_t slot = in.kv_key[q], v = in.kv_val[q];
            if (slot >= in.n_slots || v >= in.n_str) continue;   // malformed pair: ignored
            const uint8_t kind = out.st_kind[slot];
            if (kind == 0) {                             // absent: set verbatim, RETURN (main.go:189-193)
                out.st_kind[slot] = 1;
                out.st_str[slot] = v;
                break;
            }
            int64_t curr;
            if (kind == 2) {
                curr = out.st_sum[slot];                 // Atoi(Itoa(sum)) == sum
            } else {
                const LaOk o = okv[out.st_str[slot]];
                if (!o.ok) { status = 500; break; }      // main.go:195-199
                curr = o.val;
            }
            const LaOk c = okv[v];
            if (!c.ok) { status = 500; break; }          // main.go:200-204
            out.st_kind[slot] = 2;
            out.st_sum[slot] = (int64_t)((uint64_t)curr + (uint64_t)c.val);   // wraps (main.go:205)
        }
        out.status[j] = status;
    }
}

}  // namespace
}  // namespace crdt

using namespace crdt;

extern "C" int crdt_local_apply(crdt_ctx *ctx, const crdt_local_in *inp, const crdt_local_out *outp) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!inp || !outp) return CRDT_E_INVAL;
    const crdt_local_in in = *inp;
    const crdt_local_out out = *outp;
    if (in.replicas == 0) return CRDT_OK;
    if (!in.l_off || !in.c_off || !out.off) return CRDT_E_INVAL;
    if (in.n_l && (!in.l_ts || !in.l_origin)) return CRDT_E_INVAL;
    if (in.n_c && (!in.c_ts || !in.c_kv || !out.status)) return CRDT_E_INVAL;
    if (in.n_l + in.n_c && (!out.ts || !out.origin || !out.src)) return CRDT_E_INVAL;
    if (in.n_slots && (!out.st_kind || !out.st_str || !out.st_sum)) return CRDT_E_INVAL;
    if (in.n_str && (!in.str_bytes || !in.str_off)) return CRDT_E_INVAL;
    if (in.n_kv && (!in.kv_key || !in.kv_val)) return CRDT_E_INVAL;
    if (in.n_l + in.n_c >= 0xFFFFFFFFull) return CRDT_E_RANGE;   // u32 per-replica lengths and positions
    const size_t np = in.replicas, nc = in.n_c;
    const size_t need = Carve::round(nc * 4 + 4) * 2 + Carve::round(nc + 1) + Carve::round(np * 4 + 4) * 2 +
                        Carve::round((in.n_str + 1) * sizeof(LaOk)) + scan_tmp_bytes(np) + 1024;
    rc = ws_reserve(ctx, need);
    if (rc) return rc;
    Carve w(ctx->ws);
    uint32_t *k_lb = w.take<uint32_t>(nc + 1);
    uint32_t *k_j = w.take<uint32_t>(nc + 1);
    uint8_t *k_eq = w.take<uint8_t>(nc + 1);
    uint32_t *kcnt = w.take<uint32_t>(np + 1);
    uint32_t *cnt = w.take<uint32_t>(np + 1);
    LaOk *okv = w.take<LaOk>(in.n_str + 1);
    void *tmp = w.take<char>(scan_tmp_bytes(np));
    const hipStream_t s = ctx->stream;
    if (in.n_str)
        k_la_atoi<<<grid_for(in.n_str, 256, (unsigned)ctx->num_cus * 4), 256, 0, s>>>(in.str_bytes, in.str_off,
                                                                                      in.n_str, okv);
    k_la_plan<<<(unsigned)np, LB, 0, s>>>(in, k_lb, k_j, k_eq, kcnt, cnt, ctx->dev_status);
    rc = check_launch(ctx);
    if (rc) return rc;
    rc = exclusive_scan_u32(ctx, cnt, out.off, np, tmp);     // out.off[np] = new Diff total
    if (rc) return rc;
    k_la_write<<<(unsigned)np, LB, 0, s>>>(in, k_lb, k_j, k_eq, kcnt, out);
    if (nc) k_la_state<<<grid_for(np, 256, 1u << 30), 256, 0, s>>>(in, okv, kcnt, out);
    return check_launch(ctx);
}
