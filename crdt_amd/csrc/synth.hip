// synth.hip -- seeded synthetic replica state, generated in HBM.
// Element i of every stream is a pure function of (seed, stream, i), so any
// shard or sample can be regenerated independently on host (crdt_amd/synth.py)
// or device, and multi-GPU ranks generate only their own rows.
#include "common.hpp"

namespace crdt {

__device__ __forceinline__ uint64_t counter_value(uint64_t k, uint64_t i) {
    const uint64_t x = rnd(k, i);
    if ((x & 0x3FF) == 0x3FF) {                        // ~1/1024: planted edge values
        switch ((x >> 10) & 3) {
            case 0: return 0ULL;
            case 1: return 0x7FFFFFFFFFFFFFFFULL;      // 2^63 - 1
            case 2: return 0x8000000000000000ULL;      // 2^63 (sign bit: unsigned compare)
            default: return 0xFFFFFFFFFFFFFFFFULL;     // 2^64 - 1
        }
    }
    if ((x >> 61) == 0) return rnd(k ^ 0xA5A5A5A5A5A5A5A5ULL, i);   // 1/8 full range
    return (x >> 20) & 0xFFFFF;                                      // rest < 2^20
}

__global__ void k_synth_counters(uint64_t k, uint64_t *out, size_t n, uint64_t base) {
    for (size_t j = (size_t)blockIdx.x * 256 + threadIdx.x; j < n; j += (size_t)gridDim.x * 256)
        out[j] = counter_value(k, base + j);
}

__global__ void k_synth_vclock(uint64_t kb, uint64_t kc, uint64_t *a, uint64_t *b, size_t pairs,
                               size_t nodes, uint64_t pair_base) {
    const size_t n = pairs * nodes;
    for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (size_t)gridDim.x * 256) {
        const size_t j = e / nodes, kk = e % nodes;
        const uint64_t p = pair_base + j;
        uint64_t base = rnd(kb, p * nodes + kk) & 0xFFFFFFFFULL;
        const uint64_t h = rnd(kc, p);
        const unsigned cls = (unsigned)(h & 3);
        const size_t jj = nodes > 1 ? (size_t)((h >> 8) % (nodes - 1)) : 0;
        if (((h >> 32) & 1023) == 0) base = 0xFFFFFFFFFFFFFFFEULL - (base & 0xFF);   // near 2^64
        uint64_t x = base, y = base;
        const size_t last = nodes - 1;
        if (cls == 1 && kk == last) y += 1;                  // BEFORE: differs only at the last node
        if (cls == 2 && kk == last) x += 1;                  // AFTER
        if (cls == 3) {                                      // CONCURRENT
            if (kk == last) y += 1;
            if (kk == jj) x += 1;
        }
        a[e] = x;
        b[e] = y;
    }
}

__global__ void k_synth_sets(uint64_t seed, uint32_t side, uint64_t *key, uint64_t *ts, uint32_t *rep,
                             uint8_t *tomb, size_t n, uint64_t key_space) {
    const uint64_t s0 = side * 8;
    const uint64_t kkey = stream_key(seed, 20 + s0), kts = stream_key(seed, 21 + s0);
    const uint64_t krep = stream_key(seed, 22 + s0), ktomb = stream_key(seed, 23 + s0);
    const uint64_t kkey0 = stream_key(seed, 20), kts0 = stream_key(seed, 21), krep0 = stream_key(seed, 22);
    const uint64_t kdup = stream_key(seed, 40);
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        uint64_t kv = rnd(kkey, i) % key_space, tv = rnd(kts, i) & 0xFFFFF;
        uint32_t rv = (uint32_t)(rnd(krep, i) & 63);
        if (side != 0 && rnd(kdup, i) % 20 == 0) {           // 5%: the same tag as side 0's i-th
            kv = rnd(kkey0, i) % key_space;
            tv = rnd(kts0, i) & 0xFFFFF;
            rv = (uint32_t)(rnd(krep0, i) & 63);
        }
        key[i] = kv;
        ts[i] = tv;
        rep[i] = rv;
        tomb[i] = (uint8_t)(rnd(ktomb, i) % 10 == 0);        // 10% tombstones
    }
}

}  // namespace crdt

using namespace crdt;

extern "C" int crdt_synth_counters(crdt_ctx *ctx, uint64_t seed, uint32_t stream, uint64_t *out, size_t n,
                                   uint64_t index_base) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (n == 0) return CRDT_OK;
    if (!out) return CRDT_E_INVAL;
    k_synth_counters<<<grid_for(n, 256, (unsigned)ctx->num_cus * 16), 256, 0, ctx->stream>>>(
        stream_key(seed, stream), out, n, index_base);
    return check_launch(ctx);
}

extern "C" int crdt_synth_vclock_pairs(crdt_ctx *ctx, uint64_t seed, uint64_t *a, uint64_t *b, size_t pairs,
                                       size_t nodes, uint64_t pair_base) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (nodes == 0 || mul_overflows(pairs, nodes)) return CRDT_E_INVAL;
    if (pairs == 0) return CRDT_OK;
    if (!a || !b) return CRDT_E_INVAL;
    k_synth_vclock<<<grid_for(pairs * nodes, 256, (unsigned)ctx->num_cus * 16), 256, 0, ctx->stream>>>(
        stream_key(seed, 10), stream_key(seed, 11), a, b, pairs, nodes, pair_base);
    return check_launch(ctx);
}

extern "C" int crdt_synth_set_tuples(crdt_ctx *ctx, uint64_t seed, uint32_t side, const crdt_tuples *out,
                                     size_t n, uint64_t key_space) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (n == 0) return CRDT_OK;
    if (!out || !out->key || !out->ts || !out->rep || !out->tomb || key_space == 0) return CRDT_E_INVAL;
    k_synth_sets<<<grid_for(n, 256, (unsigned)ctx->num_cus * 16), 256, 0, ctx->stream>>>(
        seed, side, out->key, out->ts, out->rep, out->tomb, n, key_space);
    return check_launch(ctx);
}
