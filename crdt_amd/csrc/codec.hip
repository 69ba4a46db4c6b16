// codec.hip -- the gossip pull decoded on the device.
//
// The reference's pull (main.go:245-256) decodes the peer's whole Diff
// (Diff.ToJSON, main.go:159) into RemoteDiff and merges (main.go:257).  The
// build's binary SoA form of that body (crdt_server_gossip_binary:
// "CRDTSOA1", u64 n_entries, n_pairs, n_bytes, i64 ts[], u32 pairs[],
// u32 klen[], u32 vlen[], bytes) lands here in HBM as raw bytes and is turned
// straight into the crdt_refmerge_in R arrays:
//   r_ts[e]            = ts[i]
//   r_kv[e]            = kv_base + exclusive scan of pairs[]
//   kv_key[kv_base+j]  = slot_base(body) + id of key j in a KEY table
//   kv_val[kv_base+j]  = id of value j in a VALUE table (the merge's string arena)
// Strings are interned into device string tables (crdt_strtab): open
// addressing over 64-bit entries {hash32, id | pending-pair}, ids dense in
// first-seen order, bytes in an append-only arena with str_off offsets.
// Interning is three passes with no intra-kernel publication beyond the
// claim CAS itself: (A) every pair finds its string or CLAIMS an empty entry
// tagged with its own pair index (equal strings compare bytes against the
// claimer's bytes, which are in the immutable body); (B) claimers get dense
// ids by a scan, copy their bytes into the arena and turn the entry into the
// id; (C) every pair reads its entry's id.  Bodies the device path does not
// take (a nil map, ts not ascending, keys of an entry not strictly ascending,
// a key beyond the caller's slot range, a full table) are flagged per body:
// the host decodes those (crdt_server_ingest_binary), as the reference would.
#include <string.h>

#include <functional>
#include <vector>

#include "scan.hpp"

struct crdt_strtab {
    int device = 0;
    uint64_t *tab = nullptr;      // [H] entries, kEmpty or hash32 << 32 | tag << 31 | payload
    uint64_t H = 0;               // power of two
    uint8_t *bytes = nullptr;
    uint64_t cap_bytes = 0;
    uint64_t *off = nullptr;      // [cap_n + 1]: off[id], off[n] = bytes used
    uint64_t cap_n = 0;
    uint64_t n = 0, nbytes = 0;   // host-known (after each synchronising call)
    std::vector<uint8_t> h_bytes; // host mirror of the arena (append-only)
    std::vector<uint64_t> h_off{0};
};

namespace crdt {
namespace {

constexpr uint64_t kEmptyE = ~0ull;
constexpr uint32_t kPend = 0x80000000u;
constexpr uint32_t kIdMask = 0x7FFFFFFFu;
constexpr uint32_t kNilPairs = 0xFFFFFFFFu;
constexpr uint32_t kEmptyE32 = 0xFFFFFFFFu;  // a pair's slot record: resolved in pass A
constexpr uint32_t kRepBit = 0x80000000u;    // the pair claimed the entry (tables < 2^31 entries)

enum : uint32_t {
    kBodyMalformed = 1u,          // sizes / counts inconsistent: nothing of the body is usable
    kBodyHost = 2u,               // valid, but the device path does not take it (host decode)
    kBodyFull = 4u,               // a string table was full (grow and retry, or host decode)
};

__device__ __forceinline__ uint32_t hash32(const uint8_t *p, uint32_t n) {
    uint32_t h = 2166136261u;                          // FNV-1a
    for (uint32_t i = 0; i < n; ++i) h = (h ^ p[i]) * 16777619u;
    return h;
}

__device__ __forceinline__ uint32_t le32(const uint8_t *p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}
__device__ __forceinline__ uint64_t le64(const uint8_t *p) { return (uint64_t)le32(p) | (uint64_t)le32(p + 4) << 32; }

__device__ __forceinline__ bool bytes_eq(const uint8_t *a, const uint8_t *b, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i)
        if (a[i] != b[i]) return false;
    return true;
}

// strictly ascending as byte strings (Go string order)
__device__ __forceinline__ bool bytes_lt(const uint8_t *a, uint32_t na, const uint8_t *b, uint32_t nb) {
    const uint32_t n = na < nb ? na : nb;
    for (uint32_t i = 0; i < n; ++i)
        if (a[i] != b[i]) return a[i] < b[i];
    return na < nb;
}

// Bytes [p, p + n) (n <= 8) as a zero-padded little-endian u64, read by the
// one or two naturally aligned 8-byte words that hold them: one load (two
// when the string crosses a word) instead of a dependent load per byte; an
// aligned word that holds a byte of the string never leaves its page.
__device__ __forceinline__ uint64_t load_short(const uint8_t *p, uint32_t n) {
    if (n == 0) return 0;
    // (pointer arithmetic, not integer casts: the loads stay global loads)
    const uint32_t sh = (uint32_t)((uintptr_t)p & 7);
    const uint64_t *base = reinterpret_cast<const uint64_t *>(p - sh);
    uint64_t v = base[0] >> (8 * sh);
    if (sh + n > 8) v |= base[1] << (8 * (8 - sh));
    return n == 8 ? v : (v & ((1ull << (8 * n)) - 1));
}
__device__ __forceinline__ uint32_t hash32_short(uint64_t v, uint32_t n) {   // == hash32 of the n bytes
    uint32_t h = 2166136261u;
    for (uint32_t i = 0; i < n; ++i) h = (h ^ (uint32_t)((v >> (8 * i)) & 0xFF)) * 16777619u;
    return h;
}
// a < b as byte strings, both packed by load_short: big-endian order of the
// zero-padded bytes, the shorter first on equal padded values (a prefix)
__device__ __forceinline__ bool short_lt(uint64_t a, uint32_t na, uint64_t b, uint32_t nb) {
    const uint64_t A = __builtin_bswap64(a), B = __builtin_bswap64(b);
    return A != B ? A < B : na < nb;
}

// A table's H entries are followed by H short forms: entry i's string, when
// it has an id and at most 7 bytes, packed as load_short does with its length
// in the top byte (kNoShort otherwise), so a lookup of a short string that
// hits a resolved entry compares one word loaded beside the entry instead of
// walking entry -> offsets -> bytes (codec.short_tab).
constexpr uint64_t kNoShort = ~0ull;
__device__ __forceinline__ uint64_t short_form(uint64_t packed, uint32_t n) {
    return n <= 7 ? packed | (uint64_t)n << 56 : kNoShort;
}
__device__ __forceinline__ uint64_t short_form_bytes(const uint8_t *p, uint32_t n) {
    if (n > 7) return kNoShort;
    uint64_t v = 0;
    for (uint32_t i = 0; i < n; ++i) v |= (uint64_t)p[i] << (8 * i);
    return v | (uint64_t)n << 56;
}

struct TabView {
    uint64_t *tab;                 // [mask + 1] entries, then [mask + 1] short forms
    uint64_t mask;
    const uint8_t *bytes;
    const uint64_t *off;
};

// Pass A: find the string or claim an empty entry for pending reference
// `self`.  get(ref, &p, &len) returns the bytes of a pending reference.
// Returns the entry index (kEmptyE as uint64 on a full table); *rep = claimed.
template <class Get>
__device__ uint64_t tab_claim(const TabView &t, uint32_t h, const uint8_t *s, uint32_t len, uint32_t self,
                              const Get &get, bool *rep, uint64_t *ent, uint64_t sv, bool use_short = false) {
    // sv: the string packed by load_short when len <= 8 (compares then load
    // the candidate's bytes as one word too)
    *rep = false;
    uint64_t i = h & t.mask;
    const uint64_t want_s = use_short ? short_form(sv, len) : kNoShort;
    for (uint64_t probe = 0; probe <= t.mask; ++probe, i = (i + 1) & t.mask) {
        // a plain load first: ids from earlier calls never change inside a
        // pass; an entry it shows empty may have been claimed meanwhile (the
        // CAS then returns the claim).  Its short form is loaded beside it.
        uint64_t e = t.tab[i];
        const uint64_t es = want_s != kNoShort ? t.tab[t.mask + 1 + i] : kNoShort;
        if (es != kNoShort && e != kEmptyE && !((uint32_t)e & kPend)) {   // a resolved short string: one compare
            if (es == want_s) {
                *ent = e;
                return i;
            }
            continue;
        }
        if (e == kEmptyE) {
            const uint64_t want = (uint64_t)h << 32 | kPend | self;
            const uint64_t old = atomicCAS((unsigned long long *)&t.tab[i], (unsigned long long)kEmptyE,
                                           (unsigned long long)want);
            if (old == kEmptyE) {
                *rep = true;
                *ent = want;
                return i;
            }
            e = old;
        }
        if ((uint32_t)(e >> 32) != h) continue;
        const uint32_t pay = (uint32_t)e;
        const uint8_t *q;
        uint32_t qn;
        if (pay & kPend) {
            get(pay & kIdMask, &q, &qn);
        } else {
            const uint32_t id = pay & kIdMask;
            q = t.bytes + t.off[id];
            qn = (uint32_t)(t.off[id + 1] - t.off[id]);
        }
        if (qn == len && (len <= 8 ? load_short(q, qn) == sv : bytes_eq(q, s, len))) {
            *ent = e;
            return i;
        }
    }
    return kEmptyE;
}

// ---------------------------------------------------------------- bodies
struct BodyDesc {                  // one pulled body
    uint64_t data;                 // its address minus DecodeCtx::data (mod 2^64: bodies may sit in separate buffers)
    uint64_t e0, q0;               // first global entry / pair of the body
    uint64_t ne, np, nb;
    uint32_t slot_base;
    uint32_t pad;
    uint64_t y0;                   // the body's first byte in the pair-byte scan (boff): header n_bytes before it
};

__device__ __forceinline__ const uint8_t *body_ptr(const uint8_t *data, uint64_t at) {
    return data + at;                                  // (mod 2^64, as the offsets are)
}

__device__ __forceinline__ uint32_t find_body(const BodyDesc *b, uint32_t nbody, uint64_t x, bool pairs) {
    uint32_t lo = 0, hi = nbody;                     // last body whose first item <= x
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((pairs ? b[mid].q0 : b[mid].e0) <= x) lo = mid;
        else hi = mid;
    }
    return lo;
}

struct DecodeCtx {
    const uint8_t *data;
    const BodyDesc *bd;
    uint32_t nbody;
    uint32_t *flag;                // [nbody]
    const uint64_t *boff;          // [n_pairs + 1] scan of (klen + vlen) over all pairs
    const uint32_t *klen;          // [n_pairs]
    uint64_t n_pairs;
    unsigned long long *multi;     // entries whose pair count is not 1 (the one-pair invariant of population.hip)
    // pair j: key bytes and value bytes, clamped to the body's byte region
    // (lengths that overrun it mark the body malformed: never read past it)
    __device__ void pair_bytes(uint64_t j, const uint8_t **kp, uint32_t *kn, const uint8_t **vp, uint32_t *vn) const {
        const uint32_t b = find_body(bd, nbody, j, true);
        const BodyDesc d = bd[b];
        const uint8_t *region = body_ptr(data, d.data) + 32 + 12 * d.ne + 8 * d.np;
        const uint64_t o = boff[j] - boff[d.q0];
        const uint64_t k = klen[j], v = boff[j + 1] - boff[j] - k;
        if (o > d.nb || k > d.nb - o || v > d.nb - o - k) {
            atomicOr(&flag[b], kBodyMalformed);
            *kp = *vp = region;
            *kn = *vn = 0;
            return;
        }
        *kp = region + o;
        *kn = (uint32_t)k;
        *vp = region + o + k;
        *vn = (uint32_t)v;
    }
};

constexpr uint32_t kChunk = 1024;  // items per workgroup of the body-major grids (grid.y = body)
// pairs per workgroup of the claim pass: one per thread -- each pair's two
// table claims are a chain of dependent memory-side atomics and string
// compares, so pairs run side by side, not four deep per thread
constexpr uint32_t kClaimChunk = 256;

// per entry: ts, pair count; ts must ascend strictly within a body, no nil map
__global__ __launch_bounds__(256) void k_dec_entries(DecodeCtx c, int64_t *__restrict__ r_ts,
                                                     uint32_t *__restrict__ cnt) {
    const uint32_t b = blockIdx.y;
    const BodyDesc d = c.bd[b];
    const uint8_t *base = body_ptr(c.data, d.data) + 32;
    bool host = false;
    uint32_t multi = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kChunk + threadIdx.x; i < d.ne && i < (uint64_t)(blockIdx.x + 1) * kChunk;
         i += 256) {
        const int64_t ts = (int64_t)le64(base + 8 * i);
        uint32_t k = le32(base + 8 * d.ne + 4 * i);
        if (k == kNilPairs) {                             // a nil map: the host path keeps its flag
            host = true;
            k = 0;
        }
        if (i && (int64_t)le64(base + 8 * (i - 1)) >= ts) host = true;
        multi += k != 1;
        r_ts[d.e0 + i] = ts;
        cnt[d.e0 + i] = k;
    }
    if (__any(host) && (threadIdx.x & 63) == __ffsll((unsigned long long)__ballot(host)) - 1)
        atomicOr(&c.flag[b], kBodyHost);
    for (int m = 32; m >= 1; m >>= 1) multi += __shfl_xor(multi, m, 64);
    if ((threadIdx.x & 63) == 0 && multi && c.multi) atomicAdd(c.multi, (unsigned long long)multi);
}

// per pair: klen and klen + vlen (u32; an overflow marks the body malformed)
__global__ __launch_bounds__(256) void k_dec_pairs(DecodeCtx c, uint32_t *__restrict__ klen,
                                                   uint32_t *__restrict__ plen, uint8_t *__restrict__ first) {
    const uint32_t b = blockIdx.y;
    const BodyDesc d = c.bd[b];
    const uint8_t *base = body_ptr(c.data, d.data) + 32 + 12 * d.ne;
    for (uint64_t q = (uint64_t)blockIdx.x * kChunk + threadIdx.x; q < d.np && q < (uint64_t)(blockIdx.x + 1) * kChunk;
         q += 256) {
        const uint32_t kl = le32(base + 4 * q), vl = le32(base + 4 * d.np + 4 * q);
        const uint64_t t = (uint64_t)kl + vl;
        if (t > 0xFFFFFFFFull) atomicOr(&c.flag[b], kBodyMalformed);
        klen[d.q0 + q] = kl;
        plen[d.q0 + q] = t > 0xFFFFFFFFull ? 0u : (uint32_t)t;
        first[d.q0 + q] = 0;                              // (k_dec_kv marks the entries' first pairs)
    }
}

// ---- the decode of a few small bodies in one pass (gossip_decode_at picks it
// when every body fits kSmallItems entries and pairs): two 1024-thread
// workgroups per body, one for its pairs (k_dec_pairs and the byte scan) and
// one for its entries (k_dec_entries, the count scan, k_dec_kv, the `first`
// marks), each checking its half of k_dec_bodies.  The scans are body-local:
// r_kv and `first` are relative to the body's first pair, and boff is the
// body's own scan based at y0 (the header byte counts of the bodies before
// it; a body whose real lengths disagree with its header is flagged and
// claims nothing, so its boundary slot -- written by both neighbours with the
// same value -- never matters).  Eight launches and their host calls fewer
// for the Server.merge() shapes; large batches keep the multi-pass form.
constexpr int kSmallT = 1024, kSmallR = 8;
constexpr uint64_t kSmallItems = 1u << 18;

__device__ __forceinline__ uint64_t block1024_exclusive_scan(uint64_t v, uint64_t *total, uint64_t *wsum) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint64_t off = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kSmallT / 64; ++k) {
        const uint64_t s = wsum[k];
        off += k < w ? s : 0;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return off + x - v;
}

template <bool AL>
__device__ __forceinline__ void dec_small(DecodeCtx c, int64_t *__restrict__ r_ts,
                                                       uint32_t *__restrict__ klen, uint64_t *__restrict__ boff,
                                                       uint8_t *__restrict__ first, uint64_t n_e, uint64_t n_p,
                                                       uint64_t kv_base, uint64_t *__restrict__ r_kv,
                                                       uint64_t *__restrict__ r_off, const BodyDesc &d,
                                                       uint64_t *wsum, uint32_t b, bool entries) {
    const uint32_t tid = threadIdx.x;
    if (tid == 0 && entries) {
        r_off[b] = d.e0;                                 // (the multi-pass form uploads these)
        if (b == 0) {
            r_off[c.nbody] = n_e;
            r_kv[n_e] = kv_base + n_p;
        }
    }
    const uint8_t *base = body_ptr(c.data, d.data) + 32;
    auto ld32 = [&](const uint8_t *p) { return AL ? *(const uint32_t *)p : le32(p); };
    auto ld64 = [&](const uint8_t *p) { return AL ? *(const uint64_t *)p : le64(p); };
    bool bad = false, host = false;
    uint32_t multi = 0;                                  // entries whose pair count is not 1
    uint64_t carry = 0;
    if (!entries) {
    // pairs: klen and the scan of klen + vlen into boff.  Each thread takes
    // kSmallR consecutive items of a chunk (its own prefix in registers): one
    // workgroup scan per chunk of kSmallT * kSmallR items.  The next chunk's
    // loads are issued before this chunk's stores, so the wait for them does
    // not also wait for the stores (one memory counter covers both).
    const uint8_t *pk = base + 12 * d.ne, *pv = pk + 4 * d.np;
    constexpr uint64_t CH = (uint64_t)kSmallT * kSmallR;
    uint32_t kl[kSmallR], vl[kSmallR];
    auto load = [&](uint64_t c0) {
        const uint64_t i0 = c0 + (uint64_t)tid * kSmallR;
#pragma unroll
        for (int r = 0; r < kSmallR; ++r) {
            const bool in = i0 + r < d.np;
            kl[r] = in ? ld32(pk + 4 * (i0 + r)) : 0;
            vl[r] = in ? ld32(pv + 4 * (i0 + r)) : 0;
        }
    };
    if (d.np) load(0);
    for (uint64_t c0 = 0; c0 < d.np; c0 += CH) {
        const uint64_t i0 = c0 + (uint64_t)tid * kSmallR;
        uint32_t t[kSmallR], k0[kSmallR];
        uint64_t sum = 0;
#pragma unroll
        for (int r = 0; r < kSmallR; ++r) {
            const uint64_t x = (uint64_t)kl[r] + vl[r];
            if (x > 0xFFFFFFFFull) bad = true;
            t[r] = x > 0xFFFFFFFFull ? 0u : (uint32_t)x;
            k0[r] = kl[r];
            sum += t[r];
        }
        uint64_t tot;
        uint64_t run = carry + block1024_exclusive_scan(sum, &tot, wsum);
        if (c0 + CH < d.np) load(c0 + CH);
#pragma unroll
        for (int r = 0; r < kSmallR; ++r) {
            if (i0 + r < d.np) {
                klen[d.q0 + i0 + r] = k0[r];
                boff[d.q0 + i0 + r] = d.y0 + run;
            }
            run += t[r];
        }
        carry += tot;
    }
    if (carry != d.nb) bad = true;
    if (tid == 0) boff[d.q0 + d.np] = d.y0 + d.nb;
    } else {
    // entries: ts, pair counts (nil map / not ascending: the host path), the
    // body-local scan of the counts into r_kv and `first` of every pair (1
    // on an entry's first pair; pairs no entry covers only occur in a body
    // whose counts disagree with its header, flagged here: it claims nothing)
    for (uint64_t c0 = 0; c0 < d.ne; c0 += (uint64_t)kSmallT * kSmallR) {
        const uint64_t i0 = c0 + (uint64_t)tid * kSmallR;
        uint32_t k[kSmallR];
        uint64_t sum = 0;
        int64_t prev = i0 && i0 < d.ne ? (int64_t)ld64(base + 8 * (i0 - 1)) : 0;
#pragma unroll
        for (int r = 0; r < kSmallR; ++r) {
            const uint64_t i = i0 + r;
            k[r] = 0;
            if (i < d.ne) {
                const int64_t ts = (int64_t)ld64(base + 8 * i);
                uint32_t kk = ld32(base + 8 * d.ne + 4 * i);
                if (kk == kNilPairs) {
                    host = true;
                    kk = 0;
                }
                if (i && prev >= ts) host = true;
                prev = ts;
                r_ts[d.e0 + i] = ts;
                k[r] = kk;
                multi += kk != 1;
            }
            sum += k[r];
        }
        uint64_t tot;
        uint64_t run = carry + block1024_exclusive_scan(sum, &tot, wsum);
#pragma unroll
        for (int r = 0; r < kSmallR; ++r) {
            const uint64_t i = i0 + r;
            if (i < d.ne) {
                r_kv[d.e0 + i] = kv_base + d.q0 + run;
                for (uint32_t j = 0; j < k[r] && run + j < d.np; ++j) first[d.q0 + run + j] = j == 0;
            }
            run += k[r];
        }
        carry += tot;
    }
    if (carry != d.np) bad = true;
    }
    const uint32_t fl = (bad ? kBodyMalformed : 0u) | (host ? kBodyHost : 0u);
    uint32_t wfl = fl;
    for (int m = 32; m >= 1; m >>= 1) {
        wfl |= __shfl_xor(wfl, m, 64);
        multi += __shfl_xor(multi, m, 64);
    }
    if ((tid & 63) == 0 && wfl) atomicOr(&c.flag[b], wfl);
    if ((tid & 63) == 0 && multi && c.multi) atomicAdd(c.multi, (unsigned long long)multi);
}

__global__ __launch_bounds__(kSmallT) void k_dec_small(DecodeCtx c, int64_t *__restrict__ r_ts,
                                                       uint32_t *__restrict__ klen, uint64_t *__restrict__ boff,
                                                       uint8_t *__restrict__ first, uint64_t n_e, uint64_t n_p,
                                                       uint64_t kv_base, uint64_t *__restrict__ r_kv,
                                                       uint64_t *__restrict__ r_off) {
    __shared__ uint64_t wsum[kSmallT / 64];
    const uint32_t b = blockIdx.x >> 1;                  // two workgroups per body: its pairs, its entries
    const bool entries = blockIdx.x & 1;
    const BodyDesc d = c.bd[b];
    // word loads for a body at an 8-byte aligned address (every body the
    // Server path uploads), byte loads otherwise
    if ((((uintptr_t)body_ptr(c.data, d.data)) & 7) == 0)
        dec_small<true>(c, r_ts, klen, boff, first, n_e, n_p, kv_base, r_kv, r_off, d, wsum, b, entries);
    else
        dec_small<false>(c, r_ts, klen, boff, first, n_e, n_p, kv_base, r_kv, r_off, d, wsum, b, entries);
}

// The same one-pass decode for large batches (codec.small = 3): dec_small's
// per-thread item runs (kSmallR consecutive items, so its scans stay
// thread-local) are uncoalesced -- each load and store instruction spans
// 64 x kSmallR items.  Here every global access is coalesced (item
// c0 + r kSmallT + tid) and only the scanned values change layout, through
// one padded LDS buffer: the counts in, the prefixes out.
constexpr uint32_t kBigCH = (uint32_t)kSmallT * kSmallR;   // items per chunk at R = kSmallR (the LDS buffer's size)
__device__ __forceinline__ uint32_t big_pad(uint32_t i) { return i + (i >> 3); }
// block1024_exclusive_scan with the per-wave sums combined by shuffles (the
// sixteen sums in lanes, not in sixteen registers of every thread)
__device__ __forceinline__ uint64_t big_exclusive_scan(uint64_t v, uint64_t *total, uint64_t *wsum) {
    constexpr int NW = kSmallT / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    const uint64_t ws = lane < NW ? wsum[lane] : 0;
    uint64_t z = ws;
#pragma unroll
    for (int d = 1; d < NW; d <<= 1) {
        const uint64_t y = __shfl_up(z, d, 64);
        if (lane >= d) z += y;
    }
    const uint64_t off = __shfl(z - ws, w, 64);         // the sums of the waves before this one
    *total = __shfl(z, NW - 1, 64);
    __syncthreads();                                     // (wsum is the next call's)
    return off + x - v;
}

template <int R, bool AL, bool entries>
__device__ __forceinline__ void dec_big(DecodeCtx c, int64_t *__restrict__ r_ts, uint32_t *__restrict__ klen,
                                        uint64_t *__restrict__ boff, uint8_t *__restrict__ first, uint64_t n_e,
                                        uint64_t n_p, uint64_t kv_base, uint64_t *__restrict__ r_kv,
                                        uint64_t *__restrict__ r_off, const BodyDesc &d, uint64_t *wsum,
                                        uint64_t *buf, uint32_t b) {
    constexpr uint32_t CH = (uint32_t)kSmallT * R;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    uint32_t *buf32 = reinterpret_cast<uint32_t *>(buf);
    if (tid == 0 && entries) {
        r_off[b] = d.e0;
        if (b == 0) {
            r_off[c.nbody] = n_e;
            r_kv[n_e] = kv_base + n_p;
        }
    }
    const uint8_t *base = body_ptr(c.data, d.data) + 32;
    auto ld32 = [&](const uint8_t *p) { return AL ? *(const uint32_t *)p : le32(p); };
    auto ld64 = [&](const uint8_t *p) { return AL ? *(const uint64_t *)p : le64(p); };
    bool bad = false, host = false;
    uint32_t multi = 0;
    uint64_t carry = 0;
    const uint64_t n = entries ? d.ne : d.np;
    const uint8_t *pk = base + 12 * d.ne, *pv = pk + 4 * d.np;
    for (uint64_t c0 = 0; c0 < n; c0 += CH) {
        // coalesced: the chunk's items, the outputs that need no scan, the counts into LDS
        // (two rounds unrolled: a body at an unaligned address loads bytewise)
#pragma unroll 2
        for (int r = 0; r < R; ++r) {
            const uint32_t li = (uint32_t)r * kSmallT + tid;
            const uint64_t i = c0 + li;
            uint32_t cnt = 0;
            if constexpr (!entries) {
                if (i < n) {
                    const uint32_t kl = ld32(pk + 4 * i), vl = ld32(pv + 4 * i);
                    const uint64_t x = (uint64_t)kl + vl;
                    if (x > 0xFFFFFFFFull) bad = true;
                    cnt = x > 0xFFFFFFFFull ? 0u : (uint32_t)x;
                    klen[d.q0 + i] = kl;
                }
            } else {
                int64_t ts = 0;
                if (i < n) {
                    ts = (int64_t)ld64(base + 8 * i);
                    uint32_t kk = ld32(base + 8 * d.ne + 4 * i);
                    if (kk == kNilPairs) {
                        host = true;
                        kk = 0;
                    }
                    r_ts[d.e0 + i] = ts;
                    cnt = kk;
                    multi += kk != 1;
                }
                // ts ascending: the previous item is the previous lane's (lane 0: a reload)
                const int64_t up = (int64_t)__shfl_up((long long)ts, 1, 64);
                if (i < n && i > 0) {
                    const int64_t prev = lane ? up : (int64_t)ld64(base + 8 * (i - 1));
                    if (prev >= ts) host = true;
                }
            }
            buf32[big_pad(li)] = cnt;
        }
        __syncthreads();
        // thread-consecutive: the counts, their block scan, the prefixes
        uint32_t t[R];
        uint64_t sum = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            t[r] = buf32[big_pad(tid * R + r)];
            sum += t[r];
        }
        uint64_t tot;
        uint64_t run = carry + big_exclusive_scan(sum, &tot, wsum);   // (its barriers order the reads above)
        const uint64_t i0 = c0 + (uint64_t)tid * R;
        if constexpr (entries) {                          // each entry's pairs: 1 on its first (not unrolled)
            uint64_t rr = run;
#pragma unroll 1
            for (int r = 0; r < R; ++r) {
                if (i0 + r < n)
                    for (uint32_t j = 0; j < t[r] && rr + j < d.np; ++j) first[d.q0 + rr + j] = j == 0;
                rr += t[r];
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            buf[big_pad(tid * R + r)] = entries ? kv_base + d.q0 + run : d.y0 + run;
            run += t[r];
        }
        carry += tot;
        __syncthreads();
        // coalesced: the prefixes out
#pragma unroll 4
        for (int r = 0; r < R; ++r) {
            const uint32_t li = (uint32_t)r * kSmallT + tid;
            const uint64_t i = c0 + li;
            if (i < n) {
                if (entries) r_kv[d.e0 + i] = buf[big_pad(li)];
                else boff[d.q0 + i] = buf[big_pad(li)];
            }
        }
        __syncthreads();                                 // (the buffer is the next chunk's)
    }
    if (!entries) {
        if (carry != d.nb) bad = true;
        if (tid == 0) boff[d.q0 + d.np] = d.y0 + d.nb;
    } else if (carry != d.np) {
        bad = true;
    }
    const uint32_t fl = (bad ? kBodyMalformed : 0u) | (host ? kBodyHost : 0u);
    uint32_t wfl = fl;
    for (int m = 32; m >= 1; m >>= 1) {
        wfl |= __shfl_xor(wfl, m, 64);
        multi += __shfl_xor(multi, m, 64);
    }
    if (lane == 0 && wfl) atomicOr(&c.flag[b], wfl);
    if (lane == 0 && multi && c.multi) atomicAdd(c.multi, (unsigned long long)multi);
}

// R = 4 fits 64 VGPRs (two workgroups per CU); R = 8 takes 79 (one)
template <int R>
__device__ __forceinline__ void dec_big_body(DecodeCtx c, int64_t *__restrict__ r_ts, uint32_t *__restrict__ klen,
                                             uint64_t *__restrict__ boff, uint8_t *__restrict__ first, uint64_t n_e,
                                             uint64_t n_p, uint64_t kv_base, uint64_t *__restrict__ r_kv,
                                             uint64_t *__restrict__ r_off, uint64_t *wsum, uint64_t *buf) {
    const uint32_t b = blockIdx.x >> 1;                  // two workgroups per body: its pairs, its entries
    const bool entries = blockIdx.x & 1;
    const BodyDesc d = c.bd[b];
#define DEC_BIG(AL, EN) dec_big<R, AL, EN>(c, r_ts, klen, boff, first, n_e, n_p, kv_base, r_kv, r_off, d, wsum, buf, b)
    const bool al = (((uintptr_t)body_ptr(c.data, d.data)) & 7) == 0;
    if (entries) {
        if (al) DEC_BIG(true, true);
        else DEC_BIG(false, true);
    } else {
        if (al) DEC_BIG(true, false);
        else DEC_BIG(false, false);
    }
#undef DEC_BIG
}
__global__ __launch_bounds__(kSmallT) __attribute__((amdgpu_waves_per_eu(8))) void k_dec_big4(
    DecodeCtx c, int64_t *__restrict__ r_ts, uint32_t *__restrict__ klen, uint64_t *__restrict__ boff,
    uint8_t *__restrict__ first, uint64_t n_e, uint64_t n_p, uint64_t kv_base, uint64_t *__restrict__ r_kv,
    uint64_t *__restrict__ r_off) {
    __shared__ uint64_t wsum[kSmallT / 64];
    __shared__ uint64_t buf[kBigCH / 2 + kBigCH / 16];
    dec_big_body<4>(c, r_ts, klen, boff, first, n_e, n_p, kv_base, r_kv, r_off, wsum, buf);
}
__global__ __launch_bounds__(kSmallT) void k_dec_big8(DecodeCtx c, int64_t *__restrict__ r_ts,
                                                      uint32_t *__restrict__ klen, uint64_t *__restrict__ boff,
                                                      uint8_t *__restrict__ first, uint64_t n_e, uint64_t n_p,
                                                      uint64_t kv_base, uint64_t *__restrict__ r_kv,
                                                      uint64_t *__restrict__ r_off) {
    __shared__ uint64_t wsum[kSmallT / 64];
    __shared__ uint64_t buf[kBigCH + kBigCH / 8];
    dec_big_body<8>(c, r_ts, klen, boff, first, n_e, n_p, kv_base, r_kv, r_off, wsum, buf);
}

struct CountSrc32 {
    const uint32_t *in;
    struct Item {
        uint64_t len = 0;
    };
    __device__ Item load(uint64_t i) const { return Item{in[i]}; }
};

// per body: counts consistent with the header (pairs and bytes)
__global__ void k_dec_bodies(DecodeCtx c, const uint64_t *__restrict__ pre) {
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b >= c.nbody) return;
    const BodyDesc d = c.bd[b];
    if (pre[d.e0 + d.ne] - pre[d.e0] != d.np) atomicOr(&c.flag[b], kBodyMalformed);
    if (c.boff[d.q0 + d.np] - c.boff[d.q0] != d.nb) atomicOr(&c.flag[b], kBodyMalformed);
}

// r_kv = kv_base + the body's first pair + pre rebased to the body's first
// entry, so a body whose pair counts disagree with its header (flagged by
// k_dec_bodies) cannot shift the ranges of the bodies after it; mark the
// first pair of each entry within its own body's pair range.  Body-major
// (grid.y = body, like k_dec_entries): an entry's body is its workgroup's,
// no search (a flat grid's per-entry binary search over the body table put
// ten dependent loads in front of every entry: 124 us for 1000 x 10k).
__global__ __launch_bounds__(256) void k_dec_kv(DecodeCtx c, const uint64_t *__restrict__ pre, uint64_t n_e,
                                                uint64_t n_p, uint64_t kv_base, uint64_t *__restrict__ r_kv,
                                                uint8_t *__restrict__ first) {
    const uint32_t b = blockIdx.y;
    const BodyDesc d = c.bd[b];
    if (b == 0 && blockIdx.x == 0 && threadIdx.x == 0) r_kv[n_e] = kv_base + n_p;
    if (d.ne == 0) return;
    const uint64_t p0 = pre[d.e0];
    for (uint64_t i = (uint64_t)blockIdx.x * kChunk + threadIdx.x; i < d.ne && i < (uint64_t)(blockIdx.x + 1) * kChunk;
         i += 256) {
        const uint64_t e = d.e0 + i;
        const uint64_t a = pre[e], z = pre[e + 1];
        const uint64_t p = a - p0;
        r_kv[e] = kv_base + d.q0 + p;
        if (z > a && p < d.np) first[d.q0 + p] = 1;
    }
}

struct PendGet {                   // bytes of pending reference j (key or value part of pair j)
    DecodeCtx c;
    bool value;
    __device__ void operator()(uint32_t j, const uint8_t **p, uint32_t *n) const {
        const uint8_t *kp, *vp;
        uint32_t kn, vn;
        c.pair_bytes(j, &kp, &kn, &vp, &vn);
        *p = value ? vp : kp;
        *n = value ? vn : kn;
    }
};

// pass A over both tables, body-major.  A pair whose string is already in a
// table (an id from an earlier call) gets its ids written at once; the
// others record their entry (bit 31: this pair claimed it) for passes B / C
// and count the claims (ctr[0] keys, ctr[1] values).  kEmptyE slots: done.
// SM (codec.short_tab): 0 -- the byte walk for every candidate entry; 1 --
// a resolved short string compares the short form beside its entry; 2 -- as
// 1, and a pair whose key and value both have at most 7 bytes first probes
// both home entries at once (one round trip instead of one per table); the
// pairs that do not resolve there (new or pending strings, probe chains,
// longer strings) are listed in LDS and claimed by the loop of form 1 after
// a barrier -- kept out of the first loop so that its registers stay few.
template <int SM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_dec_claim(DecodeCtx c, TabView kt, TabView vt,
                                                   const uint8_t *__restrict__ first, const uint32_t *__restrict__ flag0,
                                                   uint32_t *__restrict__ cflag,
                                                   uint32_t key_cap,
                                                   uint64_t kv_base, uint32_t *__restrict__ kslot,
                                                   uint32_t *__restrict__ vslot, uint32_t *__restrict__ kv_key,
                                                   uint32_t *__restrict__ kv_val, unsigned long long *__restrict__ ctr) {
    static_assert(kClaimChunk == 256, "one pair per thread (forms 3 / 4: two / three)");
    constexpr int PP = SM == 4 ? 3 : 2;                      // forms 3 / 4: pairs per thread
    constexpr uint32_t CC = SM >= 3 ? PP * kClaimChunk : kClaimChunk;   // pairs per workgroup
    __shared__ uint32_t s_slow[SM >= 2 ? CC : 1];
    __shared__ uint32_t s_ns;
    const uint32_t b = blockIdx.y;
    const BodyDesc d = c.bd[b];
    const uint8_t *region = body_ptr(c.data, d.data) + 32 + 12 * d.ne + 8 * d.np;
    const uint64_t o0 = c.boff[d.q0];
    // a body the earlier passes already rejected (flag0: their flags, which
    // this pass only reads -- its own go to cflag) claims no table entries:
    // its strings never enter the persistent tables (the host decodes it)
    const bool rejected = flag0[b] != 0;
    bool host = false, bad = false, full = false;
    uint32_t nk = 0, nv = 0;
    // both claims of pair j (key, then value): ids written for strings known
    // from earlier calls, claimed / pending entries recorded for passes B / C
    auto claim = [&](uint64_t j, const uint8_t *kp, uint32_t k, uint64_t ksv, const uint8_t *vp, uint32_t v,
                     uint64_t vsv) {
        uint32_t ks = kEmptyE32, vs = kEmptyE32;
        const uint32_t kh = k <= 8 ? hash32_short(ksv, k) : hash32(kp, k);
        const uint32_t vh = v <= 8 ? hash32_short(vsv, v) : hash32(vp, v);
        bool rk = false, rv = false;
        uint64_t ek = 0, ev = 0;
        const uint64_t si = tab_claim(kt, kh, kp, k, (uint32_t)j, PendGet{c, false}, &rk, &ek, ksv, SM != 0);
        if (si == kEmptyE) {
            full = true;
        } else {
            if (!rk && !((uint32_t)ek & kPend)) {            // an existing id
                const uint32_t kid = (uint32_t)ek & kIdMask;
                if (kid >= key_cap) host = true;
                kv_key[kv_base + j] = d.slot_base + kid;
            } else {
                ks = (uint32_t)si | (rk ? kRepBit : 0u);
                nk += rk;
            }
        }
        const uint64_t sv = tab_claim(vt, vh, vp, v, (uint32_t)j, PendGet{c, true}, &rv, &ev, vsv, SM != 0);
        if (sv == kEmptyE) {
            full = true;
        } else {
            if (!rv && !((uint32_t)ev & kPend)) {
                kv_val[kv_base + j] = (uint32_t)ev & kIdMask;
            } else {
                vs = (uint32_t)sv | (rv ? kRepBit : 0u);
                nv += rv;
            }
        }
        kslot[j] = ks;
        vslot[j] = vs;
    };
    if (SM >= 2) {
        if (threadIdx.x == 0) s_ns = 0;
        __syncthreads();
    }
    if constexpr (SM >= 3) {
        // forms 3 / 4: two / three pairs per thread, each step's loads issued
        // for all of them before any is used (the chain is paid once for all)
        const uint64_t qb = (uint64_t)blockIdx.x * CC + threadIdx.x;
        bool act[PP];
        uint64_t b0[PP], b1[PP], ksv[PP], vsv[PP], hk[PP], sk[PP], hv[PP], sw[PP];
        uint32_t kl[PP], vl[PP];
#pragma unroll
        for (int p = 0; p < PP; ++p) {
            const uint64_t q = qb + 256 * p, j = d.q0 + q;
            act[p] = q < d.np && !rejected;
            if (q < d.np && rejected) kslot[j] = vslot[j] = kEmptyE32;
            b0[p] = act[p] ? c.boff[j] : 0;
            b1[p] = act[p] ? c.boff[j + 1] : 0;
            kl[p] = act[p] ? c.klen[j] : 0;
        }
#pragma unroll
        for (int p = 0; p < PP; ++p) {
            const uint64_t j = d.q0 + qb + 256 * p;
            const uint64_t o = b0[p] - o0, k = kl[p], v = b1[p] - b0[p] - k;
            if (act[p] && (o > d.nb || k > d.nb - o || v > d.nb - o - k)) {
                bad = true;
                kslot[j] = vslot[j] = kEmptyE32;
                act[p] = false;
            }
            vl[p] = (uint32_t)v;
            ksv[p] = act[p] && k <= 8 ? load_short(region + o, (uint32_t)k) : 0;
            vsv[p] = act[p] && v <= 8 ? load_short(region + o + k, (uint32_t)v) : 0;
        }
#pragma unroll
        for (int p = 0; p < PP; ++p) {
            const uint64_t q = qb + 256 * p, j = d.q0 + q;
            if (act[p] && q && !first[j]) {                  // keys of an entry strictly ascending
                const uint64_t o = b0[p] - o0, k = kl[p];
                const uint64_t po = c.boff[j - 1] - o0, pk = c.klen[j - 1];
                if (po + pk <= o) {
                    const bool lt = pk <= 8 && k <= 8
                                        ? short_lt(load_short(region + po, (uint32_t)pk), (uint32_t)pk, ksv[p], (uint32_t)k)
                                        : bytes_lt(region + po, (uint32_t)pk, region + o, (uint32_t)k);
                    if (!lt) host = true;
                }
            }
        }
#pragma unroll
        for (int p = 0; p < PP; ++p) {                       // both pairs' home entries, one round trip
            hk[p] = sk[p] = hv[p] = sw[p] = kNoShort;
            if (act[p] && kl[p] <= 7 && vl[p] <= 7) {
                const uint64_t ik = hash32_short(ksv[p], kl[p]) & kt.mask, iv = hash32_short(vsv[p], vl[p]) & vt.mask;
                hk[p] = kt.tab[ik];
                sk[p] = kt.tab[kt.mask + 1 + ik];
                hv[p] = vt.tab[iv];
                sw[p] = vt.tab[vt.mask + 1 + iv];
            }
        }
#pragma unroll
        for (int p = 0; p < PP; ++p) {
            if (!act[p]) continue;
            const uint64_t j = d.q0 + qb + 256 * p;
            // (a short form is written with its entry's id: a match is a resolved entry)
            if (kl[p] <= 7 && vl[p] <= 7 && sk[p] == short_form(ksv[p], kl[p]) && sw[p] == short_form(vsv[p], vl[p])) {
                const uint32_t kid = (uint32_t)hk[p] & kIdMask;
                if (kid >= key_cap) host = true;
                kv_key[kv_base + j] = d.slot_base + kid;
                kv_val[kv_base + j] = (uint32_t)hv[p] & kIdMask;
                kslot[j] = vslot[j] = kEmptyE32;
            } else {
                s_slow[atomicAdd(&s_ns, 1u)] = threadIdx.x + 256u * p;
            }
        }
    }
    for (uint64_t q = (uint64_t)blockIdx.x * kClaimChunk + threadIdx.x;
         SM < 3 && q < d.np && q < (uint64_t)(blockIdx.x + 1) * kClaimChunk; q += 256) {
        const uint64_t j = d.q0 + q;
        if (rejected) {
            kslot[j] = vslot[j] = kEmptyE32;
            continue;
        }
        const uint64_t o = c.boff[j] - o0, k = c.klen[j], v = c.boff[j + 1] - c.boff[j] - k;
        if (o > d.nb || k > d.nb - o || v > d.nb - o - k) {
            bad = true;
            kslot[j] = vslot[j] = kEmptyE32;
            continue;
        }
        const uint8_t *kp = region + o, *vp = region + o + k;
        // short strings (the reference's one-byte keys and short values)
        // packed in registers: one word load each, hash and compares on it
        const uint64_t ksv = k <= 8 ? load_short(kp, (uint32_t)k) : 0, vsv = v <= 8 ? load_short(vp, (uint32_t)v) : 0;
        if (q && !first[j]) {                                // keys of an entry strictly ascending
            const uint64_t po = c.boff[j - 1] - o0, pk = c.klen[j - 1];
            if (po + pk <= o) {
                const bool lt = pk <= 8 && k <= 8
                                    ? short_lt(load_short(region + po, (uint32_t)pk), (uint32_t)pk, ksv, (uint32_t)k)
                                    : bytes_lt(region + po, (uint32_t)pk, kp, (uint32_t)k);
                if (!lt) host = true;
            }
        }
        if constexpr (SM == 2) {
            bool done = false;
            if (k <= 7 && v <= 7) {                          // both home entries, one round trip
                const uint64_t wk = short_form(ksv, (uint32_t)k), wv = short_form(vsv, (uint32_t)v);
                const uint64_t ik = hash32_short(ksv, (uint32_t)k) & kt.mask, iv = hash32_short(vsv, (uint32_t)v) & vt.mask;
                const uint64_t hk = kt.tab[ik], sk = kt.tab[kt.mask + 1 + ik];
                const uint64_t hv = vt.tab[iv], sw = vt.tab[vt.mask + 1 + iv];
                // (a short form is written with its entry's id: a match is a resolved entry)
                if (sk == wk && sw == wv) {
                    const uint32_t kid = (uint32_t)hk & kIdMask;
                    if (kid >= key_cap) host = true;
                    kv_key[kv_base + j] = d.slot_base + kid;
                    kv_val[kv_base + j] = (uint32_t)hv & kIdMask;
                    kslot[j] = vslot[j] = kEmptyE32;
                    done = true;
                }
            }
            if (!done) s_slow[atomicAdd(&s_ns, 1u)] = (uint32_t)(q - (uint64_t)blockIdx.x * kClaimChunk);
        } else {
            claim(j, kp, (uint32_t)k, ksv, vp, (uint32_t)v, vsv);
        }
    }
    if constexpr (SM >= 2) {                                 // the listed pairs, claimed as form 1 claims them
        __syncthreads();
        const uint32_t ns = s_ns;
        for (uint32_t i = threadIdx.x; i < ns; i += 256) {
            const uint64_t q = (uint64_t)blockIdx.x * CC + s_slow[i], j = d.q0 + q;
            const uint64_t o = c.boff[j] - o0, k = c.klen[j], v = c.boff[j + 1] - c.boff[j] - k;   // (in range: checked above)
            const uint8_t *kp = region + o, *vp = region + o + k;
            const uint64_t ksv = k <= 8 ? load_short(kp, (uint32_t)k) : 0, vsv = v <= 8 ? load_short(vp, (uint32_t)v) : 0;
            claim(j, kp, (uint32_t)k, ksv, vp, (uint32_t)v, vsv);
        }
    }
    const uint32_t fl = (bad ? kBodyMalformed : 0u) | (host ? kBodyHost : 0u) | (full ? kBodyFull : 0u);
    for (int m = 32; m >= 1; m >>= 1) {
        nk += __shfl_xor(nk, m, 64);
        nv += __shfl_xor(nv, m, 64);
    }
    uint32_t wfl = fl;
    for (int m = 32; m >= 1; m >>= 1) wfl |= __shfl_xor(wfl, m, 64);
    if ((threadIdx.x & 63) == 0) {
        if (wfl) atomicOr(&cflag[b], wfl);
        if (nk) atomicAdd(&ctr[0], (unsigned long long)nk);
        if (nv) atomicAdd(&ctr[1], (unsigned long long)nv);
    }
}

struct RepCntSrc {                 // scan source: 1 for a claimer
    const uint32_t *slot;
    struct Item {
        uint64_t len = 0;
    };
    __device__ Item load(uint64_t j) const { return Item{(slot[j] != kEmptyE32 && (slot[j] & kRepBit)) ? 1u : 0u}; }
};

struct RepLenSrc {                 // scan source: bytes of the claimers' strings
    DecodeCtx c;
    const uint32_t *slot;
    bool value;
    struct Item {
        uint64_t len = 0;
    };
    __device__ Item load(uint64_t j) const {
        if (slot[j] == kEmptyE32 || !(slot[j] & kRepBit)) return Item{0};
        const uint8_t *kp, *vp;
        uint32_t kn, vn;
        c.pair_bytes(j, &kp, &kn, &vp, &vn);
        return Item{value ? vn : kn};
    }
};

// pass B: claimers -> dense ids, bytes into the arena, entry -> id
__global__ void k_dec_assign(DecodeCtx c, TabView t, bool value, const uint32_t *__restrict__ slot,
                             const uint64_t *__restrict__ rank, const uint64_t *__restrict__ rboff, uint64_t n_old,
                             uint64_t bytes_old, uint8_t *__restrict__ arena, uint64_t *__restrict__ off) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < c.n_pairs; j += (uint64_t)gridDim.x * 256) {
        const uint32_t sl = slot[j];
        if (sl == kEmptyE32 || !(sl & kRepBit)) continue;
        const uint8_t *kp, *vp;
        uint32_t kn, vn;
        c.pair_bytes(j, &kp, &kn, &vp, &vn);
        const uint8_t *p = value ? vp : kp;
        const uint32_t n = value ? vn : kn;
        const uint64_t id = n_old + rank[j];
        const uint64_t o = bytes_old + rboff[j];
        for (uint32_t i = 0; i < n; ++i) arena[o + i] = p[i];
        off[id] = o;
        const uint64_t si = sl & ~kRepBit;
        t.tab[si] = (t.tab[si] & 0xFFFFFFFF00000000ull) | (uint32_t)id;   // keep the hash, drop the pending tag
        t.tab[t.mask + 1 + si] = short_form_bytes(p, n);
    }
}

__global__ void k_off_end(uint64_t *__restrict__ off, const uint64_t *__restrict__ n_new_dev,
                          const uint64_t *__restrict__ bytes_new_dev, uint64_t n_old, uint64_t bytes_old,
                          unsigned long long *__restrict__ sizes) {
    off[n_old + *n_new_dev] = bytes_old + *bytes_new_dev;
    sizes[0] = *n_new_dev;                            // (read back with the flags in one copy)
    sizes[1] = *bytes_new_dev;
}

// pass C: ids of the pairs whose string was new in this call
__global__ void k_dec_ids(DecodeCtx c, const uint32_t *__restrict__ kslot, const uint32_t *__restrict__ vslot,
                          const uint64_t *__restrict__ ktab, const uint64_t *__restrict__ vtab, uint32_t key_cap,
                          uint64_t kv_base, uint32_t *__restrict__ kv_key, uint32_t *__restrict__ kv_val) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < c.n_pairs; j += (uint64_t)gridDim.x * 256) {
        const uint32_t ks = kslot[j], vs = vslot[j];
        if (ks != kEmptyE32) {
            const uint32_t b = find_body(c.bd, c.nbody, j, true);
            const uint32_t kid = (uint32_t)ktab[ks & ~kRepBit] & kIdMask;
            if (kid >= key_cap) atomicOr(&c.flag[b], kBodyHost);   // key beyond the replica's slot range
            kv_key[kv_base + j] = c.bd[b].slot_base + kid;
        }
        if (vs != kEmptyE32) kv_val[kv_base + j] = (uint32_t)vtab[vs & ~kRepBit] & kIdMask;
    }
}

// rehash: every id re-inserted (ids are unique: no byte compare needed)
__global__ void k_rehash(uint64_t *__restrict__ tab, uint64_t mask, const uint8_t *__restrict__ bytes,
                         const uint64_t *__restrict__ off, uint64_t n) {
    for (uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x; id < n; id += (uint64_t)gridDim.x * 256) {
        const uint32_t n = (uint32_t)(off[id + 1] - off[id]);
        const uint32_t h = hash32(bytes + off[id], n);
        uint64_t i = h & mask;
        for (;;) {
            const uint64_t old = atomicCAS((unsigned long long *)&tab[i], (unsigned long long)kEmptyE,
                                           (unsigned long long)((uint64_t)h << 32 | (uint32_t)id));
            if (old == kEmptyE) break;
            i = (i + 1) & mask;
        }
        tab[mask + 1 + i] = short_form_bytes(bytes + off[id], n);
    }
}

// hdr[32 b ..] = the first 32 bytes of body b (zeros if shorter)
__global__ void k_gather_headers(const uint8_t *__restrict__ data, const uint64_t *__restrict__ at,
                                 const uint64_t *__restrict__ len, uint32_t nb, uint8_t *__restrict__ hdr) {
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b >= nb) return;
    const bool ok = len[b] >= 32;
    const uint8_t *p = body_ptr(data, at[b]);
    for (int i = 0; i < 32; ++i) hdr[32 * (size_t)b + i] = ok ? p[i] : 0;
}

uint64_t pow2_at_least(uint64_t x) {
    uint64_t p = 1024;
    while (p < x) p <<= 1;
    return p;
}

int dev_grow(crdt_ctx *ctx, void **p, uint64_t old_bytes, uint64_t new_bytes) {
    void *q = nullptr;
    hipError_t e = hipMalloc(&q, new_bytes);
    if (e != hipSuccess) return hip_fail(ctx, e);
    if (*p && old_bytes) {
        e = hipMemcpyAsync(q, *p, old_bytes, hipMemcpyDeviceToDevice, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) {
            (void)hipFree(q);
            return hip_fail(ctx, e);
        }
        (void)hipFree(*p);
    }
    *p = q;
    return CRDT_OK;
}

// Room for `more` strings of `more_bytes` bytes: grow the arena / offsets
// (copy) and the hash table (rehash at load <= 1/2).
int tab_reserve(crdt_ctx *ctx, crdt_strtab *t, uint64_t more, uint64_t more_bytes) {
    int rc;
    if (t->nbytes + more_bytes > t->cap_bytes) {
        const uint64_t cap = std::max<uint64_t>(2 * t->cap_bytes, t->nbytes + more_bytes + 4096);
        rc = dev_grow(ctx, (void **)&t->bytes, t->nbytes, cap);
        if (rc) return rc;
        t->cap_bytes = cap;
    }
    if (t->n + more > t->cap_n) {
        const uint64_t cap = std::max<uint64_t>(2 * t->cap_n, t->n + more + 256);
        rc = dev_grow(ctx, (void **)&t->off, (t->n + 1) * 8, (cap + 1) * 8);
        if (rc) return rc;
        t->cap_n = cap;
    }
    if (2 * (t->n + more) > t->H) {
        const uint64_t H = pow2_at_least(4 * (t->n + more));
        uint64_t *nt = nullptr;
        hipError_t e = hipMalloc(&nt, 2 * H * 8);       // entries, then short forms
        if (e != hipSuccess) return hip_fail(ctx, e);
        e = hipMemsetAsync(nt, 0xFF, 2 * H * 8, ctx->stream);
        if (e != hipSuccess) {
            (void)hipFree(nt);
            return hip_fail(ctx, e);
        }
        if (t->n) k_rehash<<<grid_for(t->n, 256, (unsigned)ctx->num_cus * 4), 256, 0, ctx->stream>>>(
            nt, H - 1, t->bytes, t->off, t->n);
        e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) {
            (void)hipFree(nt);
            return hip_fail(ctx, e);
        }
        if (t->tab) (void)hipFree(t->tab);
        t->tab = nt;
        t->H = H;
    }
    return CRDT_OK;
}

// host mirror: pull the strings added since the last sync
int tab_pull_new(crdt_ctx *ctx, crdt_strtab *t, uint64_t n_new, uint64_t bytes_new) {
    const uint64_t n0 = t->h_off.size() - 1, b0 = t->h_bytes.size();
    t->h_off.resize(n_new + 1);
    t->h_bytes.resize(bytes_new);
    hipError_t e = hipSuccess;
    if (n_new > n0)
        e = hipMemcpyAsync(t->h_off.data() + n0 + 1, t->off + n0 + 1, (n_new - n0) * 8, hipMemcpyDeviceToHost,
                           ctx->stream);
    if (e == hipSuccess && bytes_new > b0)
        e = hipMemcpyAsync(t->h_bytes.data() + b0, t->bytes + b0, bytes_new - b0, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
    t->n = n_new;
    t->nbytes = bytes_new;
    return CRDT_OK;
}

}  // namespace
}  // namespace crdt

using namespace crdt;

extern "C" int crdt_strtab_create(crdt_ctx *ctx, size_t cap_strings, size_t cap_bytes, crdt_strtab **out) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!out) return CRDT_E_INVAL;
    *out = nullptr;
    crdt_strtab *t = new (std::nothrow) crdt_strtab();
    if (!t) return CRDT_E_NOMEM;
    t->device = ctx->device;
    rc = tab_reserve(ctx, t, std::max<size_t>(cap_strings, 16), std::max<size_t>(cap_bytes, 256));
    if (!rc) {
        hipError_t e = hipMemsetAsync(t->off, 0, 8, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) rc = hip_fail(ctx, e);
    }
    if (rc) {
        (void)crdt_strtab_destroy(t);
        return rc;
    }
    *out = t;
    return CRDT_OK;
}

extern "C" int crdt_strtab_destroy(crdt_strtab *t) {
    if (!t) return CRDT_OK;
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (cur != t->device) (void)hipSetDevice(t->device);
    if (t->tab) (void)hipFree(t->tab);
    if (t->bytes) (void)hipFree(t->bytes);
    if (t->off) (void)hipFree(t->off);
    delete t;
    return CRDT_OK;
}

extern "C" int crdt_strtab_info(const crdt_strtab *t, uint64_t *n_str, uint64_t *n_bytes, const uint8_t **bytes_dev,
                                const uint64_t **off_dev) {
    if (!t || !n_str || !n_bytes) return CRDT_E_INVAL;
    *n_str = t->n;
    *n_bytes = t->nbytes;
    if (bytes_dev) *bytes_dev = t->bytes;
    if (off_dev) *off_dev = t->off;
    return CRDT_OK;
}

// i-th string of the table's host mirror (valid until the next call that adds strings)
extern "C" int crdt_strtab_get(const crdt_strtab *t, uint64_t id, const char **p, size_t *len) {
    if (!t || !p || !len) return CRDT_E_INVAL;
    if (id >= t->n) return CRDT_E_RANGE;
    *p = (const char *)t->h_bytes.data() + t->h_off[id];
    *len = t->h_off[id + 1] - t->h_off[id];
    return CRDT_OK;
}

namespace crdt {
// The first 32 bytes of each body (zeros for a shorter one) to host memory:
// one gather kernel, one read-back.  Synchronises.
int gossip_headers(crdt_ctx *ctx, uint32_t nb, const uint8_t *data, const uint64_t *at, const uint64_t *len,
                   uint8_t *hdr) {
    if (nb == 0) return CRDT_OK;
    const hipStream_t s = ctx->stream;
    int rc = ws_reserve(ctx, Carve::round(nb * 16) + Carve::round(32 * (size_t)nb) + 512);
    if (!rc) rc = hio_reserve(ctx, (size_t)nb * 16 + 32 * (size_t)nb);
    if (rc) return rc;
    Carve w0(ctx->ws);
    uint64_t *d_al = w0.take<uint64_t>(2 * (size_t)nb);
    uint8_t *d_hdr = w0.take<uint8_t>(32 * (size_t)nb);
    uint64_t *h_al = (uint64_t *)ctx->hio;
    memcpy(h_al, at, nb * 8);
    memcpy(h_al + nb, len, nb * 8);
    hipError_t e = hipMemcpyAsync(d_al, h_al, nb * 16, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return hip_fail(ctx, e);
    k_gather_headers<<<grid_for(nb, 256, 1u << 30), 256, 0, s>>>(data, d_al, d_al + nb, nb, d_hdr);
    rc = check_launch(ctx);
    if (rc) return rc;
    uint8_t *h_hdr = (uint8_t *)ctx->hio + (size_t)nb * 16;
    e = hipMemcpyAsync(h_hdr, d_hdr, 32 * (size_t)nb, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(ctx, e);
    memcpy(hdr, h_hdr, 32 * (size_t)nb);
    return CRDT_OK;
}

static size_t decode_ws_need(uint32_t nb, uint64_t n_e, uint64_t n_p) {
    const size_t head = Carve::round(nb * sizeof(BodyDesc)) + Carve::round(nb * 8) + 64;
    return Carve::round(head) + Carve::round((n_e + 1) * 4) + Carve::round((n_e + 1) * 8) +
           Carve::round(n_p * 4 + 4) * 4 + Carve::round((n_p + 1) * 8) * 5 + Carve::round(n_p + 1) +
           scan_lb_tmp_bytes(std::max(n_p, n_e)) + 4096;
}

size_t gossip_decode_scratch_bytes(uint32_t nb, uint64_t n_e, uint64_t n_p) { return decode_ws_need(nb, n_e, n_p); }

// The decode of nb bodies at data + at[b] (mod 2^64), len[b] bytes each.  Small
// uploads and read-backs go through the context's pinned staging (ctx->hio):
// one upload of the body table with the zeroed flags and counters, one
// read-back of flags + counters per host synchronisation.
//   spec (optional): work that consumes the decode's output, enqueued right
//   behind the claim pass's read-back so that it runs before the host has
//   even looked at the claims (the common case: every string already
//   interned, nothing left to do); when new strings did arrive, their ids are
//   written afterwards and *spec_stale says spec ran on incomplete ids.  The
//   decode then works in `scratch` (>= gossip_decode_scratch_bytes), not in
//   ctx->ws, which spec's own passes use.  Without scratch, spec runs after
//   the whole decode.  Either way it has completed when this returns.
int gossip_decode_at(crdt_ctx *ctx, uint32_t nb, const uint8_t *data, const uint64_t *at, const uint64_t *len,
                     uint32_t key_cap, uint64_t kv_base, const uint32_t *slot_base, const uint8_t *host_hdr,
                     crdt_strtab *keys, crdt_strtab *vals, const crdt_gossip_decoded *out, uint32_t *body_status,
                     const std::function<int()> *spec, void *scratch, size_t scratch_cap, bool *spec_stale,
                     uint64_t *multi_pair) {
    if (spec_stale) *spec_stale = false;
    if (multi_pair) *multi_pair = 0;
    const hipStream_t s = ctx->stream;
    int rc;
    hipError_t e;
    // headers (32 B per body) to the host in one gather + one copy: the sizes
    // the decode is planned with
    std::vector<uint8_t> hdr_buf;
    const uint8_t *hdr = host_hdr;
    if (!hdr) {
        hdr_buf.resize(32 * (size_t)nb);
        rc = gossip_headers(ctx, nb, data, at, len, hdr_buf.data());
        if (rc) return rc;
        hdr = hdr_buf.data();
    }
    std::vector<BodyDesc> bd(nb);
    std::vector<uint64_t> r_off(nb + 1, 0);
    uint64_t n_e = 0, n_p = 0, n_b = 0;
    static const char magic[8] = {'C', 'R', 'D', 'T', 'S', 'O', 'A', '1'};
    for (uint32_t b = 0; b < nb; ++b) {
        const uint8_t *h = &hdr[32 * b];
        uint64_t ne = 0, np = 0, nby = 0;
        body_status[b] = 0;
        if (len[b] < 32 || memcmp(h, magic, 8) != 0) {
            body_status[b] = kBodyMalformed;
        } else {
            memcpy(&ne, h + 8, 8);
            memcpy(&np, h + 16, 8);
            memcpy(&nby, h + 24, 8);
            const uint64_t l = len[b];
            if (ne > l / 12 || np > l / 8 || nby > l || 32 + ne * 12 + np * 8 + nby != l || np >= kPend)
                body_status[b] = kBodyMalformed;
        }
        if (body_status[b]) ne = np = nby = 0;           // contributes nothing
        bd[b] = BodyDesc{at[b], n_e, n_p, ne, np, nby, slot_base[b], 0, n_b};
        n_e += ne;
        n_p += np;
        n_b += nby;
        r_off[b + 1] = n_e;
    }
    if (n_p >= kPend || n_e >= 0xFFFFFFFFull) return CRDT_E_RANGE;
    if ((n_e && (!out->r_ts || !out->r_kv)) || (n_p && (!out->kv_key || !out->kv_val))) return CRDT_E_INVAL;
    rc = tab_reserve(ctx, keys, n_p, n_b);
    if (!rc) rc = tab_reserve(ctx, vals, n_p, n_b);
    if (rc) return rc;
    // workspace; the head block [body table | flags | counters] is uploaded
    // from the pinned staging in one copy (flags and counters zeroed there)
    const size_t bd_bytes = Carve::round(nb * sizeof(BodyDesc)), fl_bytes = Carve::round(nb * 8);
    const size_t head = bd_bytes + fl_bytes + 64;
    const size_t need = decode_ws_need(nb, n_e, n_p);
    const bool early = spec && scratch && scratch_cap >= need;   // spec behind the claims, on scratch
    rc = early ? CRDT_OK : ws_reserve(ctx, need);
    if (!rc) rc = hio_reserve(ctx, head + (nb + 1) * 8);
    if (rc) return rc;
    Carve w(early ? scratch : ctx->ws);
    char *d_head = w.take<char>(head);
    BodyDesc *d_bd = (BodyDesc *)d_head;
    uint32_t *d_flag = (uint32_t *)(d_head + bd_bytes);   // [0, nb): the other passes, [nb, 2nb): the claim pass
    unsigned long long *ctr = (unsigned long long *)(d_head + bd_bytes + fl_bytes);   // [0..1] claims, [2..5] sizes
    uint32_t *cnt = w.take<uint32_t>(n_e + 1);
    uint64_t *pre = w.take<uint64_t>(n_e + 1);
    uint32_t *klen = w.take<uint32_t>(n_p + 1);
    uint32_t *plen = w.take<uint32_t>(n_p + 1);
    uint32_t *kslot = w.take<uint32_t>(n_p + 1);
    uint32_t *vslot = w.take<uint32_t>(n_p + 1);
    uint64_t *boff = w.take<uint64_t>(n_p + 1);
    uint64_t *krank = w.take<uint64_t>(n_p + 1);
    uint64_t *vrank = w.take<uint64_t>(n_p + 1);
    uint64_t *kboff = w.take<uint64_t>(n_p + 1);
    uint64_t *vboff = w.take<uint64_t>(n_p + 1);
    uint8_t *first = w.take<uint8_t>(n_p + 1);
    void *tmp = w.take<char>(scan_lb_tmp_bytes(std::max(n_p, n_e)));
    char *h_head = (char *)ctx->hio;
    memset(h_head, 0, head);
    memcpy(h_head, bd.data(), nb * sizeof(BodyDesc));
    uint64_t *h_roff = (uint64_t *)(h_head + head);
    memcpy(h_roff, r_off.data(), (nb + 1) * 8);
    DecodeCtx c{data, d_bd, nb, d_flag, boff, klen, n_p, ctr + 6};
    uint64_t max_ne = 0, max_np = 0;
    for (auto &x : bd) {
        max_ne = std::max(max_ne, x.ne);
        max_np = std::max(max_np, x.np);
    }
    // decode form (codec.small): 0 the multi-pass kernels, 2 the one-pass
    // kernel, 3 its coalesced form; 1 (auto): the one-pass kernel for a few
    // bodies of one chunk, the coalesced form for a few larger bodies (the
    // Server path) and for many bodies of up to two chunks each (the
    // population wire rounds: DESIGN.md §5.10), the multi-pass kernels
    // otherwise
    // (round 6: a few bodies of more than one 4096-item chunk -- the Server
    // path at config A, 10k entries per pull -- take the coalesced form too:
    // k_dec_big4 21.7 us against k_dec_small's 26.1 us for 5 x 10k,
    // profiles/r06/ab/server_decode_form.txt)
    int form = g_dec_small;
    if (form == 1) {
        const uint64_t mx = std::max(max_ne, max_np);
        form = nb <= (uint32_t)ctx->num_cus && mx <= 4096          ? 2
               : nb <= (uint32_t)ctx->num_cus && mx <= kSmallItems ? 3
               : mx <= 2 * kBigCH                                  ? 3
                                                                   : 0;
    }
    const bool small = form >= 2;
    e = hipMemcpyAsync(d_head, h_head, head, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && !small) e = hipMemcpyAsync(out->r_off, h_roff, (nb + 1) * 8, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return hip_fail(ctx, e);
    const dim3 ge((unsigned)std::max<uint64_t>((max_ne + kChunk - 1) / kChunk, 1), nb);
    const dim3 gp((unsigned)std::max<uint64_t>((max_np + kChunk - 1) / kChunk, 1), nb);
    const unsigned cap = (unsigned)ctx->num_cus * 8;
    if (form == 3) {
        if (g_dec_big_r == 8)
            k_dec_big8<<<2 * nb, kSmallT, 0, s>>>(c, out->r_ts, klen, boff, first, n_e, n_p, kv_base, out->r_kv,
                                              out->r_off);
        else
            k_dec_big4<<<2 * nb, kSmallT, 0, s>>>(c, out->r_ts, klen, boff, first, n_e, n_p, kv_base, out->r_kv,
                                              out->r_off);
        rc = check_launch(ctx);
        if (rc) return rc;
    } else if (small) {
        k_dec_small<<<2 * nb, kSmallT, 0, s>>>(c, out->r_ts, klen, boff, first, n_e, n_p, kv_base, out->r_kv,
                                           out->r_off);
        rc = check_launch(ctx);
        if (rc) return rc;
    } else if (n_e) {
        k_dec_entries<<<ge, 256, 0, s>>>(c, out->r_ts, cnt);
        rc = check_launch(ctx);
        if (!rc) rc = scan_lb(ctx, CountSrc32{cnt}, NoAct(), n_e, 0, pre, tmp);
        if (rc) return rc;
    } else {
        e = hipMemsetAsync(pre, 0, 8, s);
        if (e != hipSuccess) return hip_fail(ctx, e);
    }
    if (!small) {
        if (n_p) {
            k_dec_pairs<<<gp, 256, 0, s>>>(c, klen, plen, first);
            rc = check_launch(ctx);
            if (rc) return rc;
        }
        rc = scan_lb(ctx, CountSrc32{plen}, NoAct(), n_p, 0, boff, tmp);
        if (rc) return rc;
        k_dec_bodies<<<grid_for(nb, 256, 1u << 30), 256, 0, s>>>(c, pre);
        k_dec_kv<<<ge, 256, 0, s>>>(c, pre, n_e, n_p, kv_base, out->r_kv, first);
        rc = check_launch(ctx);
        if (rc) return rc;
    }
    const uint64_t kn0 = keys->n, kb0 = keys->nbytes, vn0 = vals->n, vb0 = vals->nbytes;
    TabView kt{keys->tab, keys->H - 1, keys->bytes, keys->off};
    TabView vt{vals->tab, vals->H - 1, vals->bytes, vals->off};
    if (n_p) {
        const uint64_t cc = (g_short_tab == 4 ? 3 : g_short_tab == 3 ? 2 : 1) * kClaimChunk;   // pairs per claim workgroup
        const dim3 gc((unsigned)std::max<uint64_t>((max_np + cc - 1) / cc, 1), nb);
#define DEC_CLAIM(SM)                                                                                          \
        k_dec_claim<SM><<<gc, 256, 0, s>>>(c, kt, vt, first, d_flag, d_flag + nb, key_cap, kv_base, kslot, vslot, \
                                           out->kv_key, out->kv_val, ctr)
        if (g_short_tab == 4) DEC_CLAIM(4);
        else if (g_short_tab == 3) DEC_CLAIM(3);
        else if (g_short_tab == 2) DEC_CLAIM(2);
        else if (g_short_tab == 1) DEC_CLAIM(1);
        else DEC_CLAIM(0);
#undef DEC_CLAIM
        rc = check_launch(ctx);
        if (rc) return rc;
    }
    // claims and flags to the host in one pinned copy: the id passes run only
    // when new strings arrived
    const size_t tail = fl_bytes + 64;
    char *h_tail = h_head + bd_bytes;
    const uint32_t *flags = (const uint32_t *)h_tail;
    const unsigned long long *h_ctr = (const unsigned long long *)(h_tail + fl_bytes);
    e = hipMemcpyAsync(h_tail, d_head + bd_bytes, tail, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return hip_fail(ctx, e);
    if (early) {
        rc = (*spec)();
        if (rc) {
            (void)hipStreamSynchronize(s);             // (the read-back into ctx->hio is in flight)
            return rc;
        }
    }
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(ctx, e);
    uint64_t new_k = 0, new_kb = 0, new_v = 0, new_vb = 0;
    if (h_ctr[0] || h_ctr[1]) {
        if (early && spec_stale) *spec_stale = true;
        const bool any_k = h_ctr[0] != 0, any_v = h_ctr[1] != 0;
        if (any_k) {
            rc = scan_lb(ctx, RepCntSrc{kslot}, NoAct(), n_p, 0, krank, tmp);
            if (!rc) rc = scan_lb(ctx, RepLenSrc{c, kslot, false}, NoAct(), n_p, 0, kboff, tmp);
            if (rc) return rc;
            k_dec_assign<<<grid_for(n_p, 256, cap), 256, 0, s>>>(c, kt, false, kslot, krank, kboff, kn0, kb0,
                                                                keys->bytes, keys->off);
            k_off_end<<<1, 1, 0, s>>>(keys->off, krank + n_p, kboff + n_p, kn0, kb0, ctr + 2);
        }
        if (any_v) {
            rc = scan_lb(ctx, RepCntSrc{vslot}, NoAct(), n_p, 0, vrank, tmp);
            if (!rc) rc = scan_lb(ctx, RepLenSrc{c, vslot, true}, NoAct(), n_p, 0, vboff, tmp);
            if (rc) return rc;
            k_dec_assign<<<grid_for(n_p, 256, cap), 256, 0, s>>>(c, vt, true, vslot, vrank, vboff, vn0, vb0,
                                                                vals->bytes, vals->off);
            k_off_end<<<1, 1, 0, s>>>(vals->off, vrank + n_p, vboff + n_p, vn0, vb0, ctr + 4);
        }
        k_dec_ids<<<grid_for(n_p, 256, cap), 256, 0, s>>>(c, kslot, vslot, keys->tab, vals->tab, key_cap,
                                                         kv_base, out->kv_key, out->kv_val);
        rc = check_launch(ctx);
        if (rc) return rc;
        e = hipMemcpyAsync(h_tail, d_head + bd_bytes, tail, hipMemcpyDeviceToHost, s);   // the id pass may flag a body too
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return hip_fail(ctx, e);
        if (any_k) new_k = h_ctr[2], new_kb = h_ctr[3];
        if (any_v) new_v = h_ctr[4], new_vb = h_ctr[5];
    }
    for (uint32_t b = 0; b < nb; ++b) {
        body_status[b] |= flags[b] | flags[nb + b];
        if (body_status[b] & kBodyMalformed) body_status[b] = kBodyMalformed;   // nothing else applies then
    }
    if (multi_pair) *multi_pair = h_ctr[6];
    rc = CRDT_OK;
    if (new_k) rc = tab_pull_new(ctx, keys, kn0 + new_k, kb0 + new_kb);
    if (!rc && new_v) rc = tab_pull_new(ctx, vals, vn0 + new_v, vb0 + new_vb);
    if (!rc && spec && !early) {
        rc = (*spec)();
        if (!rc) {
            e = hipStreamSynchronize(s);
            if (e != hipSuccess) return hip_fail(ctx, e);
        }
    }
    return rc;
}
}  // namespace crdt

extern "C" int crdt_gossip_decode(crdt_ctx *ctx, const crdt_gossip_bodies *in, crdt_strtab *keys,
                                  crdt_strtab *vals, const crdt_gossip_decoded *out, uint32_t *body_status) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!in || !keys || !vals || !out || !body_status) return CRDT_E_INVAL;
    if (keys->device != ctx->device || vals->device != ctx->device) return CRDT_E_INVAL;
    const uint32_t nb = in->n_bodies;
    if (nb == 0) return CRDT_OK;
    if (!in->data || !in->body_off || !in->slot_base || !out->r_off) return CRDT_E_INVAL;
    std::vector<uint64_t> at(nb), len(nb);
    for (uint32_t b = 0; b < nb; ++b) {
        if (in->body_off[b + 1] < in->body_off[b]) return CRDT_E_INVAL;
        at[b] = in->body_off[b];
        len[b] = in->body_off[b + 1] - in->body_off[b];
    }
    return gossip_decode_at(ctx, nb, in->data, at.data(), len.data(), in->key_cap, in->kv_base, in->slot_base,
                            in->host_hdr, keys, vals, out, body_status, nullptr, nullptr, 0, nullptr);
}

// Intern n strings [off[i], off[i+1]) of a device arena (host callers seeding
// a table): ids_dev[i] = the string's id.  Runs as a decode of one synthetic
// body would, via the same three passes.  Synchronises.
extern "C" int crdt_strtab_intern(crdt_ctx *ctx, crdt_strtab *t, const uint8_t *bytes_dev, const uint64_t *off_host,
                                  size_t n, uint32_t *ids_dev) {
    int rc = bind(ctx);
    if (rc) return rc;
    if (!t || (n && (!bytes_dev || !off_host || !ids_dev))) return CRDT_E_INVAL;
    if (n == 0) return CRDT_OK;
    if (n >= kPend) return CRDT_E_RANGE;
    // a synthetic body: n entries of one pair each, key = the string, value = ""
    const uint64_t nbytes = off_host[n] - off_host[0];
    std::vector<uint8_t> body(32 + 12 * n + 8 * n);
    memcpy(body.data(), "CRDTSOA1", 8);
    const uint64_t hdr[3] = {n, n, nbytes};
    memcpy(body.data() + 8, hdr, 24);
    for (size_t i = 0; i < n; ++i) {
        const int64_t ts = (int64_t)i;
        const uint32_t one = 1, kl = (uint32_t)(off_host[i + 1] - off_host[i]), vl = 0;
        memcpy(body.data() + 32 + 8 * i, &ts, 8);
        memcpy(body.data() + 32 + 8 * n + 4 * i, &one, 4);
        memcpy(body.data() + 32 + 12 * n + 4 * i, &kl, 4);
        memcpy(body.data() + 32 + 16 * n + 4 * i, &vl, 4);
    }
    uint8_t *d = nullptr;
    hipError_t e = hipMalloc(&d, body.size() + nbytes);
    if (e != hipSuccess) return hip_fail(ctx, e);
    e = hipMemcpyAsync(d, body.data(), body.size(), hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess && nbytes)
        e = hipMemcpyAsync(d + body.size(), bytes_dev + off_host[0], nbytes, hipMemcpyDeviceToDevice, ctx->stream);
    if (e != hipSuccess) {
        (void)hipFree(d);
        return hip_fail(ctx, e);
    }
    crdt_strtab *scratch = nullptr;                     // the synthetic values ("") go to a throwaway table
    rc = crdt_strtab_create(ctx, 16, 256, &scratch);
    if (rc) {
        (void)hipFree(d);
        return rc;
    }
    int64_t *r_ts = nullptr;
    uint64_t *r_kv = nullptr, *r_off = nullptr;
    uint32_t *vv = nullptr;
    e = hipMalloc(&r_ts, n * 8);
    if (e == hipSuccess) e = hipMalloc(&r_kv, (n + 1) * 8);
    if (e == hipSuccess) e = hipMalloc(&r_off, 16);
    if (e == hipSuccess) e = hipMalloc(&vv, n * 4);
    if (e == hipSuccess) {
        const uint64_t boff[2] = {0, body.size() + nbytes};
        const uint32_t sb = 0;
        crdt_gossip_bodies gb{1, 0xFFFFFFFFu, 0, d, boff, &sb, body.data()};
        crdt_gossip_decoded go{r_off, r_ts, r_kv, ids_dev, vv};
        uint32_t st = 0;
        rc = crdt_gossip_decode(ctx, &gb, t, scratch, &go, &st);
        if (!rc && (st & ~kBodyHost)) rc = (st & kBodyFull) ? CRDT_E_NOMEM : CRDT_E_INVAL;   // (order flags do not apply)
    } else {
        rc = hip_fail(ctx, e);
    }
    (void)hipStreamSynchronize(ctx->stream);
    for (void *p : {(void *)d, (void *)r_ts, (void *)r_kv, (void *)r_off, (void *)vv})
        if (p) (void)hipFree(p);
    (void)crdt_strtab_destroy(scratch);
    return rc;
}
