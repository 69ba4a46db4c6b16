// server.hip -- C++ host mirror of the reference's Server (main.go:23-113),
// with merge() routed to the batched gfx950 RefMerge (refmerge.hip).
//
// The reference's Go API surface this replaces:
//   type Server struct { InitialState, CurrentState Data; Diff, RemoteDiff
//                        treemap.Map; Port int; LastReceived int64;
//                        FriendList []string; Alive bool; Lock sync.Mutex }
//                                                            main.go:23-33
//   func NewServer(port int, initialState Data, friendList []string) *Server
//                                                            main.go:102-113
//   func (server *Server) merge()                            main.go:35-100
//   Diff.Put(time.Now().UnixMilli(), &data)   (local write)  main.go:187
//   RemoteDiff.Put(int64(atoi), value)        (gossip ingest) main.go:255
// The host keeps the treemaps (std::map under the signed int64 order of
// utils.Int64Comparator, main.go:106); merge() packs every participating
// server into one CSR batch, runs ONE device call, and rebuilds Diff and
// CurrentState from the device result.  There is no CPU merge path.
#include <algorithm>
#include <cstring>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "common.hpp"

namespace crdt {

struct Value {                       // map[string]string or *Command
    bool local = false;              // true: *Command (main.go:187), skipped by the replay
    bool nil = false;                // a nil map: pulled as JSON null (main.go:246), re-served as null
    std::vector<std::pair<std::string, std::string>> kv;   // unique keys
};

// A grow-only device buffer.
struct DBuf {
    void *p = nullptr;
    size_t cap = 0;
    template <class T> T *as() const { return (T *)p; }
};

// The Diff resident in HBM (SoA, the crdt_refmerge_in L layout of one
// replica): kv_key = key ids of the context's key table, kv_val = value
// string ids of its value table (also the merge's string arena).
struct DevDiff {
    DBuf ts, origin, kv_off, kv_key, kv_val;      // [n], [n], [n+1], [n_kv], [n_kv]
    uint64_t n = 0, n_kv = 0;
};

struct Server {
    crdt_ctx *ctx = nullptr;
    std::map<std::string, std::string> InitialState;        // main.go:24
    std::map<std::string, std::string> CurrentState;        // main.go:25 (aliases InitialState, :104-105)
    std::map<int64_t, std::shared_ptr<const Value>> Diff;   // main.go:26
    std::map<int64_t, std::shared_ptr<const Value>> RemoteDiff;  // main.go:27
    int Port = 0;                                           // main.go:28
    int64_t LastReceived = 0;                               // main.go:29 (unused by the reference)
    std::vector<std::string> FriendList;                    // main.go:30
    bool Alive = true;                                      // main.go:31
    std::mutex Lock;                                        // main.go:32
    std::vector<std::pair<std::string, std::string>> state_view;   // CurrentState snapshot for iteration
    // Device residency (servers with a context): the Diff lives in HBM
    // between merges; the host map above is a lazily rebuilt view.
    //   host_valid : Diff (the std::map) is current;
    //   dev_valid  : dd is current up to pend_cmds (local writes queued for
    //                the device, applied by crdt_local_apply at the next merge);
    //   pend       : one pulled binary body not yet parsed into RemoteDiff
    //                (the device decodes it straight into the merge's R).
    bool host_valid = true, dev_valid = false;
    DevDiff dd, dd2;                                        // current + next (swapped per merge)
    std::vector<std::pair<int64_t, std::shared_ptr<const Value>>> pend_cmds;
    char *pend_body = nullptr;         // pinned host copy of the parked pull
    size_t pend_len = 0, pend_cap = 0;
    bool pend = false;
    // The parked pull's H2D starts at ingest (into `pull`, on the context's
    // stream): it overlaps the host's validation of the next pulls instead of
    // sitting inside the merge.  pend_body is rewritten only by a later parked
    // pull, i.e. after a merge (which synchronises) or absorb_pending (which
    // drains the stream first).
    bool pend_dev = false;
    DBuf pull;
    // CurrentState as of the last device merge, per key id: kind (0 absent,
    // 1 string id, 2 sum), string id, sum.  While state_synced, CurrentState
    // is exactly the map these describe, and the next merge updates only the
    // keys whose words changed (main.go:76 rebuilds from empty: same result).
    std::vector<uint8_t> sk;
    std::vector<uint32_t> ss;
    std::vector<int64_t> su;
    bool state_synced = false;
    DBuf body, r_ts, r_kv, r_off, l_off, o_off, o_src, st_kind, st_str, st_sum, c_ts, c_kv, c_key, c_val, c_off,
        c_status;
};

static int io_reserve(crdt_ctx *ctx, size_t bytes) {
    if (bytes <= ctx->io_bytes) return CRDT_OK;
    size_t want = (bytes + bytes / 4 + (1u << 20)) & ~(size_t)((1u << 20) - 1);
    hipError_t e;
    if (ctx->io) {
        e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e);
        (void)hipFree(ctx->io);
        ctx->io = nullptr;
        ctx->io_bytes = 0;
    }
    e = hipMalloc(&ctx->io, want);
    if (e != hipSuccess) return hip_fail(ctx, e);
    ctx->io_bytes = want;
    return CRDT_OK;
}

// One host-side batch of replicas in the crdt_refmerge_in layout.
struct Batch {
    std::vector<uint64_t> l_off{0}, l_kv, r_off{0}, r_kv, str_off{0};
    std::vector<int64_t> l_ts, r_ts;
    std::vector<uint8_t> l_origin;
    std::vector<uint32_t> kv_key, kv_val;
    std::vector<uint32_t> slot_off{0};
    std::vector<const std::string *> slot_name;
    std::vector<std::shared_ptr<const Value>> l_val, r_val;
    std::string blob;
    std::unordered_map<std::string, uint32_t> sid;
    std::vector<std::pair<uint32_t, uint32_t>> l_pairs, r_pairs;   // (slot, string) before arena layout
    std::vector<uint64_t> l_cnt, r_cnt;

    uint32_t str_id(const std::string &s) {
        auto it = sid.find(s);
        if (it != sid.end()) return it->second;
        uint32_t id = (uint32_t)(str_off.size() - 1);
        sid.emplace(s, id);
        blob += s;
        str_off.push_back(blob.size());
        return id;
    }

    void add(Server &s) {
        std::unordered_map<std::string, uint32_t> slots;
        auto slot = [&](const std::string &k) {
            auto it = slots.find(k);
            if (it != slots.end()) return it->second;
            uint32_t id = (uint32_t)slot_name.size();
            slots.emplace(k, id);
            slot_name.push_back(&k);
            return id;
        };
        for (auto &e : s.Diff) {
            l_ts.push_back(e.first);
            l_origin.push_back(e.second->local ? 1 : 0);
            l_val.push_back(e.second);
            l_cnt.push_back(e.second->kv.size());
            for (auto &kv : e.second->kv) l_pairs.emplace_back(slot(kv.first), str_id(kv.second));
        }
        for (auto &e : s.RemoteDiff) {
            r_ts.push_back(e.first);
            r_val.push_back(e.second);
            r_cnt.push_back(e.second->kv.size());
            for (auto &kv : e.second->kv) r_pairs.emplace_back(slot(kv.first), str_id(kv.second));
        }
        l_off.push_back(l_ts.size());
        r_off.push_back(r_ts.size());
        slot_off.push_back((uint32_t)slot_name.size());
    }

    void finish() {
        // kv arena: every L entry's pairs, then every R entry's pairs
        l_kv.reserve(l_cnt.size() + 1);
        uint64_t q = 0;
        for (auto c : l_cnt) { l_kv.push_back(q); q += c; }
        l_kv.push_back(q);
        for (auto c : r_cnt) { r_kv.push_back(q); q += c; }
        r_kv.push_back(q);
        kv_key.reserve(q);
        kv_val.reserve(q);
        for (auto &p : l_pairs) { kv_key.push_back(p.first); kv_val.push_back(p.second); }
        for (auto &p : r_pairs) { kv_key.push_back(p.first); kv_val.push_back(p.second); }
        if (blob.empty()) blob.push_back('\0');
    }
};

template <class T> static size_t vbytes(const std::vector<T> &v) { return v.size() * sizeof(T); }

// merge() for a set of servers whose locks the caller holds.
// Device failure flags raised by the passes of one merge: while a
// StatusScope lives, the context's kernels raise their flags into a spare
// word of the status buffer (word 2, zero between merges) -- a host-side
// pointer swap, no GPU work -- and the merge's one host synchronisation reads
// it beside the caller's word 0.  A raised flag is folded into word 0 (it
// stays for crdt_ctx_device_status) and the spare word cleared; so is a
// scope left on an error path before the check.
struct StatusScope {
    crdt_ctx *ctx;
    uint32_t *saved;
    bool settled = false;
    explicit StatusScope(crdt_ctx *c) : ctx(c), saved(c->dev_status) { c->dev_status = saved + 2; }
    ~StatusScope() {
        ctx->dev_status = saved;
        if (!settled) (void)hipMemsetAsync(saved + 2, 0, 4, ctx->stream);   // (an error path: maybe dirty)
    }
    // words 0..2 of the status buffer to host memory (before the merge's synchronisation)
    hipError_t fetch(uint32_t *three) const {
        return hipMemcpyAsync(three, saved, 12, hipMemcpyDeviceToHost, ctx->stream);
    }
    // (after the synchronisation) true when a pass of this merge raised a flag
    bool raised(const uint32_t *three) {
        settled = true;
        if (!three[2]) return false;
        (void)hipMemsetD32Async((hipDeviceptr_t)saved, (int)(three[0] | three[2]), 1, ctx->stream);
        (void)hipMemsetAsync(saved + 2, 0, 4, ctx->stream);
        return true;
    }
};

static int merge_locked(crdt_ctx *ctx, Server *const *srv, size_t n) {
    Batch b;
    for (size_t i = 0; i < n; ++i) b.add(*srv[i]);
    b.finish();
    const uint64_t n_l = b.l_ts.size(), n_r = b.r_ts.size(), n_kv = b.kv_key.size();
    const uint64_t n_str = b.str_off.size() - 1, n_slots = b.slot_name.size();
    if (n_slots >= 0xFFFFFFFFull || n_str >= 0xFFFFFFFFull) return CRDT_E_RANGE;
    const uint64_t n_out = n_l + n_r;

    // device layout: inputs then outputs, 256-B aligned carve-outs
    struct Piece { const void *src; size_t bytes; size_t off; };
    std::vector<Piece> in = {
        {b.l_off.data(), vbytes(b.l_off), 0}, {b.l_ts.data(), vbytes(b.l_ts), 0},
        {b.l_origin.data(), vbytes(b.l_origin), 0}, {b.l_kv.data(), vbytes(b.l_kv), 0},
        {b.r_off.data(), vbytes(b.r_off), 0}, {b.r_ts.data(), vbytes(b.r_ts), 0},
        {b.r_kv.data(), vbytes(b.r_kv), 0}, {b.kv_key.data(), vbytes(b.kv_key), 0},
        {b.kv_val.data(), vbytes(b.kv_val), 0}, {b.blob.data(), b.blob.size(), 0},
        {b.str_off.data(), vbytes(b.str_off), 0},
    };
    size_t off = 0;
    for (auto &p : in) { p.off = off; off += Carve::round(p.bytes ? p.bytes : 1); }
    const size_t o_off = off;            off += Carve::round((n + 1) * 8);
    const size_t o_ts = off;             off += Carve::round(n_out * 8 + 8);
    const size_t o_origin = off;         off += Carve::round(n_out + 1);
    const size_t o_src = off;            off += Carve::round(n_out * 8 + 8);
    const size_t o_kind = off;           off += Carve::round(n_slots + 1);
    const size_t o_str = off;            off += Carve::round(n_slots * 4 + 4);
    const size_t o_sum = off;            off += Carve::round(n_slots * 8 + 8);
    int rc = io_reserve(ctx, off);
    if (rc) return rc;
    char *d = (char *)ctx->io;
    for (auto &p : in)
        if (p.bytes) {
            hipError_t e = hipMemcpyAsync(d + p.off, p.src, p.bytes, hipMemcpyHostToDevice, ctx->stream);
            if (e != hipSuccess) return hip_fail(ctx, e);
        }
    crdt_refmerge_in ri;
    ri.replicas = (uint32_t)n;
    ri.n_slots = (uint32_t)n_slots;
    ri.n_l = n_l; ri.n_r = n_r; ri.n_kv = n_kv; ri.n_str = n_str;
    ri.l_off = (const uint64_t *)(d + in[0].off);
    ri.l_ts = (const int64_t *)(d + in[1].off);
    ri.l_origin = (const uint8_t *)(d + in[2].off);
    ri.l_kv = (const uint64_t *)(d + in[3].off);
    ri.r_off = (const uint64_t *)(d + in[4].off);
    ri.r_ts = (const int64_t *)(d + in[5].off);
    ri.r_kv = (const uint64_t *)(d + in[6].off);
    ri.kv_key = (const uint32_t *)(d + in[7].off);
    ri.kv_val = (const uint32_t *)(d + in[8].off);
    ri.str_bytes = (const uint8_t *)(d + in[9].off);
    ri.str_off = (const uint64_t *)(d + in[10].off);
    crdt_refmerge_out ro;
    ro.off = (uint64_t *)(d + o_off);
    ro.ts = (int64_t *)(d + o_ts);
    ro.origin = (uint8_t *)(d + o_origin);
    ro.src = (int64_t *)(d + o_src);
    ro.st_kind = (uint8_t *)(d + o_kind);
    ro.st_str = (uint32_t *)(d + o_str);
    ro.st_sum = (int64_t *)(d + o_sum);
    StatusScope sc(ctx);
    rc = crdt_refmerge_batch(ctx, &ri, &ro);
    if (rc) return rc;

    std::vector<uint64_t> h_off(n + 1);
    std::vector<int64_t> h_ts(n_out), h_src(n_out);
    std::vector<uint8_t> h_kind(n_slots);
    std::vector<uint32_t> h_str(n_slots);
    std::vector<int64_t> h_sum(n_slots);
    struct Back { void *dst; size_t src; size_t bytes; };
    const Back back[] = {{h_off.data(), o_off, vbytes(h_off)}, {h_ts.data(), o_ts, vbytes(h_ts)},
                         {h_src.data(), o_src, vbytes(h_src)}, {h_kind.data(), o_kind, vbytes(h_kind)},
                         {h_str.data(), o_str, vbytes(h_str)}, {h_sum.data(), o_sum, vbytes(h_sum)}};
    for (auto &x : back)
        if (x.bytes) {
            hipError_t e = hipMemcpyAsync(x.dst, d + x.src, x.bytes, hipMemcpyDeviceToHost, ctx->stream);
            if (e != hipSuccess) return hip_fail(ctx, e);
        }
    uint32_t fl[3] = {0, 0, 0};
    hipError_t e = sc.fetch(fl);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
    if (sc.raised(fl)) return CRDT_E_DEVICE;                     // nothing below ran: the servers are untouched

    for (size_t p = 0; p < n; ++p) {
        Server &s = *srv[p];
        std::map<int64_t, std::shared_ptr<const Value>> nd;
        for (uint64_t o = h_off[p]; o < h_off[p + 1]; ++o) {
            const int64_t src = h_src[o];
            nd.emplace_hint(nd.end(), h_ts[o], src >= 0 ? b.l_val[(size_t)src] : b.r_val[(size_t)(-src - 1)]);
        }
        std::map<std::string, std::string> st;                 // main.go:76: rebuilt from empty
        for (uint32_t sl = b.slot_off[p]; sl < b.slot_off[p + 1]; ++sl) {
            if (h_kind[sl] == 1) {
                const uint32_t id = h_str[sl];
                st.emplace(*b.slot_name[sl], b.blob.substr(b.str_off[id], b.str_off[id + 1] - b.str_off[id]));
            } else if (h_kind[sl] == 2) {
                st.emplace(*b.slot_name[sl], std::to_string((long long)h_sum[sl]));   // strconv.Itoa
            }
        }
        s.Diff.swap(nd);
        s.RemoteDiff.clear();                                    // main.go:75
        s.CurrentState.swap(st);
        s.state_view.clear();
        s.state_synced = false;                                  // (no per-key words of this map)
        s.Alive = true;                                          // main.go:99
    }
    return CRDT_OK;
}

static std::shared_ptr<const Value> make_value(bool local, const char *const *keys, const size_t *klen,
                                               const char *const *vals, const size_t *vlen, size_t n) {
    auto v = std::make_shared<Value>();
    v->local = local;
    std::map<std::string, std::string> m;                       // map semantics: a repeated key overwrites
    for (size_t i = 0; i < n; ++i) m[std::string(keys[i], klen[i])] = std::string(vals[i], vlen[i]);
    v->kv.assign(m.begin(), m.end());
    return v;
}

// ---------------------------------------------------------------- device residency
// The binary SoA body of a treemap (crdt_server_gossip_binary's format):
// entries ascending, pairs of an entry sorted by key, nil maps as 0xFFFFFFFF.
constexpr uint32_t kNilPairsH = 0xFFFFFFFFu;
constexpr size_t kLocalMaxCmd = 4096;         // crdt_local_apply: commands per replica per call

static void put_u32(std::string &o, uint32_t v) { o.append((const char *)&v, 4); }
static void put_u64(std::string &o, uint64_t v) { o.append((const char *)&v, 8); }

static void encode_soa(const std::map<int64_t, std::shared_ptr<const Value>> &m, std::string &body) {
    uint64_t np = 0, nb = 0;
    for (auto &e : m) {
        np += e.second->kv.size();
        for (auto &x : e.second->kv) nb += x.first.size() + x.second.size();
    }
    body.clear();
    body.reserve(32 + 12 * m.size() + 8 * np + nb);
    body.append("CRDTSOA1", 8);
    put_u64(body, m.size());
    put_u64(body, np);
    put_u64(body, nb);
    for (auto &e : m) put_u64(body, (uint64_t)e.first);
    for (auto &e : m) put_u32(body, e.second->nil ? kNilPairsH : (uint32_t)e.second->kv.size());
    for (auto &e : m)                                  // Value::kv is key-sorted (make_value / ingest)
        for (auto &x : e.second->kv) put_u32(body, (uint32_t)x.first.size());
    for (auto &e : m)
        for (auto &x : e.second->kv) put_u32(body, (uint32_t)x.second.size());
    for (auto &e : m)
        for (auto &x : e.second->kv) {
            body += x.first;
            body += x.second;
        }
}

static bool has_nil(const std::map<int64_t, std::shared_ptr<const Value>> &m) {
    for (auto &e : m)
        if (e.second->nil) return true;
    return false;
}

static int dbuf(crdt_ctx *ctx, DBuf &b, size_t bytes, size_t keep = 0) {
    if (bytes <= b.cap) return CRDT_OK;
    const size_t want = std::max<size_t>(bytes + bytes / 2, 4096);
    void *q = nullptr;
    hipError_t e = hipMalloc(&q, want);
    if (e != hipSuccess) return hip_fail(ctx, e);
    if (b.p) {
        if (keep) e = hipMemcpyAsync(q, b.p, std::min(keep, b.cap), hipMemcpyDeviceToDevice, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        (void)hipFree(b.p);
        if (e != hipSuccess) {
            (void)hipFree(q);
            b.p = nullptr;
            b.cap = 0;
            return hip_fail(ctx, e);
        }
    }
    b.p = q;
    b.cap = want;
    return CRDT_OK;
}

static void dbuf_free(DBuf &b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
}

// Pinned host staging of the context (grow-only; the stream is drained first).
static int pinned_reserve(crdt_ctx *ctx, size_t bytes) {
    if (bytes <= ctx->pinned_bytes) return CRDT_OK;
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    ctx->pinned = nullptr;
    ctx->pinned_bytes = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 2, 1 << 20);
    e = hipHostMalloc(&ctx->pinned, want, 0);
    if (e != hipSuccess) {
        ctx->pinned = nullptr;
        return hip_fail(ctx, e);
    }
    ctx->pinned_bytes = want;
    return CRDT_OK;
}

static int ctx_tables(crdt_ctx *ctx) {
    int rc = CRDT_OK;
    if (!ctx->keys) rc = crdt_strtab_create(ctx, 1024, 1 << 14, &ctx->keys);
    if (!rc && !ctx->vals) rc = crdt_strtab_create(ctx, 1024, 1 << 16, &ctx->vals);
    return rc;
}

static std::string tab_str(const crdt_strtab *t, uint64_t id) {
    const char *p = nullptr;
    size_t n = 0;
    if (crdt_strtab_get(t, id, &p, &n) != CRDT_OK) return std::string();
    return std::string(p, n);
}

// H2D a body and decode it with the context's tables: entries -> r_ts /
// r_kv (+ kv_base), pairs -> kv_key / kv_val at kv_base.  *status = the
// body's decode status (0: taken).
// on_dev: body_dev already holds the body (a pull uploaded at ingest).
static int dev_decode(crdt_ctx *ctx, DBuf &body_dev, const char *body, size_t len, bool pinned, bool on_dev,
                      uint64_t kv_base, int64_t *r_ts, uint64_t *r_kv, uint64_t *r_off, uint32_t *kv_key,
                      uint32_t *kv_val, uint32_t *status) {
    if (!on_dev) {
        int rc = dbuf(ctx, body_dev, len);
        if (!rc && !pinned) rc = pinned_reserve(ctx, len);
        if (rc) return rc;
        if (!pinned) memcpy(ctx->pinned, body, len);
        hipError_t e = hipMemcpyAsync(body_dev.p, pinned ? body : ctx->pinned, len, hipMemcpyHostToDevice, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e);
    }
    const uint64_t boff[2] = {0, len};
    const uint32_t sb = 0;
    crdt_gossip_bodies gb{1, 0xFFFFFFFFu, kv_base, body_dev.as<uint8_t>(), boff, &sb,
                          len >= 32 ? (const uint8_t *)body : nullptr};
    crdt_gossip_decoded go{r_off, r_ts, r_kv, kv_key, kv_val};
    return crdt_gossip_decode(ctx, &gb, ctx->keys, ctx->vals, &go, status);
}

static uint64_t body_u64(const std::string &b, size_t at) {
    uint64_t v = 0;
    memcpy(&v, b.data() + at, 8);
    return v;
}

// Upload the host Diff (nil-free) into dd: decode its body; origin from the host.
static int dev_upload(crdt_ctx *ctx, Server &s) {
    std::string body;
    encode_soa(s.Diff, body);
    const uint64_t ne = s.Diff.size(), np = body_u64(body, 16);
    int rc = dbuf(ctx, s.dd.ts, ne * 8 + 8);
    if (!rc) rc = dbuf(ctx, s.dd.origin, ne + 1);
    if (!rc) rc = dbuf(ctx, s.dd.kv_off, (ne + 1) * 8);
    if (!rc) rc = dbuf(ctx, s.dd.kv_key, np * 4 + 4);
    if (!rc) rc = dbuf(ctx, s.dd.kv_val, np * 4 + 4);
    if (!rc) rc = dbuf(ctx, s.r_off, 16);
    if (rc) return rc;
    uint32_t st = 0;
    rc = dev_decode(ctx, s.body, body.data(), body.size(), false, false, 0, s.dd.ts.as<int64_t>(), s.dd.kv_off.as<uint64_t>(),
                    s.r_off.as<uint64_t>(), s.dd.kv_key.as<uint32_t>(), s.dd.kv_val.as<uint32_t>(), &st);
    if (rc) return rc;
    if (st) return CRDT_E_UNSORTED;                   // (never: a treemap's body is ascending and nil-free)
    std::vector<uint8_t> org;
    org.reserve(ne);
    for (auto &e : s.Diff) org.push_back(e.second->local ? 1 : 0);
    if (ne) {
        hipError_t e = hipMemcpyAsync(s.dd.origin.p, org.data(), ne, hipMemcpyHostToDevice, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);   // org is a local
        if (e != hipSuccess) return hip_fail(ctx, e);
    }
    s.dd.n = ne;
    s.dd.n_kv = np;
    s.dev_valid = true;
    s.pend_cmds.clear();
    return CRDT_OK;
}

// Rebuild the host Diff from dd (then the queued local writes on top).
static int make_host(Server &s) {
    if (s.host_valid) return CRDT_OK;
    crdt_ctx *ctx = s.ctx;
    const uint64_t n = s.dd.n, nk = s.dd.n_kv;
    std::vector<int64_t> ts(n);
    std::vector<uint8_t> org(n);
    std::vector<uint64_t> ko(n + 1);
    std::vector<uint32_t> kk(nk), kv(nk);
    hipError_t e = hipSuccess;
    if (n) e = hipMemcpyAsync(ts.data(), s.dd.ts.p, n * 8, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && n) e = hipMemcpyAsync(org.data(), s.dd.origin.p, n, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(ko.data(), s.dd.kv_off.p, (n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && nk) e = hipMemcpyAsync(kk.data(), s.dd.kv_key.p, nk * 4, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && nk) e = hipMemcpyAsync(kv.data(), s.dd.kv_val.p, nk * 4, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
    std::vector<std::string> kname, vname;             // the tables' strings, by id
    uint64_t nks = 0, nvs = 0, b0 = 0;
    (void)crdt_strtab_info(ctx->keys, &nks, &b0, nullptr, nullptr);
    (void)crdt_strtab_info(ctx->vals, &nvs, &b0, nullptr, nullptr);
    kname.reserve(nks);
    for (uint64_t i = 0; i < nks; ++i) kname.push_back(tab_str(ctx->keys, i));
    vname.reserve(nvs);
    for (uint64_t i = 0; i < nvs; ++i) vname.push_back(tab_str(ctx->vals, i));
    std::map<int64_t, std::shared_ptr<const Value>> m;
    for (uint64_t i = 0; i < n; ++i) {
        auto v = std::make_shared<Value>();
        v->local = org[i] != 0;
        for (uint64_t q = ko[i] - ko[0]; q < ko[i + 1] - ko[0]; ++q)
            v->kv.emplace_back(kk[q] < nks ? kname[kk[q]] : std::string(), kv[q] < nvs ? vname[kv[q]] : std::string());
        m.emplace_hint(m.end(), ts[i], std::move(v));
    }
    for (auto &c : s.pend_cmds) m[c.first] = c.second;   // queued local writes (same-ms: the later one)
    s.Diff.swap(m);
    s.host_valid = true;
    return CRDT_OK;
}

// The pulled binary body parked for the device becomes RemoteDiff entries
// (a reader of RemoteDiff, or a second pull before the merge).
static void parse_soa_into(Server &s, const char *data, size_t len);
static void absorb_pending(Server &s) {
    if (!s.pend) return;
    // an upload started at ingest may still read pend_body, which the next
    // parked pull overwrites: drain it first (every merge synchronises anyway)
    if (s.pend_dev && s.ctx && bind(s.ctx) == CRDT_OK) (void)hipStreamSynchronize(s.ctx->stream);
    s.pend = false;
    s.pend_dev = false;
    parse_soa_into(s, s.pend_body, s.pend_len);
}

// Apply one chunk of the queued local writes (distinct ts, at most
// kLocalMaxCmd: crdt_local_apply's per-replica limit) to dd.
static int dev_flush_chunk(crdt_ctx *ctx, Server &s, const std::map<int64_t, std::shared_ptr<const Value>> &cm) {
    std::string body;
    encode_soa(cm, body);
    const uint64_t nc = cm.size(), np = body_u64(body, 16);
    int rc = dbuf(ctx, s.c_ts, nc * 8 + 8);
    if (!rc) rc = dbuf(ctx, s.c_kv, (nc + 1) * 8);
    if (!rc) rc = dbuf(ctx, s.c_key, np * 4 + 4);
    if (!rc) rc = dbuf(ctx, s.c_val, np * 4 + 4);
    if (!rc) rc = dbuf(ctx, s.c_off, 16);
    if (!rc) rc = dbuf(ctx, s.l_off, 16);
    if (!rc) rc = dbuf(ctx, s.o_off, 16);
    if (!rc) rc = dbuf(ctx, s.o_src, (s.dd.n + nc) * 8 + 8);
    if (!rc) rc = dbuf(ctx, s.c_status, nc * 2 + 2);
    if (!rc) rc = dbuf(ctx, s.dd2.ts, (s.dd.n + nc) * 8 + 8);
    if (!rc) rc = dbuf(ctx, s.dd2.origin, s.dd.n + nc + 1);
    if (!rc) rc = dbuf(ctx, s.dd2.kv_off, (s.dd.n + nc + 1) * 8);
    if (!rc) rc = dbuf(ctx, s.dd2.kv_key, (s.dd.n_kv + np) * 4 + 4);
    if (!rc) rc = dbuf(ctx, s.dd2.kv_val, (s.dd.n_kv + np) * 4 + 4);
    if (rc) return rc;
    uint32_t st = 0;
    rc = dev_decode(ctx, s.body, body.data(), body.size(), false, false, 0, s.c_ts.as<int64_t>(), s.c_kv.as<uint64_t>(),
                    s.c_off.as<uint64_t>(), s.c_key.as<uint32_t>(), s.c_val.as<uint32_t>(), &st);
    if (rc) return rc;
    if (st) return CRDT_E_UNSORTED;
    const uint64_t loff[2] = {0, s.dd.n};
    hipError_t e = hipMemcpyAsync(s.l_off.p, loff, 16, hipMemcpyHostToDevice, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
    uint64_t nstr = 0, b0 = 0;
    const uint8_t *sb = nullptr;
    const uint64_t *so = nullptr;
    (void)crdt_strtab_info(ctx->vals, &nstr, &b0, &sb, &so);
    crdt_local_in li{1, 0, s.dd.n, nc, np, nstr, s.l_off.as<uint64_t>(), s.dd.ts.as<int64_t>(),
                     s.dd.origin.as<uint8_t>(), s.c_off.as<uint64_t>(), s.c_ts.as<int64_t>(), s.c_kv.as<uint64_t>(),
                     s.c_key.as<uint32_t>(), s.c_val.as<uint32_t>(), sb, so};
    crdt_local_out lo{s.o_off.as<uint64_t>(), s.dd2.ts.as<int64_t>(), s.dd2.origin.as<uint8_t>(),
                      s.o_src.as<int64_t>(), s.c_status.as<uint16_t>(), nullptr, nullptr, nullptr};
    StatusScope sc(ctx);
    rc = crdt_local_apply(ctx, &li, &lo);
    if (rc) return rc;
    uint64_t oo[2] = {0, 0};
    uint32_t fl[3] = {0, 0, 0};
    e = hipMemcpyAsync(oo, s.o_off.p, 16, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = sc.fetch(fl);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
    if (sc.raised(fl)) return CRDT_E_DEVICE;                // dd untouched (the swap below never ran)
    const uint64_t n_out = oo[1];
    rc = crdt_seg_gather2(ctx, n_out, s.o_src.as<int64_t>(), s.dd.kv_off.as<uint64_t>(), s.c_kv.as<uint64_t>(), 0,
                          s.dd2.kv_off.as<uint64_t>(), 4, s.dd.kv_key.p, s.c_key.p, s.dd2.kv_key.p, s.dd.kv_val.p,
                          s.c_val.p, s.dd2.kv_val.p);
    if (rc) return rc;
    uint64_t nkv = 0;
    e = hipMemcpyAsync(&nkv, s.dd2.kv_off.as<uint64_t>() + n_out, 8, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
    std::swap(s.dd, s.dd2);
    s.dd.n = n_out;
    s.dd.n_kv = nkv;
    return CRDT_OK;
}

// Apply the queued local writes to dd (crdt_local_apply, Diff only: the
// CurrentState apply already ran on the host when each write arrived), in
// chunks of at most kLocalMaxCmd distinct timestamps.  A chunk that fails
// leaves dd as the previous chunks made it and pend_cmds whole: re-applying
// an applied chunk is a no-op (Put of the same value at the same ts).
static int dev_flush_cmds(crdt_ctx *ctx, Server &s) {
    if (s.pend_cmds.empty()) return CRDT_OK;
    std::map<int64_t, std::shared_ptr<const Value>> all;  // Put replaces: the last same-ms write stays
    for (auto &c : s.pend_cmds) all[c.first] = c.second;
    auto it = all.begin();
    while (it != all.end()) {
        std::map<int64_t, std::shared_ptr<const Value>> cm;
        for (size_t k = 0; k < kLocalMaxCmd && it != all.end(); ++k, ++it) cm.emplace_hint(cm.end(), *it);
        const int rc = dev_flush_chunk(ctx, s, cm);
        if (rc) return rc;
    }
    s.pend_cmds.clear();
    return CRDT_OK;
}

// CurrentState from the merge's per-key words (main.go:76-96: rebuilt from
// empty; kind 1 = the string id's value, 2 = Itoa(sum), else absent), kind /
// str / sum indexed by key id, n = the key table's size.  While the previous
// words still describe CurrentState (no AddCommand or host merge since), only
// the keys whose words changed are touched -- the same map as a rebuild.
static void apply_state(crdt_ctx *ctx, Server &s, const uint8_t *kind, const uint32_t *str, const int64_t *sum,
                        uint64_t n) {
    auto kd = [](uint8_t k) -> uint8_t { return k == 1 || k == 2 ? k : 0; };
    auto text = [&](uint8_t k, uint32_t id, int64_t v) {
        return k == 1 ? tab_str(ctx->vals, id) : std::to_string((long long)v);   // strconv.Itoa
    };
    if (!s.state_synced) {
        std::map<std::string, std::string> st;
        for (uint64_t k = 0; k < n; ++k)
            if (kd(kind[k])) st.emplace(tab_str(ctx->keys, k), text(kind[k], str[k], sum[k]));
        s.CurrentState.swap(st);
        s.state_view.clear();
    } else {
        bool changed = false;
        const uint64_t old = s.sk.size();
        for (uint64_t k = 0; k < std::max(n, old); ++k) {
            const uint8_t a = k < old ? s.sk[k] : 0, b = k < n ? kd(kind[k]) : 0;
            if (a == b && (b == 0 || (b == 1 ? s.ss[k] == str[k] : s.su[k] == sum[k]))) continue;
            changed = true;
            if (b == 0) s.CurrentState.erase(tab_str(ctx->keys, k));
            else s.CurrentState[tab_str(ctx->keys, k)] = text(b, str[k], sum[k]);
        }
        if (changed) s.state_view.clear();
    }
    s.sk.resize(n);
    for (uint64_t k = 0; k < n; ++k) s.sk[k] = kd(kind[k]);
    s.ss.assign(str, str + n);
    s.su.assign(sum, sum + n);
    s.state_synced = true;
}

// merge() (main.go:35-100) of one device-resident server: the pull decoded
// on the device into R, the batched RefMerge with this Diff as L, the next
// Diff gathered in HBM; only CurrentState (one word per key slot) comes back.
static int dev_merge_one(crdt_ctx *ctx, Server &s) {
    int rc;
    if (!s.dev_valid) {
        rc = dev_upload(ctx, s);
        if (rc) return rc;
    }
    rc = dev_flush_cmds(ctx, s);
    if (rc) return rc;
    std::string rbody;
    if (!s.pend) encode_soa(s.RemoteDiff, rbody);
    const char *rp = s.pend ? s.pend_body : rbody.data();
    const size_t rlen = s.pend ? s.pend_len : rbody.size();
    uint64_t ne, np;
    memcpy(&ne, rp + 8, 8);
    memcpy(&np, rp + 16, 8);
    const uint64_t nl = s.dd.n, nkv = s.dd.n_kv;
    rc = dbuf(ctx, s.dd.kv_key, (nkv + np) * 4 + 4, nkv * 4);     // R's pairs go behind L's
    if (!rc) rc = dbuf(ctx, s.dd.kv_val, (nkv + np) * 4 + 4, nkv * 4);
    if (!rc) rc = dbuf(ctx, s.r_ts, ne * 8 + 8);
    if (!rc) rc = dbuf(ctx, s.r_kv, (ne + 1) * 8);
    if (!rc) rc = dbuf(ctx, s.r_off, 16);
    if (!rc) rc = dbuf(ctx, s.l_off, 16);
    if (!rc) rc = dbuf(ctx, s.o_off, 16);
    if (!rc) rc = dbuf(ctx, s.o_src, (nl + ne) * 8 + 8);
    if (!rc) rc = dbuf(ctx, s.dd2.ts, (nl + ne) * 8 + 8);
    if (!rc) rc = dbuf(ctx, s.dd2.origin, nl + ne + 1);
    if (!rc) rc = dbuf(ctx, s.dd2.kv_off, (nl + ne + 1) * 8);
    if (!rc) rc = dbuf(ctx, s.dd2.kv_key, (nkv + np) * 4 + 4);
    if (!rc) rc = dbuf(ctx, s.dd2.kv_val, (nkv + np) * 4 + 4);
    if (rc) return rc;
    uint32_t st = 0;
    const bool on_dev = s.pend && s.pend_dev;
    rc = dev_decode(ctx, on_dev ? s.pull : s.body, rp, rlen, s.pend, on_dev, nkv, s.r_ts.as<int64_t>(), s.r_kv.as<uint64_t>(),
                    s.r_off.as<uint64_t>(), s.dd.kv_key.as<uint32_t>(), s.dd.kv_val.as<uint32_t>(), &st);
    if (rc) return rc;
    if (st) return CRDT_E_UNSORTED;                   // (callers route such pulls to the host path first)
    uint64_t nks = 0, nstr = 0, b0 = 0;
    const uint8_t *sb = nullptr;
    const uint64_t *so = nullptr;
    (void)crdt_strtab_info(ctx->keys, &nks, &b0, nullptr, nullptr);
    (void)crdt_strtab_info(ctx->vals, &nstr, &b0, &sb, &so);
    if (nks >= 0xFFFFFFFFull) return CRDT_E_RANGE;
    rc = dbuf(ctx, s.st_kind, nks + 1);
    if (!rc) rc = dbuf(ctx, s.st_str, nks * 4 + 4);
    if (!rc) rc = dbuf(ctx, s.st_sum, nks * 8 + 8);
    // pinned staging (the decode above has synchronised: ctx->hio is free):
    // [l_off | entry count | pair total | status | sum | str | kind]
    const size_t h_sum = 64, h_str = h_sum + Carve::round(nks * 8 + 8), h_kind = h_str + Carve::round(nks * 4 + 4);
    if (!rc) rc = hio_reserve(ctx, h_kind + nks + 1);
    if (rc) return rc;
    char *hio = (char *)ctx->hio;
    uint64_t *loff = (uint64_t *)hio, *oo = loff + 2, *new_nkv = loff + 4;
    uint32_t *fl = (uint32_t *)(loff + 5);
    loff[0] = 0;
    loff[1] = nl;
    hipError_t e = hipMemcpyAsync(s.l_off.p, loff, 16, hipMemcpyHostToDevice, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
    crdt_refmerge_in ri;
    ri.replicas = 1;
    ri.n_slots = (uint32_t)nks;                       // slot = key id (one replica)
    ri.n_l = nl;
    ri.n_r = ne;
    ri.n_kv = nkv + np;
    ri.n_str = nstr;
    ri.l_off = s.l_off.as<uint64_t>();
    ri.l_ts = s.dd.ts.as<int64_t>();
    ri.l_origin = s.dd.origin.as<uint8_t>();
    ri.l_kv = s.dd.kv_off.as<uint64_t>();
    ri.r_off = s.r_off.as<uint64_t>();
    ri.r_ts = s.r_ts.as<int64_t>();
    ri.r_kv = s.r_kv.as<uint64_t>();
    ri.kv_key = s.dd.kv_key.as<uint32_t>();
    ri.kv_val = s.dd.kv_val.as<uint32_t>();
    ri.str_bytes = sb;
    ri.str_off = so;
    crdt_refmerge_out ro{s.o_off.as<uint64_t>(), s.dd2.ts.as<int64_t>(), s.dd2.origin.as<uint8_t>(),
                         s.o_src.as<int64_t>(), s.st_kind.as<uint8_t>(), s.st_str.as<uint32_t>(),
                         s.st_sum.as<int64_t>()};
    StatusScope sc(ctx);
    // the merge and the new Diff's kv pairs (copied by the merge's tile pass;
    // its entry count stays on the device, dd2 is sized for |L| + |R| and the
    // pair total also lands at kv_off[|L| + |R|]): one host synchronisation
    const crdt_refmerge_kv_out kvo{s.dd2.kv_off.as<uint64_t>(), s.dd2.kv_key.as<uint32_t>(),
                                   s.dd2.kv_val.as<uint32_t>(), nkv + np};
    rc = crdt_refmerge_batch_kv(ctx, &ri, &ro, &kvo);
    if (rc) return rc;
    // CurrentState (main.go:76-96: rebuilt from empty), the entry count and
    // the new pair count (every dst offset from the entry count on = the total)
    uint8_t *kind = (uint8_t *)(hio + h_kind);
    uint32_t *sstr = (uint32_t *)(hio + h_str);
    int64_t *ssum = (int64_t *)(hio + h_sum);
    e = hipMemcpyAsync(oo, s.o_off.p, 16, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(new_nkv, s.dd2.kv_off.as<uint64_t>() + nl + ne, 8, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && nks) e = hipMemcpyAsync(kind, s.st_kind.p, nks, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && nks) e = hipMemcpyAsync(sstr, s.st_str.p, nks * 4, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && nks) e = hipMemcpyAsync(ssum, s.st_sum.p, nks * 8, hipMemcpyDeviceToHost, ctx->stream);
    fl[0] = fl[1] = fl[2] = 0;
    if (e == hipSuccess) e = sc.fetch(fl);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
    if (sc.raised(fl)) return CRDT_E_DEVICE;                // dd / RemoteDiff untouched (the swap below never ran)
    apply_state(ctx, s, kind, sstr, ssum, nks);
    std::swap(s.dd, s.dd2);
    s.dd.n = oo[1];
    s.dd.n_kv = *new_nkv;
    s.RemoteDiff.clear();                             // main.go:75
    s.pend = false;
    s.pend_dev = false;
    s.pend_len = 0;
    s.host_valid = false;
    return CRDT_OK;
}

// ---- batched device merge of several servers (crdt_servers_merge)
struct SegPtrs {                       // one server's device Diff, for the concat / split kernels
    const int64_t *ts;
    const uint8_t *origin;
    const uint64_t *kv_off;
    const uint32_t *kv_key, *kv_val;
    int64_t *dts;                      // split destinations (the server's next Diff)
    uint8_t *dorigin;
    uint64_t *dkv_off;
    uint32_t *dkv_key, *dkv_val;
    uint64_t e0, n, q0, nq;            // entry / pair range in the batch
    uint32_t slot_base, pad;
};

// L of the batch: every server's Diff behind the previous one; kv ranges
// re-based into the shared arena, key ids into the server's slot range;
// l_kv[nl] = the arena's L pair count.
__global__ void k_srv_concat(const SegPtrs *__restrict__ sp, int64_t *__restrict__ l_ts, uint8_t *__restrict__ l_org,
                             uint64_t *__restrict__ l_kv, uint32_t *__restrict__ kv_key, uint32_t *__restrict__ kv_val,
                             uint64_t nl, uint64_t nkl) {
    const SegPtrs p = sp[blockIdx.y];
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) l_kv[nl] = nkl;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < p.n; i += (uint64_t)gridDim.x * 256) {
        l_ts[p.e0 + i] = p.ts[i];
        l_org[p.e0 + i] = p.origin[i];
        l_kv[p.e0 + i] = p.q0 + p.kv_off[i];
    }
    for (uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x; q < p.nq; q += (uint64_t)gridDim.x * 256) {
        kv_key[p.q0 + q] = p.kv_key[q] + p.slot_base;
        kv_val[p.q0 + q] = p.kv_val[q];
    }
}

// The batch's new Diffs back into each server's next buffers.  Server y's
// entry range is o_off[y, y+1) of the batch's new Diff and its pair range
// [o_kv[o_off[y]], o_kv[o_off[y+1]]): both read on the device (the
// destinations are sized for the upper bound), so the split needs no host
// round trip; the pair ranges also go to kb[] for the host.
__global__ void k_srv_split(const SegPtrs *__restrict__ sp, const int64_t *__restrict__ o_ts,
                            const uint8_t *__restrict__ o_org, const uint64_t *__restrict__ o_kv,
                            const uint32_t *__restrict__ kv_key, const uint32_t *__restrict__ kv_val,
                            const uint64_t *__restrict__ o_off, uint64_t *__restrict__ kb,
                            const uint32_t *__restrict__ status, uint32_t *__restrict__ status_out) {
    SegPtrs p = sp[blockIdx.y];
    p.e0 = o_off[blockIdx.y];
    p.n = o_off[blockIdx.y + 1] - p.e0;
    p.q0 = o_kv[p.e0];
    p.nq = o_kv[p.e0 + p.n] - p.q0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        kb[blockIdx.y] = p.q0;
        if (blockIdx.y + 1 == gridDim.y) kb[blockIdx.y + 1] = p.q0 + p.nq;
        if (blockIdx.y == 0)                         // the merge's status words, read back with the results
            for (int w = 0; w < 3; ++w) status_out[w] = status[w];
    }
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i <= p.n; i += (uint64_t)gridDim.x * 256) {
        p.dkv_off[i] = o_kv[p.e0 + i] - p.q0;
        if (i < p.n) {
            p.dts[i] = o_ts[p.e0 + i];
            p.dorigin[i] = o_org[p.e0 + i];
        }
    }
    for (uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x; q < p.nq; q += (uint64_t)gridDim.x * 256) {
        p.dkv_key[q] = kv_key[p.q0 + q] - p.slot_base;
        p.dkv_val[q] = kv_val[p.q0 + q];
    }
}

struct BatchBufs {                     // per-context scratch of the batched server merge
    DBuf head, res, body, dec, l_ts, l_org, l_kv, kv_key, kv_val, r_off, r_ts, r_kv, o_ts, o_org, o_src, n_kv, n_key,
        n_val;
    void *hp = nullptr;                // pinned image of head (upload) and res + status (read-back)
    size_t hp_cap = 0;
};

// merge() of several device-resident servers in ONE decode, ONE RefMerge and
// ONE split.  Key slots: server s owns [s*kcap, (s+1)*kcap); a pull that
// brings more new keys than the slack is reported (*retry) and the caller
// merges one server at a time instead.  Host traffic per call: one pinned
// upload of the descriptors (head), the pulls not already uploaded at ingest,
// one pinned read-back of the results (res) -- plus the decode's own.
// CRDT_SRV_PROF=1: per-phase host wall time of each batched merge on stderr
// (a development aid; every phase ends where the host next waits anyway).
struct PhaseClock {
    bool on;
    std::chrono::steady_clock::time_point t;
    const char *tag;
    char buf[512];
    int n = 0;
    explicit PhaseClock(const char *tg = "srv_merge")
        : on(getenv("CRDT_SRV_PROF") != nullptr), t(std::chrono::steady_clock::now()), tag(tg) {
        buf[0] = 0;
    }
    void mark(const char *name) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        const double us = std::chrono::duration<double, std::micro>(now - t).count();
        t = now;
        if (n < (int)sizeof(buf) - 64) n += snprintf(buf + n, sizeof(buf) - n, " %s=%.1f", name, us);
    }
    ~PhaseClock() {
        if (on) fprintf(stderr, "[%s]%s\n", tag, buf);
    }
};

static int dev_merge_batch(crdt_ctx *ctx, Server *const *srv, size_t S, bool *retry) {
    *retry = false;
    PhaseClock pc;
    if (!ctx->srv_batch) ctx->srv_batch = new (std::nothrow) BatchBufs();
    if (!ctx->srv_batch) return CRDT_E_NOMEM;
    BatchBufs &bb = *(BatchBufs *)ctx->srv_batch;      // the context's scratch (a context is single-threaded)
    int rc;
    for (size_t i = 0; i < S; ++i) {
        Server &s = *srv[i];
        if (!s.dev_valid) rc = dev_upload(ctx, s);
        else rc = CRDT_OK;
        if (!rc) rc = dev_flush_cmds(ctx, s);
        if (rc) return rc;
    }
    uint64_t nks0 = 0, b0 = 0;
    (void)crdt_strtab_info(ctx->keys, &nks0, &b0, nullptr, nullptr);
    uint64_t kcap = 64;
    while (kcap < nks0 + 256) kcap <<= 1;
    if (kcap * S >= 0xFFFFFFFFull) return CRDT_E_RANGE;
    // the pulls: parked ones were uploaded at ingest (s.pull); the rest (a
    // RemoteDiff built on the host, a parked pull whose upload was not
    // started) are staged in pinned memory and uploaded into bb.body here
    std::vector<std::string> enc(S);
    std::vector<uint64_t> blen(S), bat(S, 0), e0(S + 1, 0), q0(S + 1, 0), re(S + 1, 0), rq(S + 1, 0), pin_at(S, 0);
    std::vector<uint32_t> sbase(S);
    std::vector<uint8_t> hdr(32 * S);
    // bodies encoded here are staged in pinned memory at their offsets in
    // bb.body, so one copy uploads all of them (a copy per body waited
    // ~24 us each on the copy engine)
    uint64_t stage = 0;
    bool any_enc = false;
    for (size_t i = 0; i < S; ++i) {
        Server &s = *srv[i];
        if (!s.pend) {
            encode_soa(s.RemoteDiff, enc[i]);
            any_enc = true;
        }
        const char *b = s.pend ? s.pend_body : enc[i].data();
        memcpy(&hdr[32 * i], b, 32);                    // (every body here is >= 32 bytes)
        blen[i] = s.pend ? s.pend_len : enc[i].size();
        if (!(s.pend && s.pend_dev)) {
            bat[i] = stage;
            if (!s.pend) pin_at[i] = stage;
            stage += (blen[i] + 15) & ~(uint64_t)15;
        }
        uint64_t ne, np;
        memcpy(&ne, b + 8, 8);
        memcpy(&np, b + 16, 8);
        re[i + 1] = re[i] + ne;
        rq[i + 1] = rq[i] + np;
        e0[i + 1] = e0[i] + s.dd.n;
        q0[i + 1] = q0[i] + s.dd.n_kv;
        sbase[i] = (uint32_t)(i * kcap);
    }
    rc = pinned_reserve(ctx, any_enc ? stage : 0);    // bodies encoded here; parked pulls are pinned already
    if (rc) return rc;
    for (size_t i = 0; i < S; ++i)
        if (!srv[i]->pend) memcpy((char *)ctx->pinned + pin_at[i], enc[i].data(), enc[i].size());
    pc.mark("upload+encode");
    const uint64_t nl = e0[S], nkl = q0[S], nr = re[S], nkr = rq[S], nslots = kcap * S;
    // head (device, one upload): sp | sq | l_off;  res (device, one read-back):
    // o_off | kb | st_sum | st_str | st_kind
    const size_t h_sq = Carve::round(S * sizeof(SegPtrs)), h_loff = h_sq + Carve::round(S * sizeof(SegPtrs));
    const size_t h_bytes = h_loff + Carve::round((S + 1) * 8);
    const size_t r_kb = Carve::round((S + 1) * 8), r_sum = r_kb + Carve::round((S + 1) * 8);
    const size_t r_str = r_sum + Carve::round(nslots * 8 + 8), r_kind = r_str + Carve::round(nslots * 4 + 4);
    const size_t r_st = r_kind + Carve::round(nslots + 1), r_bytes = r_st + 16;
    rc = dbuf(ctx, bb.head, h_bytes);
    if (!rc) rc = dbuf(ctx, bb.res, r_bytes);
    if (!rc) rc = dbuf(ctx, bb.dec, gossip_decode_scratch_bytes((uint32_t)S, nr, nkr));
    if (!rc) rc = dbuf(ctx, bb.body, stage + 16);
    if (!rc) rc = dbuf(ctx, bb.l_ts, nl * 8 + 8);
    if (!rc) rc = dbuf(ctx, bb.l_org, nl + 1);
    if (!rc) rc = dbuf(ctx, bb.l_kv, (nl + 1) * 8);
    if (!rc) rc = dbuf(ctx, bb.kv_key, (nkl + nkr) * 4 + 4);
    if (!rc) rc = dbuf(ctx, bb.kv_val, (nkl + nkr) * 4 + 4);
    if (!rc) rc = dbuf(ctx, bb.r_off, (S + 1) * 8);
    if (!rc) rc = dbuf(ctx, bb.r_ts, nr * 8 + 8);
    if (!rc) rc = dbuf(ctx, bb.r_kv, (nr + 1) * 8);
    if (!rc) rc = dbuf(ctx, bb.o_ts, (nl + nr) * 8 + 8);
    if (!rc) rc = dbuf(ctx, bb.o_org, nl + nr + 1);
    if (!rc) rc = dbuf(ctx, bb.o_src, (nl + nr) * 8 + 8);
    if (!rc) rc = dbuf(ctx, bb.n_kv, (nl + nr + 1) * 8);
    if (!rc) rc = dbuf(ctx, bb.n_key, (nkl + nkr) * 4 + 4);
    if (!rc) rc = dbuf(ctx, bb.n_val, (nkl + nkr) * 4 + 4);
    // each server's next Diff buffers at their upper bound (its L + its pull),
    // so the split runs behind the merge with no host round trip for the
    // output sizes: one synchronisation per call after the decode's
    uint64_t maxs = 1, maxn = 1;
    for (size_t i = 0; i < S && !rc; ++i) {
        Server &s = *srv[i];
        const uint64_t nu = s.dd.n + (re[i + 1] - re[i]), qu = s.dd.n_kv + (rq[i + 1] - rq[i]);
        rc = dbuf(ctx, s.dd2.ts, nu * 8 + 8);
        if (!rc) rc = dbuf(ctx, s.dd2.origin, nu + 1);
        if (!rc) rc = dbuf(ctx, s.dd2.kv_off, (nu + 1) * 8);
        if (!rc) rc = dbuf(ctx, s.dd2.kv_key, qu * 4 + 4);
        if (!rc) rc = dbuf(ctx, s.dd2.kv_val, qu * 4 + 4);
        maxs = std::max<uint64_t>(maxs, std::max(nu + 1, qu));
        maxn = std::max<uint64_t>(maxn, std::max(s.dd.n, s.dd.n_kv));
    }
    if (!rc && bb.hp_cap < h_bytes + r_bytes + 64) {
        const hipError_t e = hipStreamSynchronize(ctx->stream);   // (the previous image may still be in flight)
        if (e != hipSuccess) return hip_fail(ctx, e);
        if (bb.hp) (void)hipHostFree(bb.hp);
        bb.hp = nullptr;
        bb.hp_cap = 0;
        const size_t want = (h_bytes + r_bytes + 64) * 3 / 2;
        if (hipHostMalloc(&bb.hp, want, 0) != hipSuccess) {
            bb.hp = nullptr;
            return CRDT_E_NOMEM;
        }
        bb.hp_cap = want;
    }
    if (rc) return rc;
    char *hp = (char *)bb.hp, *hres = hp + h_bytes;
    uint32_t *hfl = (uint32_t *)(hres + r_st);
    SegPtrs *sp = (SegPtrs *)hp, *sq = (SegPtrs *)(hp + h_sq);
    for (size_t i = 0; i < S; ++i) {
        Server &s = *srv[i];
        sp[i] = SegPtrs{s.dd.ts.as<int64_t>(), s.dd.origin.as<uint8_t>(), s.dd.kv_off.as<uint64_t>(),
                        s.dd.kv_key.as<uint32_t>(), s.dd.kv_val.as<uint32_t>(), nullptr, nullptr, nullptr, nullptr,
                        nullptr, e0[i], s.dd.n, q0[i], s.dd.n_kv, sbase[i], 0};
        sq[i] = SegPtrs{nullptr, nullptr, nullptr, nullptr, nullptr, s.dd2.ts.as<int64_t>(),
                        s.dd2.origin.as<uint8_t>(), s.dd2.kv_off.as<uint64_t>(), s.dd2.kv_key.as<uint32_t>(),
                        s.dd2.kv_val.as<uint32_t>(), 0, 0, 0, 0, sbase[i], 0};
    }
    memcpy(hp + h_loff, e0.data(), (S + 1) * 8);
    const hipStream_t st = ctx->stream;
    char *dh = bb.head.as<char>(), *dr = bb.res.as<char>();
    hipError_t e = hipMemcpyAsync(dh, hp, h_bytes, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return hip_fail(ctx, e);
    // L: concat
    const dim3 grid(grid_for(maxn, 256, (unsigned)ctx->num_cus * 2), (unsigned)S);
    k_srv_concat<<<grid, 256, 0, st>>>((const SegPtrs *)dh, bb.l_ts.as<int64_t>(), bb.l_org.as<uint8_t>(),
                                        bb.l_kv.as<uint64_t>(), bb.kv_key.as<uint32_t>(), bb.kv_val.as<uint32_t>(), nl,
                                        nkl);
    rc = check_launch(ctx);
    if (rc) return rc;
    // R: every pull decoded at once, pairs behind L's in the arena; bodies
    // addressed relative to bb.body (the ones uploaded at ingest live in
    // their servers' pull buffers)
    const uint8_t *base = bb.body.as<uint8_t>();
    std::vector<uint64_t> at(S);
    if (any_enc) e = hipMemcpyAsync(bb.body.as<char>(), ctx->pinned, stage, hipMemcpyHostToDevice, st);
    for (size_t i = 0; i < S && e == hipSuccess; ++i) {
        const Server &s = *srv[i];
        if (s.pend && s.pend_dev) {
            at[i] = (uint64_t)(uintptr_t)s.pull.p - (uint64_t)(uintptr_t)base;
        } else {
            at[i] = bat[i];
            if (s.pend)                                // (after the bulk copy: its slot there held no body)
                e = hipMemcpyAsync(bb.body.as<char>() + bat[i], s.pend_body, blen[i], hipMemcpyHostToDevice, st);
        }
    }
    if (e != hipSuccess) return hip_fail(ctx, e);
    std::vector<uint32_t> bst(S, 0);
    crdt_gossip_decoded go{bb.r_off.as<uint64_t>(), bb.r_ts.as<int64_t>(), bb.r_kv.as<uint64_t>(),
                           bb.kv_key.as<uint32_t>(), bb.kv_val.as<uint32_t>()};
    pc.mark("alloc+concat");
    crdt_refmerge_in ri;
    ri.replicas = (uint32_t)S;
    ri.n_slots = (uint32_t)nslots;
    ri.n_l = nl;
    ri.n_r = nr;
    ri.n_kv = nkl + nkr;
    ri.l_off = (const uint64_t *)(dh + h_loff);
    ri.l_ts = bb.l_ts.as<int64_t>();
    ri.l_origin = bb.l_org.as<uint8_t>();
    ri.l_kv = bb.l_kv.as<uint64_t>();
    ri.r_off = bb.r_off.as<uint64_t>();
    ri.r_ts = bb.r_ts.as<int64_t>();
    ri.r_kv = bb.r_kv.as<uint64_t>();
    ri.kv_key = bb.kv_key.as<uint32_t>();
    ri.kv_val = bb.kv_val.as<uint32_t>();
    crdt_refmerge_out ro{(uint64_t *)dr, bb.o_ts.as<int64_t>(), bb.o_org.as<uint8_t>(), bb.o_src.as<int64_t>(),
                         (uint8_t *)(dr + r_kind), (uint32_t *)(dr + r_str), (int64_t *)(dr + r_sum)};
    const crdt_refmerge_kv_out kvo{bb.n_kv.as<uint64_t>(), bb.n_key.as<uint32_t>(), bb.n_val.as<uint32_t>(),
                                   nkl + nkr};
    StatusScope sc(ctx);
    // the merge with the new Diffs' kv pairs (copied by its tile pass; the
    // entry count stays on the device), the split into each server's next
    // buffers, then everything the host needs in one read-back.  Enqueued by
    // the decode right behind its claim pass (the strings of a pull are
    // nearly always interned already); when the pulls brought new strings the
    // decode finishes their ids first and this runs again.
    const std::function<int()> run_merge = [&]() -> int {
        uint64_t nstr = 0, nb0 = 0;
        const uint8_t *sb = nullptr;
        const uint64_t *so = nullptr;
        (void)crdt_strtab_info(ctx->vals, &nstr, &nb0, &sb, &so);
        ri.n_str = nstr;
        ri.str_bytes = sb;
        ri.str_off = so;
        int r = crdt_refmerge_batch_kv(ctx, &ri, &ro, &kvo);
        if (r) return r;
        const dim3 g2(grid_for(maxs, 256, (unsigned)ctx->num_cus * 2), (unsigned)S);
        k_srv_split<<<g2, 256, 0, st>>>((const SegPtrs *)(dh + h_sq), bb.o_ts.as<int64_t>(), bb.o_org.as<uint8_t>(),
                                         bb.n_kv.as<uint64_t>(), bb.n_key.as<uint32_t>(), bb.n_val.as<uint32_t>(),
                                         (const uint64_t *)dr, (uint64_t *)(dr + r_kb), sc.saved,
                                         (uint32_t *)(dr + r_st));
        r = check_launch(ctx);
        if (r) return r;
        const hipError_t x = hipMemcpyAsync(hres, dr, r_bytes, hipMemcpyDeviceToHost, st);   // results + status words
        return x == hipSuccess ? CRDT_OK : hip_fail(ctx, x);
    };
    bool stale = false;
    rc = gossip_decode_at(ctx, (uint32_t)S, base, at.data(), blen.data(), (uint32_t)kcap, nkl, sbase.data(),
                          hdr.data(), ctx->keys, ctx->vals, &go, bst.data(), &run_merge, bb.dec.p, bb.dec.cap, &stale);
    if (rc) return rc;
    pc.mark("decode+merge");
    for (auto x : bst)
        if (x) {                                       // a key past the slot slack (or a malformed pull)
            *retry = true;
            return CRDT_OK;
        }
    if (stale) {                                       // new strings: the merge again, on their ids
        rc = run_merge();
        if (rc) return rc;
        e = hipStreamSynchronize(st);
        if (e != hipSuccess) return hip_fail(ctx, e);
    }
    if (sc.raised(hfl)) return CRDT_E_DEVICE;              // no server swapped in anything
    pc.mark("split+read_back");
    const uint64_t *oo = (const uint64_t *)hres, *kb = (const uint64_t *)(hres + r_kb);
    const uint8_t *kind = (const uint8_t *)(hres + r_kind);
    const uint32_t *sstr = (const uint32_t *)(hres + r_str);
    const int64_t *ssum = (const int64_t *)(hres + r_sum);
    uint64_t nks = 0;
    (void)crdt_strtab_info(ctx->keys, &nks, &b0, nullptr, nullptr);
    const uint64_t nk = std::min(nks, kcap);
    for (size_t i = 0; i < S; ++i) {
        Server &s = *srv[i];
        apply_state(ctx, s, kind + i * kcap, sstr + i * kcap, ssum + i * kcap, nk);
        std::swap(s.dd, s.dd2);
        s.dd.n = oo[i + 1] - oo[i];
        s.dd.n_kv = kb[i + 1] - kb[i];
        s.RemoteDiff.clear();                          // main.go:75
        s.pend = false;
        s.pend_dev = false;
        s.pend_len = 0;
        s.host_valid = false;
    }
    pc.mark("state");
    return CRDT_OK;
}

// Frees the context's batch scratch (crdt_ctx_destroy).
void server_ctx_release(crdt_ctx *ctx) {
    if (!ctx->srv_batch) return;
    BatchBufs *bb = (BatchBufs *)ctx->srv_batch;
    for (DBuf *b : {&bb->head, &bb->res, &bb->body, &bb->dec, &bb->l_ts, &bb->l_org, &bb->l_kv, &bb->kv_key, &bb->kv_val,
                    &bb->r_off, &bb->r_ts, &bb->r_kv, &bb->o_ts, &bb->o_org, &bb->o_src, &bb->n_kv, &bb->n_key,
                    &bb->n_val})
        dbuf_free(*b);
    if (bb->hp) (void)hipHostFree(bb->hp);
    delete bb;
    ctx->srv_batch = nullptr;
}

// Can this merge run on the device?  Not with a nil map (JSON null) in the
// Diff or the pull: the device layout has no nil flag.
static bool dev_ok(const Server &s) {
    if (!s.ctx) return false;
    if (!s.dev_valid && has_nil(s.Diff)) return false;
    if (!s.pend && has_nil(s.RemoteDiff)) return false;
    return true;
}

static void dev_free(Server &s) {
    if (s.ctx) {
        (void)bind(s.ctx);
        (void)hipStreamSynchronize(s.ctx->stream);
    }
    for (DBuf *b : {&s.dd.ts, &s.dd.origin, &s.dd.kv_off, &s.dd.kv_key, &s.dd.kv_val, &s.dd2.ts, &s.dd2.origin,
                    &s.dd2.kv_off, &s.dd2.kv_key, &s.dd2.kv_val, &s.body, &s.r_ts, &s.r_kv, &s.r_off, &s.l_off,
                    &s.o_off, &s.o_src, &s.st_kind, &s.st_str, &s.st_sum, &s.c_ts, &s.c_kv, &s.c_key, &s.c_val,
                    &s.c_off, &s.c_status, &s.pull})
        dbuf_free(*b);
    if (s.pend_body) (void)hipHostFree(s.pend_body);
    s.pend_body = nullptr;
    s.pend_cap = s.pend_len = 0;
}

}  // namespace crdt

using namespace crdt;

struct crdt_server { Server s; };

extern "C" int crdt_server_new(crdt_ctx *ctx, int port, crdt_server **out) {
    if (!out) return CRDT_E_INVAL;            // ctx NULL: a host-only server (codec, AddCommand; no merge)
    crdt_server *p = new (std::nothrow) crdt_server();
    if (!p) return CRDT_E_NOMEM;
    p->s.ctx = ctx;
    p->s.Port = port;
    *out = p;
    return CRDT_OK;
}

extern "C" int crdt_server_free(crdt_server *srv) {
    if (srv) dev_free(srv->s);
    delete srv;
    return CRDT_OK;
}

static bool kv_args_ok(const char *const *keys, const size_t *klen, const char *const *vals, const size_t *vlen,
                       size_t n) {
    if (n == 0) return true;
    if (!keys || !klen || !vals || !vlen) return false;
    for (size_t i = 0; i < n; ++i)
        if ((!keys[i] && klen[i]) || (!vals[i] && vlen[i])) return false;
    return true;
}

extern "C" int crdt_server_diff_put(crdt_server *srv, int64_t ts, int local, const char *const *keys,
                                    const size_t *klen, const char *const *vals, const size_t *vlen, size_t n) {
    if (!srv || !kv_args_ok(keys, klen, vals, vlen, n)) return CRDT_E_INVAL;
    std::lock_guard<std::mutex> g(srv->s.Lock);
    int rc = make_host(srv->s);
    if (rc) return rc;
    srv->s.Diff[ts] = make_value(local != 0, keys, klen, vals, vlen, n);   // treemap Put replaces
    srv->s.dev_valid = false;                                    // re-uploaded at the next merge
    srv->s.pend_cmds.clear();
    return CRDT_OK;
}

extern "C" int crdt_server_remote_put(crdt_server *srv, int64_t ts, const char *const *keys, const size_t *klen,
                                      const char *const *vals, const size_t *vlen, size_t n) {
    if (!srv || !kv_args_ok(keys, klen, vals, vlen, n)) return CRDT_E_INVAL;
    // main.go:255 writes RemoteDiff from the gossip goroutine without the lock;
    // here the lock is taken so concurrent callers stay safe.
    std::lock_guard<std::mutex> g(srv->s.Lock);
    absorb_pending(srv->s);
    srv->s.RemoteDiff[ts] = make_value(false, keys, klen, vals, vlen, n);
    return CRDT_OK;
}

extern "C" int crdt_servers_merge(crdt_server *const *srvs, size_t n) {
    if (n == 0) return CRDT_OK;
    if (!srvs) return CRDT_E_INVAL;
    std::vector<Server *> v;
    v.reserve(n);
    for (size_t i = 0; i < n; ++i) {
        if (!srvs[i]) return CRDT_E_INVAL;
        v.push_back(&srvs[i]->s);
    }
    std::vector<Server *> order(v);
    std::sort(order.begin(), order.end());
    if (std::adjacent_find(order.begin(), order.end()) != order.end()) return CRDT_E_INVAL;   // duplicates
    crdt_ctx *ctx = v[0]->ctx;
    for (auto *s : v)
        if (!s->ctx || s->ctx->device != ctx->device) return CRDT_E_INVAL;   // host-only servers cannot merge
    int rc = bind(ctx);
    if (rc) return rc;
    for (auto *s : v) s->Alive = false;                         // main.go:41
    for (auto *s : order) s->Lock.lock();                       // main.go:43 (address order: no deadlock)
    // Device-resident path: every server's Diff stays in HBM, its pull is
    // decoded on the device; the host path (pack, H2D, merge, D2H, rebuild)
    // takes batches holding a nil map (no device representation).
    bool dev = !fail_refmerge_armed();                     // (fault injection exercises the host path)
    for (auto *s : v) dev = dev && dev_ok(*s) && s->ctx == ctx;
    if (dev) rc = ctx_tables(ctx);
    if (dev && !rc) {
        bool retry = true;                                      // (one server: the exact-slot path)
        if (v.size() > 1) rc = dev_merge_batch(ctx, v.data(), v.size(), &retry);
        if (!rc && retry)                                       // one at a time (exact key slots)
            for (auto *s : v) {
                rc = dev_merge_one(ctx, *s);
                if (rc) break;
            }
    } else if (!rc) {
        for (auto *s : v) {
            absorb_pending(*s);
            if (!rc) rc = make_host(*s);
        }
        if (!rc) rc = merge_locked(ctx, v.data(), v.size());
        if (!rc)
            for (auto *s : v) {                                   // the host map is now the Diff
                s->dev_valid = false;
                s->pend_cmds.clear();
            }
    }
    for (auto *s : v) s->Alive = true;
    for (auto it = order.rbegin(); it != order.rend(); ++it) (*it)->Lock.unlock();
    return rc;
}

extern "C" int crdt_server_merge(crdt_server *srv) {
    if (!srv) return CRDT_E_INVAL;
    return crdt_servers_merge(&srv, 1);
}

// NewServer's initialState (main.go:102-105): CurrentState starts as it.
extern "C" int crdt_server_init_state(crdt_server *srv, const char *const *keys, const size_t *klen,
                                      const char *const *vals, const size_t *vlen, size_t n) {
    if (!srv || !kv_args_ok(keys, klen, vals, vlen, n)) return CRDT_E_INVAL;
    std::lock_guard<std::mutex> g(srv->s.Lock);
    srv->s.InitialState.clear();
    for (size_t i = 0; i < n; ++i) srv->s.InitialState[std::string(keys[i], klen[i])] = std::string(vals[i], vlen[i]);
    srv->s.CurrentState = srv->s.InitialState;
    srv->s.state_synced = false;
    srv->s.state_view.clear();
    return CRDT_OK;
}

// AddCommand (main.go:173-215) after the JSON decode: Diff.Put(ts, &data)
// (main.go:187), then the local apply (main.go:188-207) in key order (Go's
// map order is random; key order is one of its legal executions): a key not
// yet in CurrentState is set verbatim and the handler RETURNS (main.go:189-193);
// otherwise Atoi both sides (500 on error, main.go:195-204) and store
// Itoa(sum) (main.go:205-206).  *http_status = 200 / 500 / 502 (dead replica).
extern "C" int crdt_server_add_command(crdt_server *srv, int64_t ts_ms, const char *const *keys, const size_t *klen,
                                       const char *const *vals, const size_t *vlen, size_t n, int *http_status) {
    if (!srv || !http_status || !kv_args_ok(keys, klen, vals, vlen, n)) return CRDT_E_INVAL;
    Server &s = srv->s;
    std::lock_guard<std::mutex> g(s.Lock);
    if (!s.Alive) { *http_status = 502; return CRDT_OK; }
    auto v = make_value(true, keys, klen, vals, vlen, n);
    if (s.host_valid) s.Diff[ts_ms] = v;                   // same-ms writes overwrite
    if (s.dev_valid) s.pend_cmds.emplace_back(ts_ms, v);   // applied to the device Diff at the next merge
    s.state_view.clear();
    s.state_synced = false;                                 // CurrentState now differs from the device's words
    *http_status = 200;
    for (auto &kv : v->kv) {
        auto it = s.CurrentState.find(kv.first);
        if (it == s.CurrentState.end()) {
            s.CurrentState.emplace(kv.first, kv.second);
            return CRDT_OK;                                 // "Inserted", early return (main.go:192-193)
        }
        long long curr, change;
        auto atoi = [](const std::string &x, long long *out) {
            if (x.empty()) return false;
            size_t i = 0;
            bool neg = false;
            if (x[0] == '+' || x[0] == '-') { neg = x[0] == '-'; i = 1; if (x.size() == 1) return false; }
            unsigned long long acc = 0;
            for (; i < x.size(); ++i) {
                unsigned d = (unsigned char)x[i] - (unsigned)'0';
                if (d > 9 || acc > (0xFFFFFFFFFFFFFFFFULL - d) / 10) return false;
                acc = acc * 10 + d;
            }
            if ((!neg && acc >= 0x8000000000000000ULL) || (neg && acc > 0x8000000000000000ULL)) return false;
            *out = neg ? (long long)(0 - acc) : (long long)acc;
            return true;
        };
        if (!atoi(it->second, &curr) || !atoi(kv.second, &change)) { *http_status = 500; return CRDT_OK; }
        it->second = std::to_string((long long)((unsigned long long)curr + (unsigned long long)change));
    }
    return CRDT_OK;
}

extern "C" int crdt_server_diff_len(crdt_server *srv, size_t *n) {
    if (!srv || !n) return CRDT_E_INVAL;
    std::lock_guard<std::mutex> g(srv->s.Lock);
    if (!srv->s.host_valid && srv->s.pend_cmds.empty()) {       // no need to rebuild the host view
        *n = srv->s.dd.n;
        return CRDT_OK;
    }
    int rc = make_host(srv->s);
    if (rc) return rc;
    *n = srv->s.Diff.size();
    return CRDT_OK;
}

extern "C" int crdt_server_remote_len(crdt_server *srv, size_t *n) {
    if (!srv || !n) return CRDT_E_INVAL;
    std::lock_guard<std::mutex> g(srv->s.Lock);
    absorb_pending(srv->s);
    *n = srv->s.RemoteDiff.size();
    return CRDT_OK;
}

// Ascending Diff keys (Diff.Keys(), main.go:45) with their origin; either
// output may be NULL.  Writes min(cap, len) entries.
extern "C" int crdt_server_diff_keys(crdt_server *srv, int64_t *ts, uint8_t *local, size_t cap, size_t *n) {
    if (!srv || !n) return CRDT_E_INVAL;
    std::lock_guard<std::mutex> g(srv->s.Lock);
    int rc = make_host(srv->s);
    if (rc) return rc;
    size_t i = 0;
    for (auto &e : srv->s.Diff) {
        if (i >= cap) break;
        if (ts) ts[i] = e.first;
        if (local) local[i] = e.second->local ? 1 : 0;
        ++i;
    }
    *n = srv->s.Diff.size();
    return CRDT_OK;
}

extern "C" int crdt_server_state_len(crdt_server *srv, size_t *n) {
    if (!srv || !n) return CRDT_E_INVAL;
    std::lock_guard<std::mutex> g(srv->s.Lock);
    *n = srv->s.CurrentState.size();
    return CRDT_OK;
}

// i-th CurrentState entry in key order.  The returned pointers stay valid
// until the next mutation of this server.
extern "C" int crdt_server_state_at(crdt_server *srv, size_t i, const char **key, size_t *klen, const char **val,
                                    size_t *vlen) {
    if (!srv || !key || !klen || !val || !vlen) return CRDT_E_INVAL;
    std::lock_guard<std::mutex> g(srv->s.Lock);
    Server &s = srv->s;
    if (s.state_view.size() != s.CurrentState.size()) s.state_view.assign(s.CurrentState.begin(), s.CurrentState.end());
    if (i >= s.state_view.size()) return CRDT_E_INVAL;
    *key = s.state_view[i].first.data();
    *klen = s.state_view[i].first.size();
    *val = s.state_view[i].second.data();
    *vlen = s.state_view[i].second.size();
    return CRDT_OK;
}

// ---------------------------------------------------------------- gossip wire codec
// The reference's gossip wire format:
//   serve : Gossip handler (main.go:153-170): 502 "Unreachable" unless Alive,
//           else 200 + server.Diff.ToJSON() (main.go:159).  gods v1.18.1
//           treemap ToJSON = json.Marshal(map[string]interface{}) keyed by
//           strconv.FormatInt(ts): encoding/json writes map keys sorted as
//           BYTE STRINGS ("-5" < "10" < "2"), values (map[string]string or
//           *Command) as objects with sorted keys, no whitespace.
//   pull  : main.go:245-256: json.Unmarshal into map[string]map[string]string
//           (any error: the round is skipped, main.go:247-249), then for each
//           key Atoi(key) -> RemoteDiff.Put(int64(atoi), value); a key that
//           fails Atoi RETURNS from the gossip goroutine (main.go:252-253).
// Strings follow Go 1.18 encoding/json: Marshal escapes the quote and the
// backslash with a backslash, newline / CR / tab as \n \r \t, other bytes < 0x20
// and the HTML-unsafe '<' '>' '&' as \u00XX (lowercase hex), U+2028 / U+2029
// as \u2028 / \u2029, and each byte of invalid UTF-8 as \ufffd; Unmarshal
// accepts any valid JSON and replaces invalid UTF-8 / unpaired surrogates
// with U+FFFD.

static void json_put_string(std::string &o, const std::string &s) {
    static const char *hex = "0123456789abcdef";
    o.push_back('"');
    size_t i = 0;
    const size_t n = s.size();
    while (i < n) {
        const unsigned char b = (unsigned char)s[i];
        if (b < 0x80) {
            if (b >= 0x20 && b != '"' && b != '\\' && b != '<' && b != '>' && b != '&') {
                o.push_back((char)b);
            } else if (b == '"' || b == '\\') {
                o.push_back('\\');
                o.push_back((char)b);
            } else if (b == '\n') {
                o += "\\n";
            } else if (b == '\r') {
                o += "\\r";
            } else if (b == '\t') {
                o += "\\t";
            } else {
                o += "\\u00";
                o.push_back(hex[b >> 4]);
                o.push_back(hex[b & 15]);
            }
            ++i;
            continue;
        }
        // decode one UTF-8 sequence the way utf8.DecodeRuneInString does
        uint32_t cp = 0;
        size_t len = 0;
        if (b >= 0xC2 && b <= 0xDF) { len = 2; cp = b & 0x1F; }
        else if (b >= 0xE0 && b <= 0xEF) { len = 3; cp = b & 0x0F; }
        else if (b >= 0xF0 && b <= 0xF4) { len = 4; cp = b & 0x07; }
        bool ok = len != 0 && i + len <= n;
        for (size_t k = 1; ok && k < len; ++k) {
            const unsigned char c = (unsigned char)s[i + k];
            if ((c & 0xC0) != 0x80) ok = false;
            cp = (cp << 6) | (c & 0x3F);
        }
        if (ok) {   // reject overlongs, surrogates, > U+10FFFF (second-byte ranges of utf8.DecodeRune)
            const unsigned char c1 = (unsigned char)s[i + 1];
            if (b == 0xE0 && c1 < 0xA0) ok = false;
            if (b == 0xED && c1 > 0x9F) ok = false;
            if (b == 0xF0 && c1 < 0x90) ok = false;
            if (b == 0xF4 && c1 > 0x8F) ok = false;
        }
        if (!ok) {
            o += "\\ufffd";
            ++i;
            continue;
        }
        if (cp == 0x2028 || cp == 0x2029) {
            o += cp == 0x2028 ? "\\u2028" : "\\u2029";
        } else {
            o.append(s, i, len);
        }
        i += len;
    }
    o.push_back('"');
}

static void json_put_value(std::string &o, const Value &v) {
    if (v.nil) {                     // json.Marshal of a nil map[string]string (main.go:159)
        o += "null";
        return;
    }
    std::vector<const std::pair<std::string, std::string> *> kv;
    kv.reserve(v.kv.size());
    for (auto &e : v.kv) kv.push_back(&e);
    std::sort(kv.begin(), kv.end(), [](auto *a, auto *b) { return a->first < b->first; });
    o.push_back('{');
    for (size_t i = 0; i < kv.size(); ++i) {
        if (i) o.push_back(',');
        json_put_string(o, kv[i]->first);
        o.push_back(':');
        json_put_string(o, kv[i]->second);
    }
    o.push_back('}');
}

// *len = bytes of the response body; the body is copied to buf when cap
// allows (else CRDT_E_RANGE with *len = the size needed).
extern "C" int crdt_server_gossip_json(crdt_server *srv, char *buf, size_t cap, size_t *len, int *http_status) {
    if (!srv || !len || !http_status) return CRDT_E_INVAL;
    std::string body;
    {
        std::lock_guard<std::mutex> g(srv->s.Lock);                   // main.go:155-156
        int rc = make_host(srv->s);
        if (rc) return rc;
        if (!srv->s.Alive) {
            *http_status = 502;
            body = "Unreachable";                                    // main.go:166
        } else {
            *http_status = 200;
            std::vector<std::pair<std::string, const Value *>> items;
            items.reserve(srv->s.Diff.size());
            for (auto &e : srv->s.Diff) items.emplace_back(std::to_string((long long)e.first), e.second.get());
            std::sort(items.begin(), items.end(), [](auto &a, auto &b) { return a.first < b.first; });
            body.push_back('{');
            for (size_t i = 0; i < items.size(); ++i) {
                if (i) body.push_back(',');
                json_put_string(body, items[i].first);
                body.push_back(':');
                json_put_value(body, *items[i].second);
            }
            body.push_back('}');
        }
    }
    *len = body.size();
    if (!buf || cap < body.size()) return CRDT_E_RANGE;
    std::copy(body.begin(), body.end(), buf);
    return CRDT_OK;
}

namespace {

// Minimal RFC 8259 parser for exactly the shape main.go:246 decodes into:
// an object of objects of strings (or null).  Anything else is an error,
// which json.Unmarshal reports (a type error included) and main.go skips.
struct JsonIn {
    const char *p, *e;
    bool fail = false;
    void ws() {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
    }
    bool lit(const char *s) {
        const char *q = p;
        for (; *s; ++s, ++q)
            if (q >= e || *q != *s) return false;
        p = q;
        return true;
    }
    static void put_utf8(std::string &o, uint32_t cp) {
        if (cp < 0x80) o.push_back((char)cp);
        else if (cp < 0x800) { o.push_back((char)(0xC0 | (cp >> 6))); o.push_back((char)(0x80 | (cp & 0x3F))); }
        else if (cp < 0x10000) {
            o.push_back((char)(0xE0 | (cp >> 12)));
            o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            o.push_back((char)(0x80 | (cp & 0x3F)));
        } else {
            o.push_back((char)(0xF0 | (cp >> 18)));
            o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
            o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            o.push_back((char)(0x80 | (cp & 0x3F)));
        }
    }
    int hex4() {
        if (e - p < 4) return -1;
        int v = 0;
        for (int k = 0; k < 4; ++k) {
            const char c = p[k];
            int d = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
            if (d < 0) return -1;
            v = v * 16 + d;
        }
        p += 4;
        return v;
    }
    bool str(std::string &o) {
        if (p >= e || *p != '"') return false;
        ++p;
        while (p < e) {
            const unsigned char c = (unsigned char)*p;
            if (c == '"') { ++p; return true; }
            if (c < 0x20) return false;                 // raw control characters are invalid JSON
            if (c == '\\') {
                if (++p >= e) return false;
                const char x = *p++;
                switch (x) {
                    case '"': o.push_back('"'); break;
                    case '\\': o.push_back('\\'); break;
                    case '/': o.push_back('/'); break;
                    case 'b': o.push_back('\b'); break;
                    case 'f': o.push_back('\f'); break;
                    case 'n': o.push_back('\n'); break;
                    case 'r': o.push_back('\r'); break;
                    case 't': o.push_back('\t'); break;
                    case 'u': {
                        int u = hex4();
                        if (u < 0) return false;
                        uint32_t cp = (uint32_t)u;
                        if (cp >= 0xD800 && cp < 0xDC00) {       // high surrogate: pair or U+FFFD
                            if (e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                                const char *save = p;
                                p += 2;
                                const int lo = hex4();
                                if (lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (uint32_t)(lo - 0xDC00);
                                else { p = save; cp = 0xFFFD; }
                            } else {
                                cp = 0xFFFD;
                            }
                        } else if (cp >= 0xDC00 && cp < 0xE000) {
                            cp = 0xFFFD;
                        }
                        put_utf8(o, cp);
                        break;
                    }
                    default: return false;
                }
                continue;
            }
            if (c < 0x80) { o.push_back((char)c); ++p; continue; }
            // raw UTF-8: copy valid sequences, replace each invalid byte with U+FFFD
            size_t len = c >= 0xC2 && c <= 0xDF ? 2 : c >= 0xE0 && c <= 0xEF ? 3 : c >= 0xF0 && c <= 0xF4 ? 4 : 0;
            bool ok = len != 0 && (size_t)(e - p) >= len;
            for (size_t k = 1; ok && k < len; ++k) ok = ((unsigned char)p[k] & 0xC0) == 0x80;
            if (ok) {
                const unsigned char c1 = (unsigned char)p[1];
                if ((c == 0xE0 && c1 < 0xA0) || (c == 0xED && c1 > 0x9F) || (c == 0xF0 && c1 < 0x90) ||
                    (c == 0xF4 && c1 > 0x8F))
                    ok = false;
            }
            if (ok) { o.append(p, len); p += len; }
            else { put_utf8(o, 0xFFFD); ++p; }
        }
        return false;
    }
    // object of strings (or null) -> kv (duplicate keys: the last wins)
    bool inner(std::vector<std::pair<std::string, std::string>> &kv, bool *is_null) {
        ws();
        *is_null = false;
        if (lit("null")) { *is_null = true; return true; }
        if (p >= e || *p != '{') return false;
        ++p;
        ws();
        std::map<std::string, std::string> m;
        if (p < e && *p == '}') { ++p; return true; }
        for (;;) {
            std::string k, v;
            ws();
            if (!str(k)) return false;
            ws();
            if (p >= e || *p != ':') return false;
            ++p;
            ws();
            if (lit("null")) {
                // a null member leaves the map entry at its zero value "" (json.Unmarshal)
                m[k] = std::string();
            } else if (!str(v)) {
                return false;                                // non-string member: a type error
            } else {
                m[k] = v;
            }
            ws();
            if (p < e && *p == ',') { ++p; continue; }
            if (p < e && *p == '}') { ++p; break; }
            return false;
        }
        kv.assign(m.begin(), m.end());
        return true;
    }
};

bool go_atoi64(const std::string &x, long long *out) {
    if (x.empty()) return false;
    size_t i = 0;
    bool neg = false;
    if (x[0] == '+' || x[0] == '-') {
        neg = x[0] == '-';
        i = 1;
        if (x.size() == 1) return false;
    }
    unsigned long long acc = 0;
    for (; i < x.size(); ++i) {
        const unsigned d = (unsigned char)x[i] - (unsigned)'0';
        if (d > 9 || acc > (0xFFFFFFFFFFFFFFFFULL - d) / 10) return false;
        acc = acc * 10 + d;
    }
    if ((!neg && acc >= 0x8000000000000000ULL) || (neg && acc > 0x8000000000000000ULL)) return false;
    *out = neg ? (long long)(0 - acc) : (long long)acc;
    return true;
}

}  // namespace

// *outcome: 0 = ingested into RemoteDiff (the reference then calls merge(),
// main.go:257); 1 = not valid JSON of that shape: nothing ingested, the round
// is skipped (main.go:247-249); 2 = a key failed Atoi: the reference's gossip
// goroutine returns (main.go:252-253) -- nothing is ingested here (Go's
// random map order makes "that key first" one of the legal executions).
// Keys with equal Atoi values ("1", "01") are applied in byte order of the
// key strings, the last one winning (one of Go's legal orders).
extern "C" int crdt_server_ingest_json(crdt_server *srv, const char *data, size_t len, int *outcome) {
    if (!srv || !outcome || (!data && len)) return CRDT_E_INVAL;
    JsonIn in{data, data + len};
    std::map<std::string, std::pair<std::vector<std::pair<std::string, std::string>>, bool>> top;
    bool ok = true;
    in.ws();
    if (in.lit("null")) {
        in.ws();
        ok = in.p == in.e;                                   // null: the map stays nil, no error
        *outcome = ok ? 0 : 1;
        return CRDT_OK;
    }
    if (in.p >= in.e || *in.p != '{') ok = false;
    else {
        ++in.p;
        in.ws();
        if (in.p < in.e && *in.p == '}') ++in.p;
        else {
            for (;;) {
                std::string k;
                in.ws();
                if (!in.str(k)) { ok = false; break; }
                in.ws();
                if (in.p >= in.e || *in.p != ':') { ok = false; break; }
                ++in.p;
                std::vector<std::pair<std::string, std::string>> kv;
                bool is_null = false;
                if (!in.inner(kv, &is_null)) { ok = false; break; }
                top[k] = {std::move(kv), is_null};             // duplicate keys: the last wins
                in.ws();
                if (in.p < in.e && *in.p == ',') { ++in.p; continue; }
                if (in.p < in.e && *in.p == '}') { ++in.p; break; }
                ok = false;
                break;
            }
        }
        in.ws();
        if (in.p != in.e) ok = false;                        // trailing data is a syntax error
    }
    if (!ok) { *outcome = 1; return CRDT_OK; }
    std::vector<std::pair<long long, const std::pair<std::vector<std::pair<std::string, std::string>>, bool> *>> puts;
    for (auto &t : top) {
        long long ts;
        if (!go_atoi64(t.first, &ts)) { *outcome = 2; return CRDT_OK; }
        puts.emplace_back(ts, &t.second);
    }
    std::lock_guard<std::mutex> g(srv->s.Lock);
    absorb_pending(srv->s);
    for (auto &pv : puts) {
        auto v = std::make_shared<Value>();
        v->local = false;
        v->kv = pv.second->first;
        v->nil = pv.second->second;
        srv->s.RemoteDiff[(int64_t)pv.first] = std::move(v);
    }
    *outcome = 0;
    return CRDT_OK;
}

// AliveState handler (main.go:141-151) after strconv.ParseBool: sets Alive.
extern "C" int crdt_server_set_alive(crdt_server *srv, int alive) {
    if (!srv) return CRDT_E_INVAL;
    std::lock_guard<std::mutex> g(srv->s.Lock);
    srv->s.Alive = alive != 0;
    return CRDT_OK;
}

// Ascending RemoteDiff keys (RemoteDiff.Keys()); writes min(cap, len).
extern "C" int crdt_server_remote_keys(crdt_server *srv, int64_t *ts, size_t cap, size_t *n) {
    if (!srv || !n) return CRDT_E_INVAL;
    std::lock_guard<std::mutex> g(srv->s.Lock);
    absorb_pending(srv->s);
    size_t i = 0;
    for (auto &e : srv->s.RemoteDiff) {
        if (i >= cap) break;
        if (ts) ts[i] = e.first;
        ++i;
    }
    *n = srv->s.RemoteDiff.size();
    return CRDT_OK;
}

// treemap Get(ts) on Diff (remote = 0) or RemoteDiff (remote = 1):
// CRDT_E_RANGE when ts is absent; else *npairs = the value's pair count and,
// when i < *npairs, its i-th pair (key, value).  Values are immutable once
// stored, so the pointers stay valid while the entry remains in the map.
extern "C" int crdt_server_entry_at(crdt_server *srv, int remote, int64_t ts, size_t i, const char **key,
                                    size_t *klen, const char **val, size_t *vlen, size_t *npairs) {
    if (!srv || !npairs) return CRDT_E_INVAL;
    std::lock_guard<std::mutex> g(srv->s.Lock);
    if (remote) {
        absorb_pending(srv->s);
    } else {
        int rc = make_host(srv->s);
        if (rc) return rc;
    }
    auto &m = remote ? srv->s.RemoteDiff : srv->s.Diff;
    auto it = m.find(ts);
    if (it == m.end()) return CRDT_E_RANGE;
    const Value &v = *it->second;
    *npairs = v.kv.size();
    if (i < v.kv.size()) {
        if (!key || !klen || !val || !vlen) return CRDT_E_INVAL;
        *key = v.kv[i].first.data();
        *klen = v.kv[i].first.size();
        *val = v.kv[i].second.data();
        *vlen = v.kv[i].second.size();
    }
    return CRDT_OK;
}

// ---------------------------------------------------------------- binary SoA gossip codec
// The same Diff as the JSON body (§8(f) row 2, "move to a binary SoA codec
// and keep the JSON codec"), with no text round trip: little-endian
//   char magic[8] = "CRDTSOA1"; u64 n_entries, n_pairs, n_bytes;
//   i64 ts[n_entries] (ascending); u32 pairs[n_entries] (0xFFFFFFFF: a nil map, no pairs);
//   u32 klen[n_pairs], vlen[n_pairs]; u8 bytes[n_bytes]
// (each pair's key bytes then value bytes, pairs of an entry sorted by key).
// Ingest is the decode loop of main.go:245-256 without Atoi: every entry is
// put into RemoteDiff as a remote map; duplicate ts / keys: the last wins.
namespace {
constexpr char kSoaMagic[8] = {'C', 'R', 'D', 'T', 'S', 'O', 'A', '1'};
constexpr uint32_t kNilPairs = 0xFFFFFFFFu;        // pairs[i] of a nil map (JSON null): no pairs follow

template <typename T>
void put_le(std::string &o, T v) {
    for (size_t i = 0; i < sizeof(T); ++i) o.push_back((char)((uint64_t)v >> (8 * i) & 0xFF));
}

static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__, "the wire format is read with native loads");
template <typename T>
T get_le(const unsigned char *p) {                  // one unaligned native load (x86-64 / little-endian host)
    T v;
    std::memcpy(&v, p, sizeof(T));
    return v;
}
}  // namespace

extern "C" int crdt_server_gossip_binary(crdt_server *srv, char *buf, size_t cap, size_t *len, int *http_status) {
    if (!srv || !len || !http_status) return CRDT_E_INVAL;
    std::string body;
    {
        std::lock_guard<std::mutex> g(srv->s.Lock);
        int rc = make_host(srv->s);
        if (rc) return rc;
        if (!srv->s.Alive) {
            *http_status = 502;
            body = "Unreachable";
        } else {
            *http_status = 200;
            uint64_t np = 0, nb = 0;
            std::vector<std::vector<const std::pair<std::string, std::string> *>> sorted;
            sorted.reserve(srv->s.Diff.size());
            for (auto &e : srv->s.Diff) {
                std::vector<const std::pair<std::string, std::string> *> kv;
                for (auto &x : e.second->kv) {
                    kv.push_back(&x);
                    nb += x.first.size() + x.second.size();
                }
                std::sort(kv.begin(), kv.end(), [](auto *a, auto *b) { return a->first < b->first; });
                np += kv.size();
                sorted.push_back(std::move(kv));
            }
            body.append(kSoaMagic, 8);
            put_le<uint64_t>(body, srv->s.Diff.size());
            put_le<uint64_t>(body, np);
            put_le<uint64_t>(body, nb);
            for (auto &e : srv->s.Diff) put_le<int64_t>(body, e.first);
            {
                size_t i = 0;
                for (auto &e : srv->s.Diff) {
                    const uint32_t c = (uint32_t)sorted[i++].size();
                    put_le<uint32_t>(body, e.second->nil ? kNilPairs : c);
                }
            }
            for (auto &kv : sorted)
                for (auto *x : kv) put_le<uint32_t>(body, (uint32_t)x->first.size());
            for (auto &kv : sorted)
                for (auto *x : kv) put_le<uint32_t>(body, (uint32_t)x->second.size());
            for (auto &kv : sorted)
                for (auto *x : kv) {
                    body += x->first;
                    body += x->second;
                }
        }
    }
    *len = body.size();
    if (!buf || cap < body.size()) return CRDT_E_RANGE;
    std::copy(body.begin(), body.end(), buf);
    return CRDT_OK;
}

namespace crdt {
// RemoteDiff.Put of every entry of a validated binary body (duplicate ts /
// keys: the last wins).
static void parse_soa_into(Server &s, const char *data, size_t) {
    const unsigned char *p = reinterpret_cast<const unsigned char *>(data);
    const uint64_t ne = get_le<uint64_t>(p + 8), np = get_le<uint64_t>(p + 16);
    const unsigned char *pts = p + 32, *ppairs = pts + ne * 8, *pkl = ppairs + ne * 4, *pvl = pkl + np * 4,
                        *pb = pvl + np * 4;
    uint64_t j = 0, off = 0;
    for (uint64_t i = 0; i < ne; ++i) {
        const uint32_t k0 = get_le<uint32_t>(ppairs + 4 * i), k = k0 == kNilPairs ? 0 : k0;
        std::map<std::string, std::string> m;                   // duplicate keys: the last wins
        for (uint32_t u = 0; u < k; ++u, ++j) {
            const uint32_t kl = get_le<uint32_t>(pkl + 4 * j), vl = get_le<uint32_t>(pvl + 4 * j);
            std::string key(reinterpret_cast<const char *>(pb + off), kl);
            off += kl;
            m[key] = std::string(reinterpret_cast<const char *>(pb + off), vl);
            off += vl;
        }
        auto v = std::make_shared<Value>();
        v->local = false;
        v->nil = k0 == kNilPairs;
        v->kv.assign(m.begin(), m.end());
        s.RemoteDiff[get_le<int64_t>(pts + 8 * i)] = std::move(v);
    }
}
}  // namespace crdt

// *outcome: 0 = ingested into RemoteDiff; 1 = malformed (nothing ingested).
extern "C" int crdt_server_ingest_binary(crdt_server *srv, const char *data, size_t len, int *outcome) {
    if (!srv || !outcome || (!data && len)) return CRDT_E_INVAL;
    *outcome = 1;
    PhaseClock pc("srv_ingest");
    const unsigned char *p = reinterpret_cast<const unsigned char *>(data);
    if (len < 32 || std::memcmp(p, kSoaMagic, 8) != 0) return CRDT_OK;
    const uint64_t ne = get_le<uint64_t>(p + 8), np = get_le<uint64_t>(p + 16), nb = get_le<uint64_t>(p + 24);
    // sizes in 128-bit-safe arithmetic: every count is bounded by the body length first
    if (ne > len / 12 || np > len / 8 || nb > len) return CRDT_OK;
    const uint64_t need = 32 + ne * 12 + np * 8 + nb;
    if (need != len) return CRDT_OK;
    const unsigned char *pts = p + 32, *ppairs = pts + ne * 8, *pkl = ppairs + ne * 4, *pvl = pkl + np * 4,
                        *pb = pvl + np * 4;
    // One pass: the pair and byte totals must match the header, and the
    // device takes the body as it is (decoded in HBM at the merge) when it is
    // the only pull: ts strictly ascending, keys of every entry strictly
    // ascending, no nil map -- what every served body is.  Else the host parse.
    // (15 -> 11 us per 400 KB body on the box's host: native loads, the
    // previous ts in a register, the key order decided on the first byte
    // when it differs)
    uint64_t j = 0, off = 0;
    bool device_form = true;
    int64_t prev_ts = 0;
    for (uint64_t i = 0; i < ne; ++i) {
        const uint32_t k0 = get_le<uint32_t>(ppairs + 4 * i);
        const int64_t ts = get_le<int64_t>(pts + 8 * i);
        const bool asc = i == 0 || ts > prev_ts;
        prev_ts = ts;
        if (k0 == kNilPairs) {
            device_form = false;
            continue;
        }
        if (k0 > np - j) return CRDT_OK;                       // more pairs than the header holds
        if (!asc) device_form = false;
        const unsigned char *prev = nullptr;
        uint32_t prev_len = 0;
        for (uint32_t u = 0; u < k0; ++u, ++j) {
            const uint32_t kl = get_le<uint32_t>(pkl + 4 * j), vl = get_le<uint32_t>(pvl + 4 * j);
            if ((uint64_t)kl + vl > nb - off) return CRDT_OK;    // more bytes than the header holds
            const unsigned char *key = pb + off;
            if (u && device_form) {
                const uint32_t m = std::min(prev_len, kl);
                const int c = m && prev[0] != key[0] ? (prev[0] < key[0] ? -1 : 1) : std::memcmp(prev, key, m);
                if (c > 0 || (c == 0 && prev_len >= kl)) device_form = false;
            }
            prev = key;
            prev_len = kl;
            off += (uint64_t)kl + vl;
        }
    }
    if (j != np || off != nb) return CRDT_OK;
    pc.mark("validate");
    std::lock_guard<std::mutex> g(srv->s.Lock);
    Server &s = srv->s;
    if (device_form && s.ctx && !s.pend && s.RemoteDiff.empty()) {
        if (len > s.pend_cap) {
            if (s.pend_body) (void)hipHostFree(s.pend_body);
            s.pend_body = nullptr;
            s.pend_cap = 0;
            void *q = nullptr;
            if (hipHostMalloc(&q, len + len / 2, 0) != hipSuccess) return CRDT_E_NOMEM;
            s.pend_body = (char *)q;
            s.pend_cap = len + len / 2;
        }
        memcpy(s.pend_body, data, len);
        pc.mark("copy");
        s.pend_len = len;
        s.pend = true;
        // its upload starts now, ordered before the merge on the context's
        // stream; on any failure here the merge uploads it instead
        s.pend_dev = bind(s.ctx) == CRDT_OK && dbuf(s.ctx, s.pull, len) == CRDT_OK &&
                     hipMemcpyAsync(s.pull.p, s.pend_body, len, hipMemcpyHostToDevice, s.ctx->stream) == hipSuccess;
        pc.mark("upload");
    } else {
        absorb_pending(s);
        parse_soa_into(s, data, len);
    }
    *outcome = 0;
    return CRDT_OK;
}
