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
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e);

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
    srv->s.Diff[ts] = make_value(local != 0, keys, klen, vals, vlen, n);   // treemap Put replaces
    return CRDT_OK;
}

extern "C" int crdt_server_remote_put(crdt_server *srv, int64_t ts, const char *const *keys, const size_t *klen,
                                      const char *const *vals, const size_t *vlen, size_t n) {
    if (!srv || !kv_args_ok(keys, klen, vals, vlen, n)) return CRDT_E_INVAL;
    // main.go:255 writes RemoteDiff from the gossip goroutine without the lock;
    // here the lock is taken so concurrent callers stay safe.
    std::lock_guard<std::mutex> g(srv->s.Lock);
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
    rc = merge_locked(ctx, v.data(), v.size());
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
    s.Diff[ts_ms] = v;                                     // same-ms writes overwrite
    s.state_view.clear();
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
    *n = srv->s.Diff.size();
    return CRDT_OK;
}

extern "C" int crdt_server_remote_len(crdt_server *srv, size_t *n) {
    if (!srv || !n) return CRDT_E_INVAL;
    std::lock_guard<std::mutex> g(srv->s.Lock);
    *n = srv->s.RemoteDiff.size();
    return CRDT_OK;
}

// Ascending Diff keys (Diff.Keys(), main.go:45) with their origin; either
// output may be NULL.  Writes min(cap, len) entries.
extern "C" int crdt_server_diff_keys(crdt_server *srv, int64_t *ts, uint8_t *local, size_t cap, size_t *n) {
    if (!srv || !n) return CRDT_E_INVAL;
    std::lock_guard<std::mutex> g(srv->s.Lock);
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

template <typename T>
T get_le(const unsigned char *p) {
    uint64_t v = 0;
    for (size_t i = 0; i < sizeof(T); ++i) v |= (uint64_t)p[i] << (8 * i);
    return (T)v;
}
}  // namespace

extern "C" int crdt_server_gossip_binary(crdt_server *srv, char *buf, size_t cap, size_t *len, int *http_status) {
    if (!srv || !len || !http_status) return CRDT_E_INVAL;
    std::string body;
    {
        std::lock_guard<std::mutex> g(srv->s.Lock);
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

// *outcome: 0 = ingested into RemoteDiff; 1 = malformed (nothing ingested).
extern "C" int crdt_server_ingest_binary(crdt_server *srv, const char *data, size_t len, int *outcome) {
    if (!srv || !outcome || (!data && len)) return CRDT_E_INVAL;
    *outcome = 1;
    const unsigned char *p = reinterpret_cast<const unsigned char *>(data);
    if (len < 32 || std::memcmp(p, kSoaMagic, 8) != 0) return CRDT_OK;
    const uint64_t ne = get_le<uint64_t>(p + 8), np = get_le<uint64_t>(p + 16), nb = get_le<uint64_t>(p + 24);
    // sizes in 128-bit-safe arithmetic: every count is bounded by the body length first
    if (ne > len / 12 || np > len / 8 || nb > len) return CRDT_OK;
    const uint64_t need = 32 + ne * 12 + np * 8 + nb;
    if (need != len) return CRDT_OK;
    const unsigned char *pts = p + 32, *ppairs = pts + ne * 8, *pkl = ppairs + ne * 4, *pvl = pkl + np * 4,
                        *pb = pvl + np * 4;
    uint64_t pairs_total = 0, bytes_total = 0;
    for (uint64_t i = 0; i < ne; ++i) {
        const uint32_t k = get_le<uint32_t>(ppairs + 4 * i);
        pairs_total += k == kNilPairs ? 0 : k;
    }
    if (pairs_total != np) return CRDT_OK;
    for (uint64_t j = 0; j < np; ++j) bytes_total += (uint64_t)get_le<uint32_t>(pkl + 4 * j) + get_le<uint32_t>(pvl + 4 * j);
    if (bytes_total != nb) return CRDT_OK;
    std::vector<std::pair<int64_t, std::shared_ptr<Value>>> puts;
    puts.reserve(ne);
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
        puts.emplace_back(get_le<int64_t>(pts + 8 * i), std::move(v));
    }
    std::lock_guard<std::mutex> g(srv->s.Lock);
    for (auto &pv : puts) srv->s.RemoteDiff[pv.first] = std::move(pv.second);
    *outcome = 0;
    return CRDT_OK;
}
