/*
 * crdt_oracle.c -- CPU restatement (checker) of the crdt merge path.
 *
 * TEST INFRASTRUCTURE ONLY (see crdt_oracle.h).  Parity status:
 *   - oc_refmerge / oc_go_atoi: restate /root/reference/main.go:35-100 and Go
 *     1.18 strconv.Atoi; PINNED by the hand-derived known-answer tests of
 *     SURVEY.md §8(c) (tests/golden/refmerge_kat.json).  The reference itself
 *     cannot be built here (no Go toolchain, gods/gin not vendored).
 *   - counters / vclock / sets: build-defined semantics (no reference code);
 *     reference parity UNPINNED, pinned only by the tests/golden KAT fixtures and
 *     algebraic property tests.
 */
#include "crdt_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Go strconv.Atoi, 64-bit int (Go 1.18 src/strconv/atoi.go).               */
/* Fast path (len < 19): optional '+'/'-', then >=1 decimal digits.          */
/* Slow path: ParseInt(s, 10, 0) -> ParseUint(base 10: no '_', no prefix)    */
/* with range check [-2^63, 2^63-1].  Both accept exactly                    */
/* ^[+-]?[0-9]+$ within int64 range (leading zeros allowed).                 */
/* ------------------------------------------------------------------------ */
int oc_go_atoi(const char *s, size_t len, int64_t *out)
{
    if (len == 0) return 0;
    size_t i = 0;
    int neg = 0;
    if (s[0] == '+' || s[0] == '-') {
        neg = (s[0] == '-');
        i = 1;
        if (len == 1) return 0;
    }
    uint64_t acc = 0;
    for (; i < len; ++i) {
        unsigned d = (unsigned char)s[i] - (unsigned)'0';
        if (d > 9) return 0;
        /* ParseUint overflow: acc*10 + d > 2^64-1 */
        if (acc > (UINT64_MAX - d) / 10) return 0;
        acc = acc * 10 + d;
    }
    if (!neg && acc >= (1ULL << 63)) return 0;
    if (neg && acc > (1ULL << 63)) return 0;
    *out = neg ? (int64_t)(0 - acc) : (int64_t)acc;
    return 1;
}

int oc_go_itoa(int64_t v, char *buf)
{
    char tmp[24];
    int n = 0;
    uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    do { tmp[n++] = (char)('0' + (u % 10)); u /= 10; } while (u);
    int k = 0;
    if (v < 0) buf[k++] = '-';
    while (n) buf[k++] = tmp[--n];
    buf[k] = 0;
    return k;
}

/* ------------------------------------------------------------------------ */
/* G-Counter join / fold, PN-Counter value (build-defined)  */
/* ------------------------------------------------------------------------ */
typedef struct join_job {
    const uint64_t *a, *b;
    uint64_t *out;
    size_t lo, hi;
} join_job;

static void *join_worker(void *p)
{
    join_job *j = (join_job *)p;
    for (size_t i = j->lo; i < j->hi; ++i) {
        uint64_t x = j->a[i], y = j->b[i];
        j->out[i] = x > y ? x : y;          /* unsigned max */
    }
    return NULL;
}

void oc_gcounter_join(const uint64_t *a, const uint64_t *b, uint64_t *out,
                      size_t rows, size_t nodes, int threads)
{
    size_t n = rows * nodes;
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    join_job jobs[256];
    size_t per = (n + (size_t)threads - 1) / (size_t)threads;
    for (int t = 0; t < threads; ++t) {
        size_t lo = per * (size_t)t, hi = lo + per;
        if (lo > n) lo = n;
        if (hi > n) hi = n;
        jobs[t] = (join_job){a, b, out, lo, hi};
    }
    if (threads == 1) { join_worker(&jobs[0]); return; }
    for (int t = 0; t < threads; ++t) pthread_create(&tid[t], NULL, join_worker, &jobs[t]);
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
}

void oc_gcounter_fold(const uint64_t *a, size_t rows, size_t nodes, uint64_t *out)
{
    for (size_t c = 0; c < nodes; ++c) out[c] = 0;   /* identity of max on uint64 */
    for (size_t r = 0; r < rows; ++r)
        for (size_t c = 0; c < nodes; ++c) {
            uint64_t v = a[r * nodes + c];
            if (v > out[c]) out[c] = v;
        }
}

void oc_pncounter_value(const uint64_t *p, const uint64_t *n, int64_t *out,
                        size_t rows, size_t nodes)
{
    for (size_t r = 0; r < rows; ++r) {
        uint64_t sp = 0, sn = 0;                   /* uint64 wraparound sums */
        for (size_t c = 0; c < nodes; ++c) { sp += p[r * nodes + c]; sn += n[r * nodes + c]; }
        out[r] = (int64_t)(sp - sn);
    }
}

/* ------------------------------------------------------------------------ */
/* Vector-clock classification (build-defined).             */
/* le = all a<=b, ge = all a>=b; EQUAL if both, BEFORE if le only, AFTER if  */
/* ge only, CONCURRENT otherwise.  nodes == 1 degenerates to the sign of the */
/* reference comparator (main.go:106) on unsigned values.                   */
/* ------------------------------------------------------------------------ */
typedef struct vc_job {
    const uint64_t *a, *b;
    uint8_t *cls;
    size_t lo, hi, nodes;
} vc_job;

static void *vc_worker(void *p)
{
    vc_job *j = (vc_job *)p;
    for (size_t q = j->lo; q < j->hi; ++q) {
        const uint64_t *x = j->a + q * j->nodes, *y = j->b + q * j->nodes;
        int le = 1, ge = 1;
        for (size_t k = 0; k < j->nodes; ++k) {
            if (x[k] > y[k]) le = 0;
            if (x[k] < y[k]) ge = 0;
        }
        j->cls[q] = (uint8_t)(le && ge ? OC_VC_EQUAL : le ? OC_VC_BEFORE : ge ? OC_VC_AFTER
                                                                              : OC_VC_CONCURRENT);
    }
    return NULL;
}

void oc_vclock_classify(const uint64_t *a, const uint64_t *b, uint8_t *cls,
                        size_t pairs, size_t nodes, int threads)
{
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    vc_job jobs[256];
    size_t per = (pairs + (size_t)threads - 1) / (size_t)threads;
    for (int t = 0; t < threads; ++t) {
        size_t lo = per * (size_t)t, hi = lo + per;
        if (lo > pairs) lo = pairs;
        if (hi > pairs) hi = pairs;
        jobs[t] = (vc_job){a, b, cls, lo, hi, nodes};
    }
    if (threads == 1) { vc_worker(&jobs[0]); return; }
    for (int t = 0; t < threads; ++t) pthread_create(&tid[t], NULL, vc_worker, &jobs[t]);
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
}

/* ------------------------------------------------------------------------ */
/* LWW-Element-Set / OR-Set (build-defined).                */
/* Stable merge of two (key, ts, rep)-sorted inputs: on an equal tuple the   */
/* element of A (the left/local operand) comes first (tie rule of            */
/* main.go:54-65: the local value is kept).                                  */
/* ------------------------------------------------------------------------ */
static int tup_cmp(const oc_tuples *x, size_t i, const oc_tuples *y, size_t j)
{
    if (x->key[i] != y->key[j]) return x->key[i] < y->key[j] ? -1 : 1;
    if (x->ts[i] != y->ts[j]) return x->ts[i] < y->ts[j] ? -1 : 1;
    if (x->rep[i] != y->rep[j]) return x->rep[i] < y->rep[j] ? -1 : 1;
    return 0;
}

static void tup_put(oc_tuples *o, size_t k, const oc_tuples *s, size_t i)
{
    o->key[k] = s->key[i];
    o->ts[k] = s->ts[i];
    o->rep[k] = s->rep[i];
    o->tomb[k] = s->tomb[i];
}

/* LWW: one tuple per key = the max (ts, rep) element; on an exact (ts, rep)
 * tie the first element in stable merged order wins (A before B, earlier
 * index before later).  Tombstoned winners are kept (they are state). */
size_t oc_lww_merge(const oc_tuples *a, size_t na, const oc_tuples *b, size_t nb,
                    oc_tuples *out)
{
    size_t i = 0, j = 0, n = 0;
    int have = 0;
    const oc_tuples *ws = NULL;
    size_t wi = 0;
    while (i < na || j < nb) {
        const oc_tuples *s;
        size_t k;
        if (j >= nb || (i < na && tup_cmp(a, i, b, j) <= 0)) { s = a; k = i++; }
        else { s = b; k = j++; }
        if (!have || s->key[k] != ws->key[wi]) {
            if (have) tup_put(out, n++, ws, wi);
            ws = s; wi = k; have = 1;
        } else if (s->ts[k] > ws->ts[wi] || (s->ts[k] == ws->ts[wi] && s->rep[k] > ws->rep[wi])) {
            ws = s; wi = k;                     /* strictly newer (ts, replica) wins */
        }
    }
    if (have) tup_put(out, n++, ws, wi);
    return n;
}

/* OR-Set: union of unique tags (key, ts, rep); tomb is OR-ed over equal tags. */
size_t oc_orset_merge(const oc_tuples *a, size_t na, const oc_tuples *b, size_t nb,
                      oc_tuples *out)
{
    size_t i = 0, j = 0, n = 0;
    while (i < na || j < nb) {
        const oc_tuples *s;
        size_t k;
        if (j >= nb || (i < na && tup_cmp(a, i, b, j) <= 0)) { s = a; k = i++; }
        else { s = b; k = j++; }
        if (n > 0 && tup_cmp(out, n - 1, s, k) == 0) {
            out->tomb[n - 1] |= s->tomb[k];
        } else {
            tup_put(out, n++, s, k);
        }
    }
    return n;
}

/* ------------------------------------------------------------------------ */
/* RefMerge: (*Server).merge(), /root/reference/main.go:35-100.              */
/* ------------------------------------------------------------------------ */
int oc_refmerge(const int64_t *l_ts, const uint8_t *l_origin, const uint32_t *l_kv, size_t nl,
                const int64_t *r_ts, const uint32_t *r_kv, size_t nr,
                const uint32_t *kv_key, const uint32_t *kv_val,
                const uint8_t *str_bytes, const uint64_t *str_off,
                uint32_t n_keys,
                int64_t *out_ts, uint8_t *out_origin, int64_t *out_src, size_t *out_n,
                uint8_t *st_kind, uint32_t *st_str, int64_t *st_sum)
{
    /* Walk, main.go:45-73.  hasIds/outIds are key snapshots (:45-48); the loop
     * runs while both cursors are in range (:49).  Equal ts -> local kept,
     * remote rejected (:54-65).  Local ts greater -> remote inserted (:66-69).
     * Otherwise the local cursor advances (:70-72).  Remote ts beyond max(L)
     * are therefore never reached and are dropped. */
    size_t *ins = (size_t *)malloc((nr ? nr : 1) * sizeof(size_t));
    if (!ins) return -1;
    size_t nins = 0, i = 0, j = 0;
    while (i < nl && j < nr) {
        int64_t cd = l_ts[i], cr = r_ts[j];     /* Sprintf/Atoi round trip is the identity (:52-53) */
        if (cd == cr) { i++; j++; }
        else if (cd > cr) { ins[nins++] = j; j++; }   /* Diff.Put(remote) (:67-68) */
        else { i++; }
    }
    /* The tree now holds L plus the inserted remote entries, ascending by the
     * signed Int64Comparator (main.go:106).  Materialise that order. */
    size_t a = 0, b = 0, n = 0;
    while (a < nl || b < nins) {
        if (b >= nins || (a < nl && l_ts[a] < r_ts[ins[b]])) {
            out_ts[n] = l_ts[a]; out_origin[n] = l_origin[a]; out_src[n] = (int64_t)a; a++;
        } else {
            size_t rj = ins[b++];
            out_ts[n] = r_ts[rj]; out_origin[n] = 0; out_src[n] = -(int64_t)rj - 1;
        }
        n++;
    }
    *out_n = n;
    free(ins);

    /* Replay, main.go:75-98: CurrentState rebuilt from empty (:76), Diff
     * iterated in DESCENDING ts (:77-78).  Local-origin values are *Command
     * and fail the map[string]string assertion (:80) -> nil map, no keys. */
    for (uint32_t k = 0; k < n_keys; ++k) { st_kind[k] = 0; st_str[k] = 0; st_sum[k] = 0; }
    for (size_t e = n; e-- > 0;) {
        if (out_origin[e]) continue;            /* *Command: skipped (:80) */
        uint32_t kb, ke;
        if (out_src[e] >= 0) { kb = l_kv[out_src[e]]; ke = l_kv[out_src[e] + 1]; }
        else { size_t rj = (size_t)(-out_src[e] - 1); kb = r_kv[rj]; ke = r_kv[rj + 1]; }
        for (uint32_t q = kb; q < ke; ++q) {
            uint32_t key = kv_key[q], val = kv_val[q];
            if (key >= n_keys) return -2;
            if (st_kind[key] == 0) {            /* first seen: verbatim string (:82-86) */
                st_kind[key] = 1; st_str[key] = val;
                continue;
            }
            int64_t curr;
            if (st_kind[key] == 1) {            /* Atoi(val1) (:87-90) */
                const char *s = (const char *)str_bytes + str_off[st_str[key]];
                size_t len = (size_t)(str_off[st_str[key] + 1] - str_off[st_str[key]]);
                if (!oc_go_atoi(s, len, &curr)) continue;
            } else {
                curr = st_sum[key];             /* Itoa/Atoi round trip is exact */
            }
            int64_t change;                     /* Atoi(valx) (:91-94) */
            const char *s = (const char *)str_bytes + str_off[val];
            size_t len = (size_t)(str_off[val + 1] - str_off[val]);
            if (!oc_go_atoi(s, len, &change)) continue;
            st_kind[key] = 2;                   /* curr + change, int64 wrap (:95-96) */
            st_sum[key] = (int64_t)((uint64_t)curr + (uint64_t)change);
        }
    }
    return 0;
}
