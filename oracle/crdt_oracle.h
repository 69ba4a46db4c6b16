/*
 * crdt_oracle.h -- CPU restatement of the merge path of anuragsarkar97/crdt.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under crdt_amd/ links, loads or calls
 * this library.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may use it, and only as the checker / the timed CPU
 * baseline -- never as a product path.
 *
 * Reference: /root/reference/main.go (Go 1.18, gods v1.18.1 treemap).
 *   - oc_refmerge()  restates (*Server).merge()            main.go:35-100
 *   - oc_go_atoi()   restates strconv.Atoi (Go 1.18, 64-bit int) used at
 *                    main.go:52-53, :87, :91
 *   - int64 comparator = utils.Int64Comparator             main.go:106-107
 * The G-Counter / PN-Counter / vector-clock / LWW-Set / OR-Set functions have
 * NO reference code: they restate the standard
 * state-based CRDT joins (Shapiro et al.) with the reference's tie rule
 * (left/local operand wins on an exact tie, main.go:54-65) and its integer
 * wraparound (main.go:95).  Parity for those is against this restatement;
 * reference parity is unpinned for them.
 */
#ifndef CRDT_ORACLE_H
#define CRDT_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Go strconv.Atoi (64-bit) : returns 1 and sets *out on success, 0 on any error ---- */
int oc_go_atoi(const char *s, size_t len, int64_t *out);
/* ---- Go strconv.Itoa : writes decimal text, returns length (buf >= 21 bytes) ---- */
int oc_go_itoa(int64_t v, char *buf);

/* ---- G-Counter / vector clock (a6): elementwise unsigned max ---- */
void oc_gcounter_join(const uint64_t *a, const uint64_t *b, uint64_t *out,
                      size_t rows, size_t nodes, int threads);
void oc_gcounter_fold(const uint64_t *a, size_t rows, size_t nodes, uint64_t *out);
/* PN-Counter value: sum(P[r,:]) - sum(N[r,:]) with uint64 wrap, read as int64 */
void oc_pncounter_value(const uint64_t *p, const uint64_t *n, int64_t *out,
                        size_t rows, size_t nodes);

/* ---- vector-clock classification (a7) ---- */
enum { OC_VC_EQUAL = 0, OC_VC_BEFORE = 1, OC_VC_AFTER = 2, OC_VC_CONCURRENT = 3 };
void oc_vclock_classify(const uint64_t *a, const uint64_t *b, uint8_t *cls,
                        size_t pairs, size_t nodes, int threads);

/* ---- LWW-Element-Set / OR-Set (a8): SoA tuples (key, ts, replica, tomb) ---- */
typedef struct oc_tuples {
    uint64_t *key;
    uint64_t *ts;
    uint32_t *rep;
    uint8_t  *tomb;
} oc_tuples;
/* Inputs sorted ascending by (key, ts, rep).  Returns the output count. */
size_t oc_lww_merge(const oc_tuples *a, size_t na, const oc_tuples *b, size_t nb,
                    oc_tuples *out);
size_t oc_orset_merge(const oc_tuples *a, size_t na, const oc_tuples *b, size_t nb,
                      oc_tuples *out);

/* ---- RefMerge (a1-a3): (*Server).merge(), main.go:35-100, one replica ----
 * Diff (L) / RemoteDiff (R) as ascending unique int64 ts arrays, each entry with
 * a CSR range into a key/value arena.  kv_key = per-replica dense key id,
 * kv_val = value string id into (str_bytes, str_off).
 * Outputs:
 *   out_ts/out_origin/out_src : the new Diff (ascending); out_src >= 0 is an L
 *                               index, out_src < 0 encodes R index as -(j+1).
 *   *out_n                    : size of the new Diff.
 *   st_kind[k]  0 = key absent, 1 = verbatim string (st_str[k] = string id),
 *               2 = integer sum (st_sum[k]), for k in [0, n_keys).
 */
int oc_refmerge(const int64_t *l_ts, const uint8_t *l_origin, const uint32_t *l_kv, size_t nl,
                const int64_t *r_ts, const uint32_t *r_kv, size_t nr,
                const uint32_t *kv_key, const uint32_t *kv_val,
                const uint8_t *str_bytes, const uint64_t *str_off,
                uint32_t n_keys,
                int64_t *out_ts, uint8_t *out_origin, int64_t *out_src, size_t *out_n,
                uint8_t *st_kind, uint32_t *st_str, int64_t *st_sum);

#ifdef __cplusplus
}
#endif
#endif
