/*
 * crdt_amd.h -- C-ABI of the MI355X-native batched CRDT merge engine.
 *
 * This is the drop-in boundary for the merge/compare path of
 * anuragsarkar97/crdt (/root/reference/main.go).  The reference exposes no
 * FFI: its path is the unexported Go method `func (server *Server) merge()`
 * (main.go:35-100) over a gods treemap ordered by `utils.Int64Comparator`
 * (main.go:106-107).  Every entry point below names the reference interface
 * it replaces; INTEGRATION.md shows the cgo binding a maintainer would add.
 *
 * Conventions:
 *   - plain pointers and sizes; no C++/torch types cross the boundary;
 *   - every call returns int: 0 = CRDT_OK, < 0 = crdt_status (never aborts,
 *     never throws);
 *   - "dev" pointers are device (HBM) addresses; work is enqueued on the
 *     context's stream and is asynchronous unless the name says _sync/_host;
 *   - the library never retains caller pointers past a call (cgo rule);
 *   - a context is single-stream and not thread-safe: one context per
 *     Server/goroutine, mirroring the reference's one mutex per Server
 *     (main.go:32, :43-44).
 */
#ifndef CRDT_AMD_H
#define CRDT_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CRDT_AMD_ABI_VERSION 1

typedef enum crdt_status {
    CRDT_OK = 0,
    CRDT_E_INVAL = -1,      /* bad argument (null pointer, size overflow, bad option) */
    CRDT_E_HIP = -2,        /* HIP runtime error; see crdt_ctx_last_hip_error() */
    CRDT_E_NOMEM = -3,      /* device allocation failed */
    CRDT_E_NODEV = -4,      /* no usable gfx950 device */
    CRDT_E_UNSORTED = -5,   /* input violates the documented sort order */
    CRDT_E_RANGE = -6,      /* an index/size does not fit the kernel's integer width */
    CRDT_E_COMM = -7,       /* RCCL error; see crdt_shard_comm_last_error() */
    CRDT_E_DEVICE = -8      /* a kernel raised a device-side failure flag (CRDT_DEV_*): output invalid */
} crdt_status;

typedef struct crdt_ctx crdt_ctx;

/* ---------------------------------------------------------------- library */
int         crdt_abi_version(void);
const char *crdt_status_str(int status);
int         crdt_device_count(int *count);

/* ---------------------------------------------------------------- context */
/* stream: a hipStream_t (e.g. torch.cuda.current_stream().cuda_stream), or
 * NULL for the device's default (null) stream.  The context never creates a
 * stream of its own: its work is ordered with the caller's copies. */
int crdt_ctx_create(int device, void *stream, crdt_ctx **out);
int crdt_ctx_destroy(crdt_ctx *ctx);
int crdt_ctx_set_stream(crdt_ctx *ctx, void *stream);
/* A non-blocking stream for hosts that want one (e.g. to overlap merges with
 * copies); pass it to crdt_ctx_create / crdt_ctx_set_stream. */
int crdt_stream_create(int device, void **stream);
int crdt_stream_destroy(void *stream);
int crdt_ctx_sync(crdt_ctx *ctx);
/* Device-side failure flags raised by kernels since the last clear (the
 * kernels cannot return an error): synchronises the context's stream, then
 * *flags = CRDT_DEV_* bits; clear != 0 resets them.  A set merge whose
 * decoupled look-back exceeded its bounded wait (a scheduling fault, never
 * expected) raises CRDT_DEV_LOOKBACK and its output is invalid. */
#define CRDT_DEV_LOOKBACK 1u
#define CRDT_DEV_RANGE 2u          /* a batch exceeded a per-replica kernel limit, or a pass found its
                                      inputs inconsistent (merge bitmaps): the output is invalid */
#define CRDT_DEV_PLAN 4u           /* a planned D2 merge's inputs fell outside its plan (or an OR-Set key
                                      chunk outgrew its LDS): that call's output is invalid, its count ~0 */
int crdt_ctx_device_status(crdt_ctx *ctx, uint32_t *flags, int clear);
int crdt_ctx_last_hip_error(const crdt_ctx *ctx);
/* Pre-size the context's device workspace so that later calls never
 * allocate (needed before graph capture). */
int crdt_ctx_reserve(crdt_ctx *ctx, size_t bytes);
/* Kernel-shape knobs (crdt_amd/csrc/knobs.inc: "join.unroll", "sets.lww_parts",
 * "sort.plan_cache", "codec.short_tab", ...).  In the product library
 * (libcrdt_amd.so) they are compile-time constants at their measured
 * defaults: crdt_set_option refuses every name with CRDT_E_INVAL, so no
 * process-global state is shared between contexts and no timing diagnostic
 * or failpoint can reach a caller.  The diagnostic build (libcrdt_amd_diag.so,
 * -DCRDT_DIAG; linked by tests and tools only) accepts them process-wide for
 * A/B runs, plus the timing diagnostics ("sort.rdd_diag",
 * "refmerge.diag_fold": kernels skip work, output wrong) and the failpoints
 * "fail.refmerge" (n: the next n RefMerge calls return CRDT_E_NOMEM before
 * touching the device) and "fail.zero_bits" (n: the next n two-pass merges
 * zero their merge bitmaps between the passes: the write pass must raise
 * CRDT_DEV_RANGE, never read out of range).  CRDT_E_INVAL for an unknown
 * name or value. */
int crdt_set_option(const char *name, int64_t value);
/* The knob's value in this build; "build.diag" reads 1 in the diagnostic
 * build, 0 in the product.  CRDT_E_INVAL for an unknown name. */
int crdt_get_option(const char *name, int64_t *value);

/* Device memory for hosts without an allocator of their own (the Go side). */
int crdt_dev_alloc(crdt_ctx *ctx, size_t bytes, void **dev);
int crdt_dev_free(crdt_ctx *ctx, void *dev);
int crdt_memcpy_h2d(crdt_ctx *ctx, void *dev_dst, const void *host_src, size_t bytes);
int crdt_memcpy_d2h(crdt_ctx *ctx, void *host_dst, const void *dev_src, size_t bytes);
int crdt_memset(crdt_ctx *ctx, void *dev_dst, int byte, size_t bytes);

/* ------------------------------------------------------- compare (a2)
 * utils.Int64Comparator (main.go:106-107): signed total order, -1/0/+1. */
int crdt_compare_int64(int64_t a, int64_t b);

/* ------------------------------------------------ G-Counter / PN-Counter (a6)
 * Replica population state: row-major [rows x nodes] uint64 in HBM.
 * No reference code: build-defined state-based CRDT joins. */

/* out[r][n] = max(a[r][n], b[r][n]) (unsigned).  out may alias a or b. */
int crdt_gcounter_join(crdt_ctx *ctx, const uint64_t *a_dev, const uint64_t *b_dev,
                       uint64_t *out_dev, size_t rows, size_t nodes);
/* out[n] = max_r a[r][n]  (the join of a whole population; identity 0). */
int crdt_gcounter_fold(crdt_ctx *ctx, const uint64_t *a_dev, size_t rows, size_t nodes,
                       uint64_t *out_dev);
/* out[r] = sum_n a[r][n] (uint64 wrap): the G-Counter value of every replica. */
int crdt_gcounter_value(crdt_ctx *ctx, const uint64_t *a_dev, size_t rows, size_t nodes,
                        uint64_t *out_dev);
/* PN-Counter = (P, N) pair: both joined in one launch.  Outputs may alias. */
int crdt_pncounter_join(crdt_ctx *ctx, const uint64_t *pa_dev, const uint64_t *na_dev,
                        const uint64_t *pb_dev, const uint64_t *nb_dev,
                        uint64_t *pout_dev, uint64_t *nout_dev, size_t rows, size_t nodes);
/* out[r] = (int64)(sum_n P[r][n] - sum_n N[r][n]) with uint64 wrap (main.go:95). */
int crdt_pncounter_value(crdt_ctx *ctx, const uint64_t *p_dev, const uint64_t *n_dev,
                         int64_t *out_dev, size_t rows, size_t nodes);

/* ------------------------------------------- streaming peaks
 * Measurement utilities, no reference counterpart: the bench reports every
 * kernel's fraction of a self-measured copy-kernel peak beside the spec peak.
 * crdt_stream_copy: dst = src, `bytes` (multiple of 16, 16-B aligned), 16-B
 * nontemporal loads / stores, `unroll` in {1,2,4,8} vectors in flight per
 * lane, grid = CUs x blocks_per_cu workgroups of 256.
 * crdt_stream_read: reads `bytes` of src, writes one word per workgroup to
 * sink_dev (sink_words >= CUs x blocks_per_cu). */
int crdt_stream_copy(crdt_ctx *ctx, const void *src_dev, void *dst_dev, size_t bytes, int unroll,
                     int blocks_per_cu);
int crdt_stream_read(crdt_ctx *ctx, const void *src_dev, size_t bytes, uint64_t *sink_dev, size_t sink_words,
                     int unroll, int blocks_per_cu);

/* ------------------------------------------------------ vector clocks (a7) */
typedef enum crdt_vc_class {
    CRDT_VC_EQUAL = 0,      /* a == b                  */
    CRDT_VC_BEFORE = 1,     /* a <  b  (a happened-before b) */
    CRDT_VC_AFTER = 2,      /* a >  b                  */
    CRDT_VC_CONCURRENT = 3  /* neither dominates        */
} crdt_vc_class;
/* Join of vector clocks is the elementwise max: crdt_gcounter_join. */
/* cls[p] = classify(a[p], b[p]) for [pairs x nodes] uint64 clocks.  With
 * nodes == 1 this is the sign of Int64Comparator (main.go:106) on unsigned
 * values, mapped EQUAL/BEFORE/AFTER. */
int crdt_vclock_classify(crdt_ctx *ctx, const uint64_t *a_dev, const uint64_t *b_dev,
                         uint8_t *cls_dev, size_t pairs, size_t nodes);

/* ---------------------------------------------- LWW-Element-Set / OR-Set (a8)
 * Structure-of-arrays tuples, sorted ascending by (key, ts, rep).
 * Tie rule: on an exactly equal (ts, rep) the left operand (a, the local
 * replica) wins, as the reference keeps the local value on an equal
 * timestamp (main.go:54-65). */
typedef struct crdt_tuples {
    uint64_t *key;
    uint64_t *ts;
    uint32_t *rep;
    uint8_t  *tomb;
} crdt_tuples;

/* LWW: one tuple per distinct key = the max (ts, rep) element (left wins an
 * exact tie; tombstoned winners are kept).  out capacity >= na + nb;
 * *out_count_dev (device uint64) receives the output length.  key / ts / rep
 * must be naturally aligned (8 / 8 / 4 bytes; CRDT_E_INVAL otherwise): the
 * passes stage them by LDS-DMA from any element offset. */
int crdt_lww_merge(crdt_ctx *ctx, const crdt_tuples *a, size_t na, const crdt_tuples *b,
                   size_t nb, crdt_tuples *out, uint64_t *out_count_dev);
/* OR-Set: union of unique tags (key, ts, rep); tomb OR-ed over equal tags. */
int crdt_orset_merge(crdt_ctx *ctx, const crdt_tuples *a, size_t na, const crdt_tuples *b,
                     size_t nb, crdt_tuples *out, uint64_t *out_count_dev);
/* The same two merges on UNSORTED inputs (config D2), as one device sort of
 * both sides together with a side bit between rep and tomb -- composite
 * order (key, ts, rep, side, tomb) is the stable merge of the two sorted
 * sides -- followed by a neighbour dedup of the sorted composites.  Where
 * the key offsets are dense enough no radix pass runs: the tuples are
 * grouped per tile by the key's top byte, then LWW gathers each byte's runs
 * into an LDS table of per-key winners and OR-Set gathers them into 2^9-key
 * chunks sorted in LDS; on large calls those forms are planned from a
 * sample of the inputs that the grouping pass checks (a miss redoes the
 * call from the exact ranges), and a context keeps the last sampled plan
 * per mode and size (later calls of that size launch from it with no
 * sample and no read-back; a tuple outside its ranges is a miss).  Output identical to
 * crdt_tuples_sort of each side then crdt_lww_merge / crdt_orset_merge.
 * Synchronises once at the end in the dense-key forms (the sample's check,
 * the OR-Set chunks' LDS limits), once more to read a plan the context does
 * not hold, and once to size the radix passes otherwise.  na + nb < 2^32; out capacity >=
 * na + nb; out must not overlap a or b (CRDT_E_INVAL: the dense-key forms
 * store before they know whether the call is redone from the inputs). */
int crdt_lww_merge_unsorted(crdt_ctx *ctx, const crdt_tuples *a, size_t na, const crdt_tuples *b,
                            size_t nb, crdt_tuples *out, uint64_t *out_count_dev);
int crdt_orset_merge_unsorted(crdt_ctx *ctx, const crdt_tuples *a, size_t na, const crdt_tuples *b,
                              size_t nb, crdt_tuples *out, uint64_t *out_count_dev);
/* Stream-ordered D2 merges (no host synchronisation: a HIP graph can capture
 * them).  The calls above may read their plan -- field ranges, composite
 * layout, which dense-key form applies -- back from the device and check the
 * sampled ranges at the end (one synchronisation each).  A host that merges
 * the same shape repeatedly (a replica population's key space; the gossip
 * loop of main.go:226-258 calls merge() every round) plans once:
 * crdt_set_merge_plan (mode 0 = LWW, 1 = OR-Set; synchronises once) computes
 * the exact plan of a, b -- widen != 0 widens each field range by 1/256 of
 * its span, for later inputs that drift -- and reserves the context's
 * workspace for it.  The _planned calls then enqueue the merge with no
 * read-back, for inputs of the same na / nb (CRDT_E_INVAL otherwise): the
 * composing pass checks every tuple against the plan, and a tuple outside it
 * (or an OR-Set key chunk over its LDS limits) raises CRDT_DEV_PLAN in the
 * context's status word and sets *out_count_dev = ~0 -- run the unplanned
 * call then.  Otherwise the output is the unplanned call's, bit for bit. */
typedef struct crdt_set_plan {
    uint64_t w[24];
} crdt_set_plan;
int crdt_set_merge_plan(crdt_ctx *ctx, int mode, const crdt_tuples *a, size_t na, const crdt_tuples *b,
                        size_t nb, uint32_t widen, crdt_set_plan *plan);
int crdt_lww_merge_unsorted_planned(crdt_ctx *ctx, const crdt_set_plan *plan, const crdt_tuples *a, size_t na,
                                    const crdt_tuples *b, size_t nb, crdt_tuples *out, uint64_t *out_count_dev);
int crdt_orset_merge_unsorted_planned(crdt_ctx *ctx, const crdt_set_plan *plan, const crdt_tuples *a, size_t na,
                                      const crdt_tuples *b, size_t nb, crdt_tuples *out, uint64_t *out_count_dev);
/* Sort n SoA tuples (device) into ascending (key, ts, rep, tomb) order --
 * the merge input order, with tomb (0/1) breaking exact tag ties so the
 * result does not depend on the input order (config D2: unsorted state).
 * LSD radix sort of a packed composite of the fields' offsets from their
 * minima; synchronises the stream once (to size the passes).  in and out
 * must not overlap.  n < 2^32. */
int crdt_tuples_sort(crdt_ctx *ctx, const crdt_tuples *in, size_t n, crdt_tuples *out);
/* out[i] = lower_bound(sorted[0..n), probes[i]) in unsigned order, for m
 * probes (device arrays): key-range sharding of a sorted set (§8(e) D). */
int crdt_u64_lower_bound(crdt_ctx *ctx, const uint64_t *sorted_dev, size_t n, const uint64_t *probes_dev,
                         size_t m, uint64_t *out_dev);
/* Sortedness check (host-facing validation): *bad_dev = number of adjacent
 * pairs with t[i] > t[i+1]. */
int crdt_tuples_count_unsorted(crdt_ctx *ctx, const crdt_tuples *t, size_t n,
                               uint64_t *bad_dev);
/* Stable merge of two sorted tuple arrays, every tuple kept (on an equal tag
 * a's copies first): out[0 .. na + nb).  The key-range owner's rank-order
 * merge of received runs in crdt_shard_*_merge_local (the population's side
 * = the stable merge of every rank's side in rank order); its length is known
 * on the host, so a tree of these merges needs no read-back. */
int crdt_tuples_merge(crdt_ctx *ctx, const crdt_tuples *a, size_t na, const crdt_tuples *b, size_t nb,
                      const crdt_tuples *out);

/* ------------------------------------------------ RefMerge (a1-a5)
 * Batched, bit-exact (*Server).merge() (main.go:35-100) for many replicas.
 * Each replica's Diff (L) and RemoteDiff (R) are ascending unique int64 ts
 * arrays (treemap keys under Int64Comparator, main.go:106), concatenated
 * over replicas with CSR offsets.  Entry e owns key/value pairs
 * [kv_off[e], kv_off[e+1]) of one kv arena (L entries' ranges and R
 * entries' ranges both index it).  kv_key is a key SLOT: the host interns
 * each replica's key strings into its own disjoint slot range.  kv_val is a
 * value string id into (str_bytes, str_off).
 * origin: 1 = local write (*Command, main.go:187) -- skipped by the replay
 * (main.go:80); 0 = remote map (main.go:245-255). */
typedef struct crdt_refmerge_in {
    uint32_t replicas;
    uint32_t n_slots;
    uint64_t n_l, n_r, n_kv, n_str;
    const uint64_t *l_off;      /* [replicas+1] */
    const int64_t  *l_ts;       /* [n_l] */
    const uint8_t  *l_origin;   /* [n_l] */
    const uint64_t *l_kv;       /* [n_l+1] */
    const uint64_t *r_off;      /* [replicas+1] */
    const int64_t  *r_ts;       /* [n_r] */
    const uint64_t *r_kv;       /* [n_r+1] */
    const uint32_t *kv_key;     /* [n_kv] slot id < n_slots */
    const uint32_t *kv_val;     /* [n_kv] string id < n_str */
    const uint8_t  *str_bytes;
    const uint64_t *str_off;    /* [n_str+1] */
} crdt_refmerge_in;

typedef struct crdt_refmerge_out {
    uint64_t *off;      /* [replicas+1] new Diff ranges */
    int64_t  *ts;       /* capacity n_l + n_r: new Diff keys, ascending per replica */
    uint8_t  *origin;   /* origin of each new Diff entry */
    int64_t  *src;      /* >= 0: index into L; < 0: R index j encoded as -(j+1) */
    uint8_t  *st_kind;  /* [n_slots] CurrentState: 0 absent, 1 verbatim, 2 sum */
    uint32_t *st_str;   /* [n_slots] verbatim value string id (kind 1) */
    int64_t  *st_sum;   /* [n_slots] Itoa() operand (kind 2) */
} crdt_refmerge_out;

/* All pointers in `in` / `out` are device pointers. */
int crdt_refmerge_batch(crdt_ctx *ctx, const crdt_refmerge_in *in, const crdt_refmerge_out *out);
/* crdt_refmerge_batch that also materialises the new Diff's kv pairs (the
 * values the reference's Diff.Put carries along with each key, main.go:60-64):
 * new entry i owns kv_key/kv_val[kv_off[i] .. kv_off[i+1]), a copy of its
 * source entry's pairs (out.src), and kv_off[out.off[replicas]] = the total
 * (also written at kv_off[n_l + n_r]).
 * The kv offsets come out of the merge's own passes, so the separate
 * segmented gather over out.src (crdt_seg_gather2_n) is not needed.
 * kv_off: capacity n_l + n_r + 1; kv_key / kv_val: capacity kv_cap (a total
 * over kv_cap raises CRDT_DEV_RANGE, nothing written past it). */
typedef struct crdt_refmerge_kv_out {
    uint64_t *kv_off;
    uint32_t *kv_key;
    uint32_t *kv_val;
    uint64_t kv_cap;
} crdt_refmerge_kv_out;
int crdt_refmerge_batch_kv(crdt_ctx *ctx, const crdt_refmerge_in *in, const crdt_refmerge_out *out,
                           const crdt_refmerge_kv_out *kv);
/* In-place pulls (an anti-entropy round, main.go:226-261, where every
 * replica's RemoteDiff is a peer's whole Diff already in HBM): replica p's R
 * is r_ts / r_kv [r_off[p] .. r_end[p]) -- ranges may overlap and r_ts /
 * r_kv / the kv arena may alias the L arrays, so no RemoteDiff is
 * assembled.  r_slot_delta (nullable) is added (mod 2^32) to the key slot
 * of every R pair of replica p (a peer's slots re-based to p's).  in->n_r
 * MUST equal the total of the R ranges (outputs sized n_l + n_r): ranges
 * summing past it, or a reversed range (r_end < r_off), raise CRDT_DEV_RANGE
 * and nothing is merged.  out.src of an R entry is -(its index in r_ts) - 1.
 * kv: as crdt_refmerge_batch_kv; REQUIRED (CRDT_E_INVAL otherwise) when
 * r_slot_delta is given -- a gather of the new Diff's pairs by src after
 * the merge cannot re-base the pulled slots. */
typedef struct crdt_refmerge_pull {
    const uint64_t *r_end;          /* [replicas] */
    const uint32_t *r_slot_delta;   /* [replicas] or NULL */
} crdt_refmerge_pull;
int crdt_refmerge_batch_pull(crdt_ctx *ctx, const crdt_refmerge_in *in, const crdt_refmerge_out *out,
                             const crdt_refmerge_pull *pull, const crdt_refmerge_kv_out *kv);
/* ts-range-sharded RefMerge (§8(e)): one batch of replicas whose logs are
 * split by ts range over G shards (one per GPU).  Steps per shard:
 *   1. crdt_refmerge_local_maxl -> all-reduce(MAX) over shards: max(L) per replica;
 *   2. crdt_refmerge_batch_ex(maxl = that, acc = per-slot accumulators): the
 *      shard's slice of the new Diff (shards concatenate in ts order) and its
 *      unreduced replay fold (state outputs untouched);
 *   3. acc_rank -> all-reduce(MAX) = cmax; acc_owner_str -> all-reduce(SUM);
 *      all-reduce(SUM) of acc.sum and acc.npar; acc_set_best;
 *   4. crdt_refmerge_finalize: CurrentState (st_*) from the reduced accumulators.
 * Integer-only reductions: bit-exact for any shard count. */
typedef struct crdt_refmerge_acc {
    uint64_t *best;     /* [n_slots] 0 = no remote holder; else rank << 32 | string id */
    int64_t  *sum;      /* [n_slots] wrapped sum of the parsable values (main.go:95) */
    uint32_t *npar;     /* [n_slots] number of parsable values */
} crdt_refmerge_acc;
/* maxl_dev (nullable): per-replica max(L) replacing the local L's last key
 * (INT64_MIN: none).  acc (nullable): per-slot accumulators written there
 * instead of finalising st_kind/st_str/st_sum. */
int crdt_refmerge_batch_ex(crdt_ctx *ctx, const crdt_refmerge_in *in, const crdt_refmerge_out *out,
                           const int64_t *maxl_dev, const crdt_refmerge_acc *acc);
int crdt_refmerge_local_maxl(crdt_ctx *ctx, const crdt_refmerge_in *in, int64_t *maxl_dev);
/* c[s] = best ? shard << 40 | rank : 0  (shards in ts order; shard < 2^23) */
int crdt_refmerge_acc_rank(crdt_ctx *ctx, const crdt_refmerge_acc *acc, size_t n_slots, uint32_t shard,
                           int64_t *c_dev);
/* v[s] = the string id if this shard holds the global max (c == cmax), else 0 */
int crdt_refmerge_acc_owner_str(crdt_ctx *ctx, const crdt_refmerge_acc *acc, size_t n_slots, const int64_t *c_dev,
                                const int64_t *cmax_dev, int64_t *v_dev);
/* acc.best[s] = cmax ? 1 << 32 | v : 0 (the reduced accumulator) */
int crdt_refmerge_acc_set_best(crdt_ctx *ctx, const crdt_refmerge_acc *acc, size_t n_slots, const int64_t *cmax_dev,
                               const int64_t *v_dev);
int crdt_refmerge_finalize(crdt_ctx *ctx, const crdt_refmerge_acc *acc, size_t n_slots, const uint8_t *str_bytes_dev,
                           const uint64_t *str_off_dev, uint64_t n_str, const crdt_refmerge_out *out);

/* Incremental replay (§8(f) row 3).  The reference re-folds the whole Diff
 * on every merge (main.go:76); a merge only adds remote entries, so a
 * per-key state keyed by ts can be carried across merges:
 *   crdt_replay_state_init(L)     -- state of the L logs' remote entries;
 *   crdt_refmerge_delta(L, R, st) -- the merge of crdt_refmerge_batch, but
 *       the replay folds only the inserted R entries into st (updated in
 *       place) and CurrentState (st_*) is finalised from st.
 * Bit-exact with crdt_refmerge_batch as long as st describes the L passed
 * in: after a delta merge the caller's next L is the new Diff.  A local
 * write that replaces a remote entry at the same ms (main.go:187) removes a
 * holder: rebuild st with crdt_replay_state_init then. */
typedef struct crdt_replay_state {
    uint64_t *best_key;  /* [n_slots] max over remote holders of ts ^ 2^63 (order-preserving) */
    uint32_t *best_str;  /* [n_slots] string id of that holder */
    int64_t  *sum;       /* [n_slots] wrapped sum of the parsable values */
    uint32_t *npar;      /* [n_slots] parsable holders */
    uint32_t *nhold;     /* [n_slots] remote holders (0: key absent from CurrentState) */
} crdt_replay_state;
int crdt_replay_state_init(crdt_ctx *ctx, const crdt_refmerge_in *in, const crdt_replay_state *st);
int crdt_refmerge_delta(crdt_ctx *ctx, const crdt_refmerge_in *in, const crdt_refmerge_out *out,
                        const crdt_replay_state *st);
/* Batched local apply (§8(f) row 1): AddCommand (main.go:173-215) for many
 * replicas in one call.  Replica p's commands are c_off[p] .. c_off[p+1] in
 * ARRIVAL order, command j = (c_ts[j], pairs [c_kv[j], c_kv[j+1]) of the
 * kv_key / kv_val arena, applied in the order given).  Per command, as the
 * handler does: Diff.Put(ts, &data) (main.go:187: an equal ts is REPLACED, so
 * of several same-ms commands the last stays), then the CurrentState apply
 * (main.go:188-207): an absent key is set verbatim and the command stops
 * (status 200); else Atoi(current) + Atoi(value) -> Itoa (int64 wrap), an
 * Atoi failure stops it with status 500.  The new Diff is written like a
 * RefMerge output (src >= 0: Diff index, < 0: command j as -(j+1)); the
 * state (kind/str/sum per key slot, as crdt_refmerge_out) is updated in
 * place.  At most 4096 commands per replica per call: a replica over the
 * limit raises CRDT_DEV_RANGE and nothing of it is applied (its Diff range
 * is empty, its state untouched, its commands' status 0), so the caller can
 * split its commands over several calls; the Alive check (502) is the
 * host's. */
typedef struct crdt_local_in {
    uint32_t replicas;
    uint32_t n_slots;
    uint64_t n_l, n_c, n_kv, n_str;
    const uint64_t *l_off;      /* [replicas+1] the Diffs (ascending unique ts per replica) */
    const int64_t  *l_ts;
    const uint8_t  *l_origin;
    const uint64_t *c_off;      /* [replicas+1] commands per replica */
    const int64_t  *c_ts;       /* [n_c] */
    const uint64_t *c_kv;       /* [n_c+1] pair ranges */
    const uint32_t *kv_key;     /* [n_kv] key slot */
    const uint32_t *kv_val;     /* [n_kv] value string id */
    const uint8_t  *str_bytes;
    const uint64_t *str_off;    /* [n_str+1] */
} crdt_local_in;
typedef struct crdt_local_out {
    uint64_t *off;              /* [replicas+1] */
    int64_t  *ts;               /* capacity n_l + n_c */
    uint8_t  *origin;
    int64_t  *src;
    uint16_t *status;           /* [n_c] HTTP status of each command: 200 / 500 */
    uint8_t  *st_kind;          /* [n_slots] CurrentState, in / out */
    uint32_t *st_str;
    int64_t  *st_sum;
} crdt_local_out;
int crdt_local_apply(crdt_ctx *ctx, const crdt_local_in *in, const crdt_local_out *out);

/* Go strconv.Atoi over a string arena: ok[s] = parsable, val[s] = value. */
int crdt_atoi_batch(crdt_ctx *ctx, const uint8_t *str_bytes_dev, const uint64_t *str_off_dev,
                    uint64_t n_str, uint8_t *ok_dev, int64_t *val_dev);

/* ------------------------------------------------ Server (a4): host mirror
 * The reference's state holder (main.go:23-33) kept on the host, with
 * merge() routed to crdt_refmerge_batch.  Key/value arguments are parallel
 * arrays of (pointer, length) byte strings; a repeated key overwrites (Go
 * map semantics).  All functions lock the server's mutex (main.go:32). */
typedef struct crdt_server crdt_server;
/* NewServer(port, initialState, friendList) (main.go:102-113).  ctx may be
 * NULL for a host-only server (gossip codec, AddCommand): merge() then
 * returns CRDT_E_INVAL. */
int crdt_server_new(crdt_ctx *ctx, int port, crdt_server **out);
int crdt_server_free(crdt_server *srv);
int crdt_server_init_state(crdt_server *srv, const char *const *keys, const size_t *key_lens,
                           const char *const *vals, const size_t *val_lens, size_t n);
/* Diff.Put(ts, value): local != 0 stores a *Command (main.go:187), else a
 * remote map (as merge inserts it, main.go:68).  Replaces an equal ts. */
int crdt_server_diff_put(crdt_server *srv, int64_t ts, int local, const char *const *keys,
                         const size_t *key_lens, const char *const *vals, const size_t *val_lens,
                         size_t n);
/* RemoteDiff.Put(int64(atoi(key)), value): gossip ingest (main.go:250-256). */
int crdt_server_remote_put(crdt_server *srv, int64_t ts, const char *const *keys,
                           const size_t *key_lens, const char *const *vals,
                           const size_t *val_lens, size_t n);
/* AddCommand after JSON decode (main.go:173-215): Diff.Put(ts_ms, &data) and
 * the local apply; *http_status = 200, 500 or 502. */
int crdt_server_add_command(crdt_server *srv, int64_t ts_ms, const char *const *keys,
                            const size_t *key_lens, const char *const *vals,
                            const size_t *val_lens, size_t n, int *http_status);
/* (*Server).merge() (main.go:35-100) on the GPU. */
int crdt_server_merge(crdt_server *srv);
/* merge() of n distinct servers (same device) in ONE batched device call. */
int crdt_servers_merge(crdt_server *const *servers, size_t n);
int crdt_server_diff_len(crdt_server *srv, size_t *n);
int crdt_server_remote_len(crdt_server *srv, size_t *n);
/* Ascending Diff keys and origins (1 = *Command); writes min(cap, len). */
int crdt_server_diff_keys(crdt_server *srv, int64_t *ts, uint8_t *local, size_t cap, size_t *n);
int crdt_server_state_len(crdt_server *srv, size_t *n);
/* i-th CurrentState entry in key order; pointers valid until the next
 * mutation of the server. */
int crdt_server_state_at(crdt_server *srv, size_t i, const char **key, size_t *key_len,
                         const char **val, size_t *val_len);

/* ------------------------------------------------ sharding (a9)
 * Contiguous row range [*begin, *end) of rank `rank` in a world of `world`
 * ranks (replica populations shard by contiguous rows). */
int crdt_shard_range(uint64_t rows, int world, int rank, uint64_t *begin, uint64_t *end);
/* Order-preserving map between uint64 and int64 (x ^ 2^63): lets a signed
 * int64 MAX all-reduce (RCCL/gloo) compute the unsigned max exactly. */
int crdt_u64_to_ordered_i64(crdt_ctx *ctx, const uint64_t *in_dev, int64_t *out_dev, size_t n);
int crdt_ordered_i64_to_u64(crdt_ctx *ctx, const int64_t *in_dev, uint64_t *out_dev, size_t n);

/* Multi-GPU joins over RCCL (xGMI).  The reference's analog is pull gossip of
 * whole logs over HTTP (main.go:226-258); there is no reference collective.
 * A communicator has one or more LOCAL members (a GPU, its crdt_ctx and its
 * RCCL rank):
 *   crdt_shard_comm_create    -- ONE process drives every listed GPU
 *                                (ncclCommInitAll; calls are RCCL groups);
 *   crdt_shard_comm_init_rank -- one member per process (one process per GPU,
 *                                ncclCommInitRank); `id` is rank 0's
 *                                crdt_shard_unique_id, shipped to every rank
 *                                by the host (any channel).
 * Per-member arguments are arrays indexed by member; pointers in them are
 * device pointers on that member's GPU.  Work is enqueued on each member's
 * context stream (crdt_shard_member_ctx) unless a call says it synchronises. */
typedef struct crdt_comm crdt_comm;
#define CRDT_SHARD_ID_BYTES 128
int crdt_shard_unique_id(void *id, size_t cap);
int crdt_shard_comm_create(const int *devices, int n, crdt_comm **out);
int crdt_shard_comm_init_rank(crdt_ctx *ctx, const void *id, int nranks, int rank, crdt_comm **out);
/* Loopback communicator: `members` ranks (1 .. 64) on ONE device in this
 * process, each with its own context and stream; the collectives are device
 * copies and a reduction kernel on a transport stream, ordered against the
 * member streams by events (no host synchronisation).  Every crdt_shard_*
 * protocol runs unchanged on it, so its multi-rank planning, offsets, tree
 * merges and reductions run at R > 1 on one GPU.  Real multi-GPU
 * communicators (the two calls above) use RCCL. */
int crdt_shard_comm_create_loopback(int device, int members, crdt_comm **out);
int crdt_shard_comm_destroy(crdt_comm *comm);
int crdt_shard_comm_info(const crdt_comm *comm, int *members, int *nranks, int *rank0);
enum { CRDT_SHARD_RCCL = 0, CRDT_SHARD_LOOPBACK = 1 };
int crdt_shard_comm_transport(const crdt_comm *comm, int *kind);
/* The RCCL this process runs: *version = ncclGetVersion (e.g. 22606 for
 * 2.26.6) and path (NUL-terminated, truncated to cap) = the shared object
 * the dynamic linker resolved ncclGetVersion to.  The library is linked
 * against /opt/rocm/lib/librccl, but in a process that already loaded
 * another librccl of the same soname (PyTorch's) that one is used. */
int crdt_rccl_info(int *version, char *path, size_t cap);
int crdt_shard_member_ctx(crdt_comm *comm, int member, crdt_ctx **ctx);
int crdt_shard_comm_last_error(const crdt_comm *comm);     /* last ncclResult_t */
int crdt_shard_sync(crdt_comm *comm);
/* Config E1: member i folds its [rows[i] x nodes] row shard (crdt_gcounter_fold),
 * then an all-reduce(max) of the nodes-long folds (RCCL: ncclAllReduce(ncclUint64,
 * ncclMax)): every
 * member's out[i] holds the global join of the whole population. */
int crdt_shard_fold_max_u64(crdt_comm *comm, const uint64_t *const *shard_dev, const size_t *rows, size_t nodes,
                            uint64_t *const *out_dev);
/* Config E2: divergent full-state copies joined in place,
 * ncclAllReduce(ncclUint64, ncclMax). */
int crdt_shard_allreduce_max_u64(crdt_comm *comm, uint64_t *const *buf_dev, size_t n);
/* Generic in-place all-reduce for the sharded RefMerge accumulators. */
enum { CRDT_SHARD_I64 = 0, CRDT_SHARD_U64 = 1, CRDT_SHARD_U32 = 2, CRDT_SHARD_I32 = 3 };
enum { CRDT_SHARD_SUM = 0, CRDT_SHARD_MAX = 1 };
int crdt_shard_allreduce(crdt_comm *comm, void *const *buf_dev, size_t n, int type, int op);
/* Keyed sets: member i contributes local[i] (n_local[i] tuples); every
 * member's out[i] (capacity cap) receives all ranks' tuples concatenated in
 * rank order; *n_total = that length (CRDT_E_RANGE if > cap).  Synchronises. */
int crdt_shard_set_allgather_v(crdt_comm *comm, const crdt_tuples *local, const size_t *n_local,
                               const crdt_tuples *out, size_t cap, size_t *n_total);
/* Key-range-sharded LWW / OR-Set merge of sorted inputs that EVERY member
 * holds in full (a[i], b[i]): splitters = rank quantiles of a sample of both
 * key arrays (identical data, so no exchange), each member merges its range,
 * then crdt_shard_set_allgather_v.  out[i] == crdt_lww_merge / crdt_orset_merge
 * of the whole inputs on every member.  Synchronises. */
int crdt_shard_lww_merge(crdt_comm *comm, const crdt_tuples *a, size_t na, const crdt_tuples *b, size_t nb,
                         const crdt_tuples *out, size_t cap, size_t *n_out);
int crdt_shard_orset_merge(crdt_comm *comm, const crdt_tuples *a, size_t na, const crdt_tuples *b, size_t nb,
                           const crdt_tuples *out, size_t cap, size_t *n_out);

/* All-to-all-v: member i sends send_counts[i * nranks + q] elements of
 * elem_size bytes to global rank q (its send buffer holds the segments in
 * rank order) and receives recv_counts[i * nranks + p] elements from rank p
 * into its recv buffer (segments in rank order); grouped ncclSend / ncclRecv
 * on the member streams, enqueued. */
int crdt_shard_alltoallv(crdt_comm *comm, const void *const *send, const size_t *send_counts, void *const *recv,
                         const size_t *recv_counts, size_t elem_size);
/* Keyed-set merge of a DISTRIBUTED population (the reference
 * analog is the whole-log exchange of main.go:226-258): member i holds only
 * its own tuples a[i] (na[i]) and b[i] (nb[i]), each sorted by (key, ts,
 * rep).  The population's A is the stable merge of every rank's A in rank
 * order (B likewise) and the result is crdt_lww_merge / crdt_orset_merge of
 * the two -- computed by key-range owners: sampled splitters weighted by the
 * ranks' sizes (one ncclAllGather), every rank's tuples sent to their owner
 * (crdt_shard_alltoallv), the owner's merge of the received runs (rank-order
 * pairwise merges of A's runs and of B's, then A with B).  gather != 0:
 * every member's out[i] receives the whole merged state, n_out[i] its
 * length; gather == 0: out[i] / n_out[i] = the member's own key range of it
 * (ranges ascend with rank).  CRDT_E_RANGE if a result exceeds cap.
 * Synchronises. */
int crdt_shard_lww_merge_local(crdt_comm *comm, const crdt_tuples *a, const size_t *na, const crdt_tuples *b,
                               const size_t *nb, const crdt_tuples *out, size_t cap, size_t *n_out, int gather);
int crdt_shard_orset_merge_local(crdt_comm *comm, const crdt_tuples *a, const size_t *na, const crdt_tuples *b,
                                 const size_t *nb, const crdt_tuples *out, size_t cap, size_t *n_out, int gather);
/* The same, each member's own key range only (gather == 0), its length
 * written to n_out_dev[i] (a device uint64 on member i's GPU) on the member
 * stream: no trailing synchronisation (with nranks > 1 planning still reads
 * back the samples and the count matrix).  CRDT_E_RANGE if cap is below a
 * member's received tuples.  Device-side failures: crdt_ctx_device_status. */
int crdt_shard_lww_merge_local_dev(crdt_comm *comm, const crdt_tuples *a, const size_t *na, const crdt_tuples *b,
                                   const size_t *nb, const crdt_tuples *out, size_t cap, uint64_t *const *n_out_dev);
int crdt_shard_orset_merge_local_dev(crdt_comm *comm, const crdt_tuples *a, const size_t *na, const crdt_tuples *b,
                                     const size_t *nb, const crdt_tuples *out, size_t cap,
                                     uint64_t *const *n_out_dev);
/* (*Server).merge() (main.go:35-100) of ONE batch of replicas whose Diff /
 * RemoteDiff logs are split by ts range over the ranks (global rank g holds
 * the g-th ts range of every replica; every member's kv_val ids index the
 * same string table): in[i] / out[i] are member i's slice and outputs in the
 * crdt_refmerge_batch layout.  One call runs the whole protocol on the
 * communicator's streams, no host synchronisation: all-reduce(MAX) of each
 * replica's max(L) (remote ts above the global max are dropped, main.go:49),
 * the local merge, the replay accumulators reduced across ranks (MAX of the
 * holder rank, SUM of its string id, of the wrapped sums and of the
 * parsable counts), CurrentState finalised on every member.  out[i].off /
 * ts / origin / src = member i's slice of the new Diffs (slices concatenate
 * in rank order); st_* = the whole CurrentState.  Bit-exact with
 * crdt_refmerge_batch of the unsharded batch. */
int crdt_shard_refmerge(crdt_comm *comm, const crdt_refmerge_in *in, const crdt_refmerge_out *out);

/* ------------------------------------------------ anti-entropy rounds (§8(f) row 4)
 * The gossip loop of main.go:226-261 for a whole replica population at once:
 * every round each replica pulls one friend's whole Diff (main.go:230, :159),
 * ingests it as remote maps (main.go:245-256) and merges (main.go:257); a
 * dead friend (-1) skips the round (main.go:234-239) -- Diff and CurrentState
 * unchanged.  Rounds are synchronous: every pull sees the Diffs as of the
 * round's start (one legal schedule of the reference's goroutines).  The
 * population's Diffs, string arena and CurrentState stay in HBM between
 * rounds; a round that raises a device flag returns CRDT_E_DEVICE and
 * leaves the population as it was.
 *
 * init (host arrays, the crdt_refmerge_in layout of ONE block of replicas):
 * replicas P, K = keys per replica (local replica i's key k is slot i*K + k),
 * first = the global id of local replica 0; l_off [P + 1] (l_off[0] = 0),
 * l_ts / l_origin (1 = *Command) [n_l], l_kv [n_l + 1] (l_kv[0] = 0),
 * kv_key (local slot ids) / kv_val (string ids) [l_kv[n_l]], the string
 * arena str_bytes / str_off [n_str + 1].  CurrentState starts empty
 * (NewServer with an empty initialState, main.go:102-105). */
typedef struct crdt_population crdt_population;
typedef struct crdt_strtab crdt_strtab;           /* (string tables: below, with the gossip decode) */
typedef struct crdt_population_init {
    uint32_t replicas;
    uint32_t keys_per_replica;
    uint64_t first;
    uint64_t n_str;
    const uint64_t *l_off;
    const int64_t *l_ts;
    const uint8_t *l_origin;
    const uint64_t *l_kv;
    const uint32_t *kv_key;
    const uint32_t *kv_val;
    const uint8_t *str_bytes;
    const uint64_t *str_off;
} crdt_population_init;
int crdt_population_create(crdt_ctx *ctx, const crdt_population_init *init, crdt_population **out);
int crdt_population_destroy(crdt_population *pop);
int crdt_population_info(const crdt_population *pop, uint32_t *replicas, size_t *n_entries, size_t *n_kv);
/* Copy the Diffs (init layout; kv_key as local slot ids) and CurrentState
 * (st_kind 0 absent / 1 string id st_str / 2 decimal st_sum, per slot) to
 * host buffers sized by crdt_population_info; any pointer may be NULL.
 * Synchronises. */
int crdt_population_read(crdt_population *pop, uint64_t *l_off, int64_t *ts, uint8_t *origin, uint64_t *l_kv,
                         uint32_t *kv_key, uint32_t *kv_val, uint8_t *st_kind, uint32_t *st_str, int64_t *st_sum);
/* One round with every peer on this population: local replica i pulls global
 * replica peers[i] (host array of P; == first + i: a self-pull, merge() runs
 * and rebuilds CurrentState, main.go:76; -1: dead).  The merge reads the
 * peers' Diffs in place (crdt_refmerge_batch_pull, key slots re-based, kv
 * pairs from its own passes).  The per-replica arrays go up through a
 * staging kernel that reads them from coherent pinned memory, and the last
 * kernel writes the next Diffs' bounds back into it with a completion word
 * the call polls (no copy-engine transfers; option pop.direct = 0 restores
 * hipMemcpyAsync + hipStreamSynchronize).  Returns once the round is done. */
int crdt_population_round(crdt_population *pop, const int64_t *peers);
/* POST /data on every replica at once (AddCommand, main.go:173-215, through
 * crdt_local_apply): replica p's commands c_off[p] .. c_off[p+1] in ARRIVAL
 * order (host arrays), command j = (c_ts[j], pairs [c_kv[j], c_kv[j+1]) of
 * kv_key (local slot ids of replica p's range) / kv_val (string ids of the
 * population's arena)).  Diff.Put of the *Command (an equal ts replaced,
 * main.go:187), then the CurrentState apply with the early return after a
 * new key and the 500 on an unparsable value (main.go:188-207);
 * status[j] = 200 / 500.  Any number of commands per replica (chunks of
 * 4096 per device call: chunk r = commands r*4096 .. of every replica).  On
 * an error the chunks before the failing one stay applied (their status
 * 200 / 500) and every command of the failing and later chunks has status 0
 * (not applied); a failed call leaves nothing to undo.  Synchronises. */
typedef struct crdt_population_cmds {
    const uint64_t *c_off;      /* [replicas + 1] */
    const int64_t *c_ts;        /* [n_c] */
    const uint64_t *c_kv;       /* [n_c + 1], c_kv[0] = 0 */
    const uint32_t *kv_key;
    const uint32_t *kv_val;
} crdt_population_cmds;
int crdt_population_add_commands(crdt_population *pop, const crdt_population_cmds *cmds, uint16_t *status);
/* Undo the last round (local or sharded): the Diffs and CurrentState as they
 * were before it -- they stay in the population's spare buffers until the
 * next round; CRDT_E_INVAL when there is nothing to undo.  Host bookkeeping
 * only (no synchronisation: later work is ordered on the population's stream). */
int crdt_population_undo(crdt_population *pop);
/* One round over a communicator (main.go:226-258 across GPUs): member i's
 * population (created on crdt_shard_member_ctx(comm, i)) holds global
 * replicas crdt_shard_range(total, nranks, rank0 + i); peers_all [total]
 * (host) is every replica's draw, identical on every rank.  The per-replica
 * counts are all-gathered, every rank sends only the Diffs others pull (one
 * point-to-point group) and merges what it received in place.
 * Synchronises. */
int crdt_population_round_sharded(crdt_comm *comm, crdt_population *const *pops, const int64_t *peers_all,
                                  uint64_t total);
/* One round whose pulls arrive on the wire (main.go:226-258 with the
 * Gossip body of main.go:159 in the binary form of crdt_server_gossip_binary):
 * body i = bodies[body_off[i], body_off[i+1]) (device memory; body_off host,
 * replicas + 1) is local replica i's pulled Diff, an empty body a failed GET
 * (the round skipped for i, main.go:234-239).  Decoded on the device against
 * the string tables (keys: key id k of replica i -> slot i*K + k, ids < K;
 * vals: the value ids -- the first wire round checks that vals holds the
 * population's strings at their ids and adopts its arena), the pulled pairs
 * behind the current Diff's, then merged as crdt_population_round.  A body
 * the device decode does not take (malformed, a nil map, unsorted, a key id
 * >= K) fails the call with CRDT_E_UNSORTED, its status in body_status[i]
 * (host, replicas words): nothing is committed (the previous round can no
 * longer be undone: the merge may already have run into the spare buffers).
 * Synchronises. */
int crdt_population_round_wire(crdt_population *pop, crdt_strtab *keys, crdt_strtab *vals, const uint8_t *bodies,
                               const uint64_t *body_off, uint32_t *body_status);

/* ------------------------------------------------ synthetic state (bench/tests)
 * SplitMix64-seeded generators; identical to the numpy
 * restatement in crdt_amd/synth.py. */
int crdt_synth_counters(crdt_ctx *ctx, uint64_t seed, uint32_t stream, uint64_t *out_dev,
                        size_t n, uint64_t index_base);
int crdt_synth_vclock_pairs(crdt_ctx *ctx, uint64_t seed, uint64_t *a_dev, uint64_t *b_dev,
                            size_t pairs, size_t nodes, uint64_t pair_base);
int crdt_synth_set_tuples(crdt_ctx *ctx, uint64_t seed, uint32_t side, const crdt_tuples *out,
                          size_t n, uint64_t key_space);

/* ------------------------------------------------ anti-entropy rounds (§8(f) row 4)
 * Device assembly of gossip pull rounds (main.go:226-261) for a replica
 * population held in the crdt_refmerge_in layout (crdt_amd/gossip.py).
 * Segmented copy with two sources: segment s copies source segment code[s]
 * (>= 0: A's segment code[s]; < 0: B's segment -code[s]-1, B may be NULL
 * when no code is negative) of elem_size-byte elements (1, 4 or 8) to
 * dst + dst_off[s] * elem_size; with delta (4-byte elements only) each
 * element of segment s gets + delta[s] (mod 2^32: key-slot re-basing).
 * wide = 1: one workgroup per segment (long segments), else one thread. */
int crdt_seg_offsets(crdt_ctx *ctx, size_t n_seg, const int64_t *code_dev, const uint64_t *a_off_dev,
                     const uint64_t *b_off_dev, uint64_t base, uint64_t *dst_off_dev);
int crdt_seg_copy(crdt_ctx *ctx, size_t n_seg, const int64_t *code_dev, const uint64_t *a_off_dev,
                  const uint64_t *b_off_dev, const uint64_t *dst_off_dev, size_t elem_size, const void *a_dev,
                  const void *b_dev, void *dst_dev, const uint32_t *delta_dev, int wide);
/* Two arrays by the same segment map in one pass: segment s of a0/b0 ->
 * dst0 with + delta0[s] (an elem_size-byte integer, mod 2^(8*elem_size);
 * delta0 may be NULL) and, when dst1 != NULL, of a1/b1 -> dst1 verbatim. */
int crdt_seg_copy2(crdt_ctx *ctx, size_t n_seg, const int64_t *code_dev, const uint64_t *a_off_dev,
                   const uint64_t *b_off_dev, const uint64_t *dst_off_dev, size_t elem_size, const void *a0_dev,
                   const void *b0_dev, void *dst0_dev, const void *delta0_dev, const void *a1_dev,
                   const void *b1_dev, void *dst1_dev, int wide);
/* crdt_seg_offsets and a one-thread-per-segment crdt_seg_copy2 (no delta)
 * fused into one pass: each segment is copied as soon as its scanned offset
 * is known (dst_off[n_seg] = base + total). */
int crdt_seg_gather2(crdt_ctx *ctx, size_t n_seg, const int64_t *code_dev, const uint64_t *a_off_dev,
                     const uint64_t *b_off_dev, uint64_t base, uint64_t *dst_off_dev, size_t elem_size,
                     const void *a0_dev, const void *b0_dev, void *dst0_dev, const void *a1_dev,
                     const void *b1_dev, void *dst1_dev);
/* crdt_seg_gather2 for 4-byte elements over the first *n_dev (device
 * memory, <= n_max) of n_max segments, base 0: the count stays on the device
 * (segments past it scan as empty, dst_off[i] = the total for i >= *n_dev),
 * so a caller needs no host round trip between the merge that wrote the
 * count and this gather (the gossip round's next-Diff kv pairs). */
int crdt_seg_gather2_n(crdt_ctx *ctx, size_t n_max, const uint64_t *n_dev, const int64_t *code_dev,
                       const uint64_t *a_off_dev, const uint64_t *b_off_dev, uint64_t *dst_off_dev,
                       const uint32_t *a0_dev, const uint32_t *b0_dev, uint32_t *dst0_dev, const uint32_t *a1_dev,
                       const uint32_t *b1_dev, uint32_t *dst1_dev);
/* dst[dst_off[s] .. dst_off[s+1]) = val[s] */
int crdt_seg_fill_u32(crdt_ctx *ctx, size_t n_seg, const uint64_t *dst_off_dev, const uint32_t *val_dev,
                      uint32_t *dst_dev);
/* off[i] = base + sum(counts[0..i)), off[n] = base + total; and back. */
int crdt_counts_to_offsets(crdt_ctx *ctx, const uint32_t *counts_dev, size_t n, uint64_t base, uint64_t *off_dev);
int crdt_offsets_to_counts(crdt_ctx *ctx, const uint64_t *off_dev, size_t n, uint32_t *counts_dev);

/* ------------------------------------------------ gossip wire codec (§8(f) row 2)
 * Gossip handler (main.go:153-170): *http_status = 502 ("Unreachable")
 * unless Alive, else 200 with server.Diff.ToJSON() (main.go:159): gods
 * treemap ToJSON -> json.Marshal of {FormatInt(ts): value}, keys sorted as
 * byte strings, Go 1.18 encoding/json escaping.  The body goes to buf when
 * cap allows (else CRDT_E_RANGE, *len = size needed). */
int crdt_server_gossip_json(crdt_server *srv, char *buf, size_t cap, size_t *len, int *http_status);
/* Gossip pull decode (main.go:245-256): json.Unmarshal into
 * map[string]map[string]string, then RemoteDiff.Put(int64(Atoi(key)), value).
 * *outcome: 0 ingested (call merge next, main.go:257); 1 invalid JSON or shape,
 * round skipped (main.go:247-249); 2 a key failed Atoi, the reference's
 * gossip goroutine returns (main.go:252-253), nothing ingested. */
int crdt_server_ingest_json(crdt_server *srv, const char *data, size_t len, int *outcome);
/* Binary SoA form of the same Diff (§8(f) row 2: keep JSON for
 * compatibility, add a binary codec): "CRDTSOA1", u64 n_entries, n_pairs,
 * n_bytes, i64 ts[], u32 pairs[], u32 klen[], u32 vlen[], bytes (little
 * endian).  Ingest: *outcome 0 = put into RemoteDiff, 1 = malformed. */
int crdt_server_gossip_binary(crdt_server *srv, char *buf, size_t cap, size_t *len, int *http_status);
int crdt_server_ingest_binary(crdt_server *srv, const char *data, size_t len, int *outcome);
/* Device string tables (string -> dense id in first-seen order, bytes in an
 * append-only arena; str_off[n] = bytes used): the key dictionary and the
 * value arena the device gossip decode interns into.  A table belongs to one
 * device; calls that add strings synchronise and refresh a host mirror
 * (crdt_strtab_get). */
/* (crdt_strtab: declared with crdt_population above) */
int crdt_strtab_create(crdt_ctx *ctx, size_t cap_strings, size_t cap_bytes, crdt_strtab **out);
int crdt_strtab_destroy(crdt_strtab *tab);
/* counts and the device arena (bytes_dev / off_dev nullable): off_dev[0..n_str]
 * is the crdt_refmerge_in str_off of the table's strings. */
int crdt_strtab_info(const crdt_strtab *tab, uint64_t *n_str, uint64_t *n_bytes, const uint8_t **bytes_dev,
                     const uint64_t **off_dev);
int crdt_strtab_get(const crdt_strtab *tab, uint64_t id, const char **p, size_t *len);
/* Intern the n strings [off_host[i], off_host[i+1]) of a device byte arena:
 * ids_dev[i] = the string's id (new strings appended).  Synchronises. */
int crdt_strtab_intern(crdt_ctx *ctx, crdt_strtab *tab, const uint8_t *bytes_dev, const uint64_t *off_host, size_t n,
                       uint32_t *ids_dev);

/* Gossip pull decoded on the device (§8(f) row 2; main.go:245-256): binary SoA
 * bodies (crdt_server_gossip_binary) concatenated in HBM become the
 * crdt_refmerge_in R arrays of one replica each: r_off (0-based entry ranges
 * per body), r_ts, r_kv (= kv_base + pair offsets), and at
 * [kv_base, kv_base + pairs) the kv arena's key slots (slot_base[b] + the
 * key's id in `keys`) and value string ids (ids in `vals`: the merge's string
 * arena is that table's).  body_status[b] (host): 0 decoded; 1 malformed
 * (nothing of it is usable, as crdt_server_ingest_binary's outcome 1); 2 valid
 * but not taken by the device path (a nil map, ts not strictly ascending,
 * keys of an entry not strictly ascending, a key id >= key_cap): decode that
 * body on the host; 4 a table was full.  The decoded arrays of a non-zero
 * body are not valid.  Synchronises once (once more for the headers when
 * host_hdr is NULL, and once more when new strings were interned). */
typedef struct crdt_gossip_bodies {
    uint32_t n_bodies;
    uint32_t key_cap;           /* key ids >= key_cap: status 2 (the replica's slot range is full) */
    uint64_t kv_base;           /* first kv-arena index of the decoded pairs */
    const uint8_t *data;        /* device: the bodies, concatenated */
    const uint64_t *body_off;   /* host [n_bodies+1]: byte ranges of the bodies in data */
    const uint32_t *slot_base;  /* host [n_bodies]: key slot of key id 0, per body */
    const uint8_t *host_hdr;    /* host [32*n_bodies] or NULL: each body's first 32 bytes, when the caller
                                   already holds them (skips the header gather and its wait) */
} crdt_gossip_bodies;
typedef struct crdt_gossip_decoded {
    uint64_t *r_off;            /* device [n_bodies+1] */
    int64_t  *r_ts;             /* device [entries] */
    uint64_t *r_kv;             /* device [entries+1] */
    uint32_t *kv_key;           /* device, written at [kv_base, kv_base + pairs) */
    uint32_t *kv_val;
} crdt_gossip_decoded;
int crdt_gossip_decode(crdt_ctx *ctx, const crdt_gossip_bodies *in, crdt_strtab *keys, crdt_strtab *vals,
                       const crdt_gossip_decoded *out, uint32_t *body_status);

/* AliveState handler (main.go:141-151), after strconv.ParseBool. */
int crdt_server_set_alive(crdt_server *srv, int alive);
/* Ascending RemoteDiff keys; writes min(cap, len). */
int crdt_server_remote_keys(crdt_server *srv, int64_t *ts, size_t cap, size_t *n);
/* treemap Get(ts) on Diff (remote = 0) / RemoteDiff (remote = 1): CRDT_E_RANGE
 * if absent; else *npairs and, when i < *npairs, the i-th (key, value) pair. */
int crdt_server_entry_at(crdt_server *srv, int remote, int64_t ts, size_t i, const char **key,
                         size_t *key_len, const char **val, size_t *val_len, size_t *npairs);

#ifdef __cplusplus
}
#endif
#endif /* CRDT_AMD_H */
