/*
 * tt.h — C ABI of libtt.so, the MI355X (gfx950) hot path of the two-tower
 * retrieval trainer and brute-force index.
 *
 * Every entry point is stream-ordered and asynchronous: it validates its
 * arguments on the host, enqueues HIP kernels on `stream` and returns.  No
 * entry point allocates device memory or synchronises; scratch comes from a
 * caller-owned workspace whose size is given by the matching *_workspace_size
 * query.  All pointers are device pointers unless stated otherwise; all
 * matrices are row-major with an explicit leading dimension (in elements).
 *
 * Return value: TT_OK (0) or a TT_ERR_* code; tt_last_error() returns a
 * thread-local message describing the last failure on the calling thread.
 *
 * Reference interfaces each entry point replaces are cited as
 * /root/reference/<file>:<line> (SelvinSelbaraju/hm-retrieval-two-tower).
 * The reference has no FFI: its "operator API" is the Keras layer/model
 * classes, so the citations name the TF op call sites.
 */
#ifndef TT_H_
#define TT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* tt_stream_t; /* a hipStream_t; NULL selects the null stream */

enum {
  TT_OK = 0,
  TT_ERR_BAD_ARG = 1,     /* invalid shape / pointer / parameter            */
  TT_ERR_HIP = 2,         /* a HIP runtime call failed                      */
  TT_ERR_UNSUPPORTED = 3, /* valid request this build does not implement    */
  TT_ERR_WORKSPACE = 4    /* workspace missing or smaller than required     */
};

/* Library version string, e.g. "tt 0.1.0 gfx950". */
const char* tt_version(void);
/* Thread-local description of the last error ("" if none). */
const char* tt_last_error(void);

/* Measurement hook (no reference counterpart): the NEXT launch of `kernel`
 * issued by the calling thread is bracketed by hipEventRecord(ev_start) and
 * hipEventRecord(ev_stop) on its launch stream; the probe then disarms.  Lets
 * a benchmark time one kernel of a multi-launch entry point with HIP events
 * on the stream it runs on.  ev_start/ev_stop are hipEvent_t (NULL disarms). */
enum {
  TT_PROBE_INBATCH_ROWS = 0, /* inbatch_pass_kernel<D,0> (rows pass)        */
  TT_PROBE_INBATCH_COLS = 1, /* inbatch_pass_kernel<D,1> (cols pass)        */
  TT_PROBE_INDEX_SCREEN = 2, /* screen kernel of tt_bruteforce_search       */
  TT_PROBE_INDEX_FINALIZE = 3, /* finalize kernel of tt_bruteforce_search   */
  TT_PROBE_COUNT = 4
};
int tt_probe_arm(int32_t kernel, void* ev_start, void* ev_stop);
/* As tt_probe_arm, and the armed launch is issued `reps` (>= 1) times back to
 * back between the two events (in-batch passes only: they are idempotent), so
 * the per-launch time is (stop - start) / reps without one event pair per
 * launch.  Other kernels ignore reps. */
int tt_probe_arm_repeat(int32_t kernel, void* ev_start, void* ev_stop, int32_t reps);

/* ------------------------------------------------------------------------ *
 * K2+K3  Grouped embedding gather + concat.
 * Replaces InputLayer.call  (pkg/modelling/layers/input_layer.py:45-69):
 * numeric features copied first, then per categorical feature
 * Embedding(table)[ids] (input_layer.py:37-41,67), concatenated on the last
 * axis (input_layer.py:68).  One launch for all features; each segment
 * writes straight into its column range of `out`.
 * Out-of-range ids produce zero rows (TF GPU gather semantics).
 * ------------------------------------------------------------------------ */
#define TT_MAX_SEGMENTS 32

typedef struct {
  const float* table;   /* [num_rows, dim] fp32, or [batch] values if ids==NULL */
  const int32_t* ids;   /* [batch] row ids; NULL = numeric pass-through column  */
  int64_t num_rows;     /* rows of `table` (ignored for numeric columns)        */
  int32_t dim;          /* embedding size (1 for numeric columns)               */
  int32_t col_offset;   /* first column of this segment in `out`                */
} tt_gather_segment;

int tt_gather_grouped(const tt_gather_segment* segs, int32_t num_segs,
                      int64_t batch, float* out, int64_t out_stride,
                      tt_stream_t stream);

/* Several InputLayer.call's of one batch (e.g. the query and the candidate
 * tower, two_tower_model.py:65-92) in ONE launch: call i gathers its
 * `num_segs` segments into its own `out` [batch, out_stride].  At most
 * TT_MAX_SEGMENTS segments in total. */
typedef struct {
  const tt_gather_segment* segs;
  int32_t num_segs;
  float* out;
  int64_t out_stride;
} tt_gather_call;

int tt_gather_multi(const tt_gather_call* calls, int32_t num_calls,
                    int64_t batch, tt_stream_t stream);

/* Row-sharded tables (data parallel / SURVEY C5): the owner of a shard
 * answers row requests from every rank in one launch.  Request j reads row
 * rows[j] of tables[tags[j]] into out[j, 0:dim] (zeros for an invalid tag or
 * row).  All tables must share `dim`. */
typedef struct {
  const float* table;  /* [num_rows, dim] fp32 */
  int64_t num_rows;
} tt_row_table;

int tt_gather_tagged(const tt_row_table* tables, int32_t num_tables, int32_t dim,
                     const int32_t* tags, const int32_t* rows, int64_t n,
                     float* out, int64_t out_stride, tt_stream_t stream);

/* Request routing for row-sharded tables (no reference counterpart: the
 * reference trains on one CPU; this is the exchange the data-parallel step
 * needs).  Global row r of a sharded table lives on rank
 * r % world.  tt_route_requests deduplicates a rank's lookups into ONE
 * request list, owner-major (inside an owner: by tag, then row ascending; an
 * id outside its table becomes row -1, owned by rank world-1, sorted first):
 *   send [R, 2] int32 (global row, tag), counts [world] int64 (requests per
 *   owner, R = their sum, also written to *num_requests), idx [num_lookups,
 *   batch] int32 = the position in `send` of each lookup's request.
 * Capacity: send holds num_lookups*batch pairs.  tt_route_owner expands the
 * n requests an owner received (recv [n, 2]) into tags [n], local rows [n]
 * (gid / world, -1 if invalid) and per tag the local rows of that tag's
 * requests with -1 elsewhere (table_ids [num_tags, n]). */
typedef struct {
  const int32_t* ids; /* [batch] row ids of one lookup (one feature)        */
  int64_t num_rows;   /* rows of the (global) table it reads               */
  int32_t tag;        /* table index, 0..num_tags-1                         */
} tt_route_lookup;

size_t tt_route_workspace_size(int32_t num_lookups, int64_t batch, int32_t world,
                               int64_t max_rows, int32_t num_tags);
int tt_route_requests(const tt_route_lookup* lookups, int32_t num_lookups,
                      int64_t batch, int32_t world, int32_t num_tags,
                      int32_t* send, long long* counts, int32_t* num_requests,
                      int32_t* idx, void* workspace, size_t workspace_bytes,
                      tt_stream_t stream);
/* tt_route_requests plus the route's sorted order, so a sparse sum / update
 * keyed by the requests needs no second sort (tt_sparse_routed):
 *   order [num_lookups*batch] = the lookup (l*batch + b) at each sorted
 *   position (owner, tag, row ascending; a request's lookups in lookup
 *   order), grp_first / grp_last [world*num_tags] = the first / last sorted
 *   position of each (owner, tag) group (empty: 0 / -1).  Any of the three
 *   may be NULL (grp_first and grp_last together). */
int tt_route_requests_ordered(const tt_route_lookup* lookups, int32_t num_lookups,
                              int64_t batch, int32_t world, int32_t num_tags,
                              int32_t* send, long long* counts, int32_t* num_requests,
                              int32_t* idx, int32_t* order, int32_t* grp_first,
                              int32_t* grp_last, void* workspace,
                              size_t workspace_bytes, tt_stream_t stream);
int tt_route_owner(const int32_t* recv, int64_t n, int32_t world,
                   int32_t num_tags, int32_t* tags, int32_t* rows,
                   int32_t* table_ids, tt_stream_t stream);

/* Fixed-capacity routing (no host sync, graph-capturable): the compact
 * owner-major requests of tt_route_requests (send, counts on the device, idx
 * [num_lookups]) laid into `cap` slots per owner: request j of owner o at
 * slot o*cap + j of send_padded [world*cap, 2], unused slots (-1, -1) (an
 * owner answers them with zero rows and applies nothing); idx_padded
 * [num_lookups] = each lookup's slot.  Every exchange of the step then has
 * the split sizes [cap]*world.  cap = num_lookups never overflows; a smaller
 * cap drops an owner's requests past it, adds their number to *overflow
 * (optional, zero it first) and marks their lookups idx_padded = -1 - owner:
 * the lookup reads a zero row and contributes no gradient (the step reports
 * the overflow and the sharded trainer raises on it). */
int tt_route_pad(const int32_t* send, const long long* counts, const int32_t* idx,
                 int64_t num_lookups, int32_t world, int64_t cap,
                 int32_t* send_padded, int32_t* idx_padded, int32_t* overflow,
                 tt_stream_t stream);

/* The whole fixed-capacity route in one call: the outputs of
 * tt_route_requests_ordered (counts, optional order / grp_first / grp_last)
 * and tt_route_pad (send_padded, idx_padded, optional overflow), and at world
 * 1 optionally tt_route_owner's view of the slots (owner_tags / owner_rows
 * [cap], owner_table_ids [num_tags, cap]: at one rank the slots ARE the
 * owner's requests).  Up to 8192 lookups whose keys fit 32 bits run as ONE
 * workgroup launch (LDS radix sort + scan + slot writes; TT_ROUTE_FUSED=0
 * forces the multi-launch path); otherwise the three calls above.  Results
 * are identical either way.  Workspace: tt_route_fixed_workspace_size. */
size_t tt_route_fixed_workspace_size(int32_t num_lookups, int64_t batch, int32_t world,
                                     int64_t max_rows, int32_t num_tags);
int tt_route_fixed(const tt_route_lookup* lookups, int32_t num_lookups, int64_t batch,
                   int32_t world, int32_t num_tags, int64_t cap, int32_t* send_padded,
                   int32_t* idx_padded, long long* counts, int32_t* overflow,
                   int32_t* order, int32_t* grp_first, int32_t* grp_last,
                   int32_t* owner_tags, int32_t* owner_rows, int32_t* owner_table_ids,
                   void* workspace, size_t workspace_bytes, tt_stream_t stream);

/* Opt-in fp32-faithful products: tt_inbatch_softmax_xent_loss's contract
 * (prepped = 0; loss may be NULL) with every score S_ij AND the softmax-
 * weighted sums P.V from bf16x3 products (x = hi + lo, both bf16: hi.hi +
 * hi.lo + lo.hi, fp32 accumulation — the reference's fp32 logits and
 * gradients, two_tower_model.py:92,124, to ~2^-16 relative) in both passes.
 * At trained score magnitudes (|S| ~ 100) this holds dQ and dC to the fp64
 * gradients within 1e-3 where the default bf16 operands do not.
 * Three MFMAs where the default issues one, one workgroup per CU. */
size_t tt_inbatch_fused_x3_workspace_size(int64_t n, int32_t dim);
int tt_inbatch_softmax_xent_x3(const float* q, int64_t ldq, const float* c,
                               int64_t ldc, int64_t n, int32_t dim,
                               const float* logq, float* lse, float* row_loss,
                               float* dq, float* dc, float loss_scale,
                               float* loss, void* workspace,
                               size_t workspace_bytes, tt_stream_t stream);

/* ------------------------------------------------------------------------ *
 * K8+K9  Sparse optimizer step on embedding tables.
 * Replaces the legacy Keras optimizer's sparse path reached from
 * TwoTowerModel.train_step -> optimizer.minimize
 * (pkg/modelling/models/two_tower_model.py:124, optimizer_factory.py:15-18):
 * _deduplicate_indexed_slices (Unique + UnsortedSegmentSum, duplicates summed
 * in batch order) followed by ResourceSparseApplyAdagradV2 /
 * the legacy Adam sparse update.
 *
 * A table may be looked up by several features of one batch (the reference's
 * duplicated `product_type_name`, main.py:57-68 with input_layer.py:31,66-67):
 * list each lookup as a source; the index list is the concatenation of the
 * sources' ids in source order and duplicates are summed in that order.
 * ------------------------------------------------------------------------ */
#define TT_MAX_SOURCES 4

typedef struct {
  float* table;        /* [num_rows, dim] parameters, updated in place          */
  float* slot0;        /* Adagrad accumulator / Adam first moment [num_rows,dim] */
  float* slot1;        /* Adam second moment, NULL for Adagrad                  */
  int64_t num_rows;
  int32_t dim;
  int32_t num_sources; /* 1..TT_MAX_SOURCES                                     */
  const int32_t* ids[TT_MAX_SOURCES];      /* [batch] row ids per source         */
  int32_t grad_col_offset[TT_MAX_SOURCES]; /* column of the source's slice in grad */
  /* Optional per-table gradient buffer: when non-NULL, this table's sources
   * read rows b of grad + b*grad_ld (+ grad_col_offset[s]) instead of the
   * call's grad / grad_stride — so ONE call (one sort) updates the tables of
   * both towers, whose input gradients are separate buffers.                */
  const float* grad;
  int64_t grad_ld;
} tt_sparse_table;

size_t tt_sparse_workspace_size(const tt_sparse_table* tables, int32_t num_tables,
                                int64_t batch);

/* acc += g*g ; w -= lr*g / (sqrt(acc) + epsilon) on every touched row, g the
 * duplicate-summed gradient (TF ResourceSparseApplyAdagradV2 CPU kernel). */
int tt_sparse_adagrad(const tt_sparse_table* tables, int32_t num_tables,
                      int64_t batch, const float* grad, int64_t grad_stride,
                      float lr, float epsilon, void* workspace,
                      size_t workspace_bytes, tt_stream_t stream);

/* The same update in two stages.  tt_sparse_sort builds and sorts the
 * (table | row id, lookup) keys — it reads only the ids, so it can run early
 * on a side stream, overlapped with the forward/backward compute;
 * tt_sparse_adagrad_sorted then does the segmented sums and the apply.  Both
 * calls must see the same tables (<= 16), batch and workspace, in that order.
 * Results are identical to tt_sparse_adagrad. */
int tt_sparse_sort(const tt_sparse_table* tables, int32_t num_tables,
                   int64_t batch, void* workspace, size_t workspace_bytes,
                   tt_stream_t stream);
int tt_sparse_adagrad_sorted(const tt_sparse_table* tables, int32_t num_tables,
                             int64_t batch, const float* grad, int64_t grad_stride,
                             float lr, float epsilon, void* workspace,
                             size_t workspace_bytes, tt_stream_t stream);

/* Adagrad on DISTINCT rows (no sort, no duplicate sums): slot j (< n) applies
 * grad row j (grad + j*grad_ld, tables[*].dim columns) to row rows[j] of
 * tables[tags[j]] (tags[j] < 0 or a row outside the table: nothing).  Every
 * (tag, row) must occur at most once — e.g. the requests a one-rank owner
 * receives from tt_route_requests.  Bit-identical to tt_sparse_adagrad on
 * those rows.  Tables share one dim; ids / grad_col_offset are ignored. */
int tt_sparse_adagrad_rows(const tt_sparse_table* tables, int32_t num_tables,
                           const int32_t* tags, const int32_t* rows, int64_t n,
                           const float* grad, int64_t grad_ld, float lr,
                           float epsilon, tt_stream_t stream);

/* The sparse calls never fault on a mismatched workspace: the sort stage
 * stamps the first 256 bytes of the workspace with a fingerprint of the
 * lookups it sorted, and the apply passes (of every sparse entry point above
 * and below) check it before touching a table.  A presorted apply that finds
 * another call's keys (or a sorted lookup pointing outside the call's
 * gradient) applies nothing from the affected blocks and records the error
 * in the header.  tt_sparse_status synchronises `stream`, returns
 * TT_ERR_BAD_ARG (message in tt_last_error) if an error was recorded since
 * the last check, and clears it.  A fresh workspace should start zeroed. */
int tt_sparse_status(void* workspace, size_t workspace_bytes, tt_stream_t stream);

/* Legacy Keras Adam sparse path: m,v decayed over the WHOLE slot, the scaled
 * duplicate-summed gradient scatter-added, then the WHOLE table updated with
 * lr_t = lr*sqrt(1-beta2^step)/(1-beta1^step) (step is 1-based). */
int tt_sparse_adam(const tt_sparse_table* tables, int32_t num_tables,
                   int64_t batch, const float* grad, int64_t grad_stride,
                   float lr, float beta1, float beta2, float epsilon,
                   int64_t step, void* workspace, size_t workspace_bytes,
                   tt_stream_t stream);

/* Dense gradient of each table from its lookups: every touched row of
 * `table` (a zero-filled [num_rows, dim] gradient buffer; slots unused) is
 * set to its duplicate-summed gradient, in the same summation order as
 * tt_sparse_adagrad.  Used by data-parallel training to all-reduce the
 * gradients of small replicated tables. */
int tt_sparse_scatter_sum(const tt_sparse_table* tables, int32_t num_tables,
                          int64_t batch, const float* grad, int64_t grad_stride,
                          void* workspace, size_t workspace_bytes,
                          tt_stream_t stream);

/* The per-request sums / updates of routed lookups, keyed by the route's own
 * sort (tt_route_requests_ordered + tt_route_pad): no second sort.  Table i
 * lists its lookups as sources (ids = the lookups' slots, idx_padded rows, in
 * lookup order) exactly as for tt_sparse_scatter_sum; `rs` maps every routed
 * lookup l to (tag, table, source).  Each table must take the lookups of one
 * tag.  Keys: the lookup's slot, or slot_row[slot] when slot_row is given
 * (e.g. tt_route_owner's local rows at world 1; -1 = nothing).  op 0: the
 * duplicate-summed rows written into each table (tt_sparse_scatter_sum);
 * op 1: Adagrad on them (tt_sparse_adagrad, lr / epsilon).  Results equal
 * those calls' on the same keys whenever the route lists each table's
 * lookups in the order that call sorts them (world 1: always). */
#define TT_ROUTE_MAX_LOOKUPS 32
typedef struct {
  const int32_t* order;     /* [num_lookups*batch], tt_route_requests_ordered */
  const int32_t* grp_first; /* [world*num_tags]                              */
  const int32_t* grp_last;
  const int32_t* slot;      /* [num_lookups*batch] slot of each lookup (idx_padded) */
  const int32_t* slot_row;  /* optional [world*cap]: key = slot_row[slot]     */
  int64_t cap;
  int32_t world;
  int32_t num_tags;
  int32_t num_lookups;
  int32_t lookup_tag[TT_ROUTE_MAX_LOOKUPS];
  int32_t lookup_table[TT_ROUTE_MAX_LOOKUPS];
  int32_t lookup_source[TT_ROUTE_MAX_LOOKUPS];
} tt_route_sorted;

int tt_sparse_routed(const tt_sparse_table* tables, int32_t num_tables, int64_t batch,
                     const float* grad, int64_t grad_stride, const tt_route_sorted* rs,
                     int32_t op, float lr, float epsilon, void* workspace,
                     size_t workspace_bytes, tt_stream_t stream);

/* tt_sparse_scatter_sum's block / join passes on keys tt_sparse_sort sorted
 * earlier (same tables, batch and workspace; the sort reads only the ids and
 * accepts tables without slots): the sort can run beside other work. */
int tt_sparse_scatter_sum_sorted(const tt_sparse_table* tables, int32_t num_tables,
                                 int64_t batch, const float* grad, int64_t grad_stride,
                                 void* workspace, size_t workspace_bytes,
                                 tt_stream_t stream);

/* Dedup only (K8), for parity checks: writes the U distinct ids of
 * ids[0..n) in ascending order, the per-id gradient sums [U, dim] (rows of
 * `grad` summed in index order) and U (device int32).  Capacity n rows. */
size_t tt_dedup_workspace_size(int64_t n, int32_t dim);
int tt_dedup_sum(const int32_t* ids, int64_t n, int64_t num_rows,
                 const float* grad, int64_t grad_stride, int32_t dim,
                 int32_t* unique_ids, float* summed, int32_t* num_unique,
                 void* workspace, size_t workspace_bytes, tt_stream_t stream);

/* K10  Dense optimizer steps on a flat parameter buffer (tower MLP weights).
 * ResourceApplyAdagradV2 / ResourceApplyAdam (optimizer_factory.py:15-18). */
int tt_dense_adagrad(float* param, float* accum, const float* grad, int64_t n,
                     float lr, float epsilon, tt_stream_t stream);
/* tt_dense_adagrad on up to 8 buffers in one launch (bit-identical to one
 * call per buffer). */
typedef struct {
  float* param;
  float* accum;
  const float* grad;
  int64_t n;
} tt_dense_job;
int tt_dense_adagrad_many(const tt_dense_job* jobs, int32_t num_jobs, float lr, float epsilon,
                          tt_stream_t stream);
int tt_dense_adam(float* param, float* m, float* v, const float* grad,
                  int64_t n, float lr, float beta1, float beta2, float epsilon,
                  int64_t step, tt_stream_t stream);

/* ------------------------------------------------------------------------ *
 * K5+K6+K7  Fused in-batch scores, logQ correction and softmax
 * cross-entropy (reduction SUM) with its gradient.
 * Replaces TwoTowerModel.call's matmul (two_tower_model.py:92),
 * LogQCorrection.__call__ (logq_correction.py:66-71), the eye-label
 * CategoricalCrossentropy(from_logits, SUM) (two_tower_model.py:119-122,
 * runner.py:78-83) and the tape gradient of that chain.
 *
 *   S'[i][j] = q_i . c_j - logq[j]
 *   loss_i   = logsumexp_j S'[i][j] - S'[i][pos(i)]
 *   dq_i     = sum_j softmax_j(S'[i]) c_j - c_pos(i)
 *   dc_j     = sum_i softmax(S'[i])_j q_i - q_pos^-1(j)
 *
 * Arithmetic contract: the NEGATIVE pairs are scored with bf16 (RNE)
 * operands and fp32 accumulation, and their exp weights enter the P.C /
 * P^T.Q products rounded to bf16 (relative to a power-of-two scale, so the
 * rounding is reproducible: oracle.inbatch_softmax_xent_bf16); the positive
 * pair is scored in fp32 and enters through the exact 1 - P_pos
 * (row_loss = softplus(lse_neg - pos), dq = (1 - P_pos)(mean_neg c - c_pos)),
 * so there is no P - I cancellation.  fp32 outputs; the [rows, cols]
 * score matrix is never materialised.  Rows and columns are given
 * separately so a rank can score its local rows against all-gathered
 * columns (global in-batch negatives): the positive column of local row i
 * is i + pos_offset, the positive row of local column j is j + pos_offset.
 * ------------------------------------------------------------------------ */
size_t tt_inbatch_workspace_size(int64_t n_rows, int64_t n_cols, int32_t dim);

/* Row pass: lse[i], row_loss[i] = lse[i] - S'[i][i+pos_offset], and (if dq
 * != NULL) dq [n_rows, dim] (ld = dim). */
int tt_inbatch_xent_rows(const float* q, int64_t ldq, int64_t n_rows,
                         const float* c, int64_t ldc, int64_t n_cols,
                         int32_t dim, const float* logq, int64_t pos_offset,
                         float* lse, float* row_loss, float* dq,
                         void* workspace, size_t workspace_bytes,
                         tt_stream_t stream);

/* Column pass: dc [n_cols, dim] (ld = dim) from all rows' q, lse and
 * row_loss (the rows pass's outputs; 1 - P_pos = -expm1(-row_loss).
 * row_loss may be NULL: then 1 - P_pos comes from lse and the fp32 positive
 * score, which cancels when the positive dominates). */
int tt_inbatch_xent_cols(const float* q, int64_t ldq, int64_t n_rows,
                         const float* lse, const float* row_loss,
                         const float* c, int64_t ldc, int64_t n_cols,
                         int32_t dim, const float* logq, int64_t pos_offset,
                         float* dc, void* workspace, size_t workspace_bytes,
                         tt_stream_t stream);

/* Single-device form of the two passes above (rows = cols = the batch,
 * positive of row i is column i): one shared bf16 preparation of q and c,
 * outputs lse, row_loss [n], dq, dc [n, dim] (ld = dim). */
size_t tt_inbatch_fused_workspace_size(int64_t n, int32_t dim);
int tt_inbatch_softmax_xent(const float* q, int64_t ldq, const float* c,
                            int64_t ldc, int64_t n, int32_t dim,
                            const float* logq, float* lse, float* row_loss,
                            float* dq, float* dc, void* workspace,
                            size_t workspace_bytes, tt_stream_t stream);

/* The same entry split at its preparation, so each tower's bf16 copy can be
 * made on the stream that produced that tower's output (the two towers that
 * TwoTowerModel.train_step runs, pkg/modelling/models/two_tower_model.py:
 * 111, finish on separate streams): tt_inbatch_prep with operand 0
 * prepares q, with operand 1 prepares c and the logQ bias vectors (logq may
 * be NULL, as above); both must be ordered before
 * tt_inbatch_softmax_xent_prepped on the same workspace, which then runs the
 * passes only.  Results are bit-identical to tt_inbatch_softmax_xent. */
int tt_inbatch_prep(const float* x, int64_t ldx, int64_t n, int32_t dim,
                    int32_t operand, const float* logq, void* workspace,
                    size_t workspace_bytes, tt_stream_t stream);
int tt_inbatch_softmax_xent_prepped(const float* q, int64_t ldq,
                                    const float* c, int64_t ldc, int64_t n,
                                    int32_t dim, const float* logq,
                                    float* lse, float* row_loss, float* dq,
                                    float* dc, void* workspace,
                                    size_t workspace_bytes,
                                    tt_stream_t stream);

/* tt_inbatch_softmax_xent (prepped = 0) or tt_inbatch_softmax_xent_prepped
 * (prepped = 1), also writing the step's loss *loss = loss_scale *
 * sum(row_loss) (the reference's SUM reduction, two_tower_model.py:122,
 * runner.py:78-83): one extra workgroup of the last launch sums the row
 * losses in tt_sum's order, so the value equals a tt_sum call bit for bit
 * without its launch. */
int tt_inbatch_softmax_xent_loss(const float* q, int64_t ldq, const float* c,
                                 int64_t ldc, int64_t n, int32_t dim,
                                 const float* logq, float* lse,
                                 float* row_loss, float* dq, float* dc,
                                 float loss_scale, float* loss,
                                 int32_t prepped, void* workspace,
                                 size_t workspace_bytes, tt_stream_t stream);

/* ------------------------------------------------------------------------ *
 * K11+K12  Brute-force scoring with fused top-K.
 * Replaces BruteForceIndex.call (pkg/modelling/indices/brute_force.py:76-81):
 * matmul(queries, candidates^T) then tf.math.top_k(k) (sorted descending,
 * ties -> lower index).  A bf16 MFMA screen keeps, per query, the scores
 * above a sampled rank estimate; the finalize certifies that list against
 * the bf16 error bound (or answers the query by an exact scan), rescores it
 * in fp32 as a k-ordered fmaf chain and returns the exact top-k.  Indices
 * are candidate positions + index_offset (the global offset of a shard).
 * ------------------------------------------------------------------------ */
/* Bytes of a prepared candidate image: 64-B header (sizes, max row norms),
 * bf16 copy [n_pad, D], then per row (|bf16(c)|_2, |c - bf16(c)|_2) for the
 * finalize's per-row screen bound. */
size_t tt_bruteforce_index_bytes(int64_t n_cand, int32_t dim);
int tt_bruteforce_build(const float* cand, int64_t ldc, int64_t n_cand,
                        int32_t dim, void* index, size_t index_bytes,
                        tt_stream_t stream);
size_t tt_bruteforce_workspace_size(int64_t n_queries, int64_t n_cand,
                                    int32_t dim, int32_t k);
int tt_bruteforce_search(const void* index, const float* cand, int64_t ldc,
                         int64_t n_cand, int32_t dim, const float* queries,
                         int64_t ldq, int64_t n_queries, int32_t k,
                         int64_t index_offset, float* out_scores,
                         int32_t* out_idx, void* workspace,
                         size_t workspace_bytes, tt_stream_t stream);

/* Candidate-sharded two-phase search (ShardedBruteForceIndex).
 * Replaces the same BruteForceIndex.call (brute_force.py:76-83) with the
 * candidate rows split over G ranks, each holding only its rows:
 *  1. tt_bruteforce_shard_screen on the rank's rows: bf16 screen + the
 *     finalize's select; kth_lb[q] = a lower bound on the k-th largest exact
 *     score of these rows (-inf when the query's certificate failed);
 *  2. the caller all-reduces kth_lb with MAX over the ranks: floor[q] bounds
 *     the GLOBAL k-th exact score from below;
 *  3. tt_bruteforce_shard_finalize: rescoring of the screened entries that
 *     can still reach floor, the shard's exact top-k of them with global
 *     indices (index_offset = the shard's first global row), padded with
 *     (-inf, INT32_MAX) past the survivors; failed certificates are scanned
 *     exactly over the shard.  Merging the G lists (tt_topk_merge) gives the
 *     exact global top-k.
 * Queries go in chunks of n_queries <= plan_queries; every call pair of one
 * search passes the same plan_queries, which must be equal on every rank
 * (tt_bruteforce_shard_chunk(total, n_g, ...) is rank g's recommendation: take
 * the minimum over the ranks) and the workspace is sized for it
 * (tt_bruteforce_shard_workspace_size(plan_queries, n_g, ...)).  A screen /
 * finalize pair of one chunk shares the workspace. */
int64_t tt_bruteforce_shard_chunk(int64_t n_queries, int64_t n_cand,
                                  int32_t dim, int32_t k);
size_t tt_bruteforce_shard_workspace_size(int64_t plan_queries, int64_t n_cand,
                                          int32_t dim, int32_t k);
int tt_bruteforce_shard_screen(const void* index, int64_t n_cand, int32_t dim,
                               const float* queries, int64_t ldq,
                               int64_t n_queries, int64_t plan_queries, int32_t k,
                               int64_t index_offset, float* kth_lb,
                               void* workspace, size_t workspace_bytes,
                               tt_stream_t stream);
int tt_bruteforce_shard_finalize(const void* index, const float* cand,
                                 int64_t ldc, int64_t n_cand, int32_t dim,
                                 const float* queries, int64_t ldq,
                                 int64_t n_queries, int64_t plan_queries,
                                 int32_t k, int64_t index_offset,
                                 const float* floor,
                                 float* out_scores, int32_t* out_idx,
                                 void* workspace, size_t workspace_bytes,
                                 tt_stream_t stream);

/* Merge `num_lists` per-shard sorted top-k_in lists laid out
 * [num_lists][n_queries][k_in] into the global top-k_out with the same
 * order (score descending, index ascending on ties). */
int tt_topk_merge(const float* scores, const int32_t* idx, int32_t num_lists,
                  int64_t n_queries, int32_t k_in, int32_t k_out,
                  float* out_scores, int32_t* out_idx, tt_stream_t stream);

/* The in-batch loss's batch reduction (CategoricalCrossentropy reduction
 * SUM, runner.py:78-83): out[0] = scale * sum(x[0..n)), one deterministic
 * single-workgroup launch. */
int tt_sum(const float* x, int64_t n, float scale, float* out, tt_stream_t stream);

/* ------------------------------------------------------------------------ *
 * K14  Recall hits (IndexRecall.__call__, metrics/index_recall.py:52-58):
 * hits[t] += #{b : true_ids[b] in cand_ids[b, 0:ks[t]]}.  hits is int64
 * [num_ks], accumulated (not overwritten).
 * ------------------------------------------------------------------------ */
int tt_recall_hits(const int32_t* true_ids, const int32_t* cand_ids,
                   int64_t batch, int32_t k_total, const int32_t* ks_host,
                   int32_t num_ks, int64_t* hits, tt_stream_t stream);


/* ------------------------------------------------------------------------ *
 * K15  Input pipeline.
 * Replaces the TFRecord dataset (pkg/modelling/tfrecord_dataset.py:59-98)
 * and the per-batch StringLookup (pkg/modelling/layers/input_layer.py:33-36).
 *
 * Host vocabulary (CPU only, no device memory): strings are passed as an
 * Arrow-style arena — `data` bytes and `offsets[n + 1]` (int64, value i is
 * data[offsets[i] .. offsets[i+1])).  vocab[i] -> row i + 1, any other value
 * -> row 0 (StringLookup num_oov_indices=1); a value listed twice maps to its
 * last row.  tt_vocab_create copies the arena; `num_threads` <= 0 uses every
 * hardware thread (at most 64).
 * ------------------------------------------------------------------------ */
int tt_vocab_create(const char* data, const int64_t* offsets, int64_t n, void** out_vocab);
int64_t tt_vocab_size(const void* vocab);
int tt_vocab_encode(const void* vocab, const char* data, const int64_t* offsets, int64_t n,
                    int32_t* out_rows, int32_t num_threads);
int tt_vocab_destroy(void* vocab);

/* Device batch assembly from an HBM-resident dataset of 32-bit words
 * (int32 rows / float32 values), column-major `src[ncols][src_ld]`:
 *   dst[c * dst_ld + b] = src[c * src_ld + perm[*cursor + b]],  b < batch,
 * then (advance != 0) *cursor += batch.  perm (int64 [n_rows]) is the
 * epoch's example order (the reference's shuffle buffer), cursor an int64 in
 * device memory, so the call can be captured in a replayed graph.  A position
 * or permutation entry outside [0, n_rows) writes zero words and ORs 1 into
 * *status (optional device int32). */
int tt_batch_take(const void* src, int64_t src_ld, int32_t ncols, const int64_t* perm, int64_t n_rows,
                  int64_t* cursor, int64_t batch, int32_t advance, void* dst, int64_t dst_ld,
                  int32_t* status, tt_stream_t stream);

/* ------------------------------------------------------------------------ *
 * K4  Tower MLP, row-streaming GEMM (Dense layers, pkg/modelling/models/
 * tower.py:41-49): C[M, N] = epi(maskA(A) . B) for a tall fp32 activation
 * A [M, K] and a small weight operand B [K, N] (N <= 384), on bf16x3 MFMA
 * (fp32-faithful: a_lo b_hi + a_hi b_lo + a_hi b_hi, fp32 accumulation).
 *   maskA (amask != NULL):  A := (amask > 0) ? A * (*scale) : 0   (ReluGrad)
 *   epilogue:  + bias[n] (bias != NULL), relu (relu != 0), then
 *              C := (cmask > 0) ? C : 0 (cmask != NULL)
 * B is first packed by tt_mlp_pack into a bf16 hi/lo image in MFMA fragment
 * order (img_bytes >= tt_mlp_pack_bytes(K, N)); trans != 0 packs B = W^T of a
 * row-major W [N, K] (the input-gradient GEMMs).  scale is a device scalar.
 * ------------------------------------------------------------------------ */
size_t tt_mlp_pack_bytes(int32_t K, int32_t N);
int tt_mlp_pack(const float* w, int64_t ldw, int32_t K, int32_t N, int32_t trans, void* img, size_t img_bytes,
                tt_stream_t stream);
/* Up to 8 packs in one launch (a tower's forward and transposed images). */
typedef struct {
  const float* w;
  int64_t ldw;
  int32_t K, N, trans;
  void* img;
  size_t img_bytes;
} tt_mlp_pack_job;
int tt_mlp_pack_many(const tt_mlp_pack_job* jobs, int32_t num_jobs, tt_stream_t stream);
/* tt_gather_multi and tt_mlp_pack_many in ONE launch (independent work: the
 * towers' input gather and the weight images their forward reads), so the
 * train step's forward starts with no pack launch and no fork in front of
 * it.  Results identical to the two calls.  batch >= 1, 1..8 jobs. */
int tt_gather_multi_pack(const tt_gather_call* calls, int32_t num_calls, int64_t batch,
                         const tt_mlp_pack_job* jobs, int32_t num_jobs, tt_stream_t stream);
/* colsum != NULL: also colsum[n] = sum_m C[m][n] (the bias gradient of the
 * layer below, BiasAddGrad): per-workgroup partial sums in the epilogue, then
 * one small launch adds them in workgroup order (deterministic); needs a
 * caller workspace of tt_mlp_rows_workspace_size(M, N) bytes. */
size_t tt_mlp_rows_workspace_size(int64_t M, int32_t N);
int tt_mlp_rows(const float* A, int64_t lda, const float* amask, int64_t ldam, const float* scale, int64_t M,
                int32_t K, const void* img, int32_t N, const float* bias, int32_t relu, const float* cmask,
                int64_t ldcm, float* C, int64_t ldc, float* colsum, void* workspace, size_t workspace_bytes,
                tt_stream_t stream);
/* Weight + bias gradient of a Dense layer (the tape's MatMul and BiasAddGrad):
 * dwb[Ka + 1, N] = [A | 1]^T . Gm, Gm = G, or (gmask > 0) ? G * (*scale) : 0
 * (gmask != NULL: the layer's own ReluGrad).  dwb row-major with ld N — the
 * flat parameter layout of kernel [Ka, N] followed by bias [N].  bf16x3 MFMA,
 * batch split over workgroups, partials added in split order (deterministic;
 * workspace of tt_mlp_wgrad_workspace_size bytes).  Ka + 1 <= 288, N <= 256. */
size_t tt_mlp_wgrad_workspace_size(int64_t M, int32_t Ka, int32_t N);
int tt_mlp_wgrad(const float* A, int64_t lda, const float* G, int64_t ldg, const float* gmask, int64_t ldgm,
                 const float* scale, int64_t M, int32_t Ka, int32_t N, float* dwb, void* workspace,
                 size_t workspace_bytes, tt_stream_t stream);
/* tt_mlp_wgrad plus the layer's Adagrad step (ResourceApplyAdagradV2 on
 * param / accum, the layer's [Ka + 1, N] region of the flat buffer and its
 * accumulator, 16-B aligned) applied by the partial-sum launch to the summed
 * gradient — tt_dense_adagrad's arithmetic, without its launch. */
int tt_mlp_wgrad_adagrad(const float* A, int64_t lda, const float* G, int64_t ldg, const float* gmask,
                         int64_t ldgm, const float* scale, int64_t M, int32_t Ka, int32_t N, float* dwb,
                         float* param, float* accum, float lr, float epsilon, void* workspace,
                         size_t workspace_bytes, tt_stream_t stream);

/* The two towers' layers as ONE launch each (the query and the candidate
 * tower are independent chains of the same shape of work: one stream, no
 * fork/join).  p points at 2 problems with tt_mlp_rows' / tt_mlp_wgrad's
 * arguments and contracts (rows: no colsum); the results equal two single
 * calls bit for bit.  Replaces the two towers' Dense layers of
 * two_tower_model.py:90-91 (query_tower(x), candidate_tower(x)). */
typedef struct {
  const float* A;
  int64_t lda;
  const float* amask;
  int64_t ldam;
  const float* scale;
  int64_t M;
  int32_t K;
  const void* img;
  int32_t N;
  const float* bias;
  int32_t relu;
  const float* cmask;
  int64_t ldcm;
  float* C;
  int64_t ldc;
} tt_mlp_rows_problem;
int tt_mlp_rows_pair(const tt_mlp_rows_problem* p, tt_stream_t stream);
typedef struct {
  const float* A;
  int64_t lda;
  const float* G;
  int64_t ldg;
  const float* gmask;
  int64_t ldgm;
  const float* scale;
  int64_t M;
  int32_t Ka, N;
  float* dwb;
} tt_mlp_wgrad_problem;
size_t tt_mlp_wgrad_pair_workspace_size(const tt_mlp_wgrad_problem* p);
int tt_mlp_wgrad_pair(const tt_mlp_wgrad_problem* p, void* workspace, size_t workspace_bytes, tt_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* TT_H_ */
