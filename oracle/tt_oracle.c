/*
 * tt_oracle.c — CPU restatement of the reference hot path (TEST
 * INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker; never shipped, never the
 * measured product).
 *
 * Restates, from /root/reference (SelvinSelbaraju/hm-retrieval-two-tower):
 *   - BruteForceIndex.call: matmul(Q, C^T) + tf.math.top_k(k)
 *     (pkg/modelling/indices/brute_force.py:75-83). Scores are the k-ordered
 *     fp32 fmaf chain; top_k order: score descending, ties -> lower index.
 *   - legacy Keras optimizer sparse path (pkg/modelling/models/
 *     two_tower_model.py:124 -> optimizer_factory.py:15-18):
 *     _deduplicate_indexed_slices = Unique + UnsortedSegmentSum (rows of one
 *     id summed in increasing batch position starting from 0), then
 *     ResourceSparseApplyAdagradV2: acc += g*g; w -= lr*g/(sqrt(acc)+eps).
 * Compiled with -ffp-contract=off so no FMA is introduced where TF has none.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
  float s;
  int32_t i;
} entry_t;

/* a ranks before b (tf.math.top_k order) */
static inline int better(entry_t a, entry_t b) { return a.s > b.s || (a.s == b.s && a.i < b.i); }

/* min-heap on "worst first" */
static void sift_down(entry_t* h, int n, int p) {
  for (;;) {
    int l = 2 * p + 1, r = l + 1, w = p;
    if (l < n && better(h[w], h[l])) w = l;
    if (r < n && better(h[w], h[r])) w = r;
    if (w == p) return;
    entry_t t = h[p];
    h[p] = h[w];
    h[w] = t;
    p = w;
  }
}

static int cmp_better(const void* x, const void* y) {
  entry_t a = *(const entry_t*)x, b = *(const entry_t*)y;
  if (better(a, b)) return -1;
  if (better(b, a)) return 1;
  return 0;
}

float oracle_fmaf_dot(const float* q, const float* c, int dim) {
  float acc = 0.0f;
  for (int e = 0; e < dim; ++e) acc = fmaf(q[e], c[e], acc);
  return acc;
}

/* Exact fp32 brute-force top-k: out_s/out_i [nq, k].  Returns threads used. */
int oracle_bruteforce_topk(const float* q, int64_t ldq, int64_t nq, const float* c, int64_t ldc, int64_t n,
                           int dim, int k, float* out_s, int32_t* out_i, int nthreads) {
  int used = 1;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
  {
#pragma omp single
    used = omp_get_num_threads();
  }
#else
  (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t qi = 0; qi < nq; ++qi) {
    entry_t* h = (entry_t*)malloc(sizeof(entry_t) * (size_t)k);
    int hn = 0;
    const float* qr = q + qi * ldq;
    for (int64_t j = 0; j < n; ++j) {
      entry_t e;
      e.s = oracle_fmaf_dot(qr, c + j * ldc, dim) + 0.0f;
      e.i = (int32_t)j;
      if (hn < k) {
        h[hn++] = e;
        if (hn == k)
          for (int p = k / 2 - 1; p >= 0; --p) sift_down(h, k, p);
      } else if (better(e, h[0])) {
        h[0] = e;
        sift_down(h, k, 0);
      }
    }
    qsort(h, (size_t)hn, sizeof(entry_t), cmp_better);
    for (int t = 0; t < hn; ++t) {
      out_s[qi * k + t] = h[t].s;
      out_i[qi * k + t] = h[t].i;
    }
    free(h);
  }
  return used;
}

/* All fp32 fmaf-chain scores [nq, n]. */
void oracle_scores(const float* q, int64_t ldq, int64_t nq, const float* c, int64_t ldc, int64_t n, int dim,
                   float* out) {
#pragma omp parallel for schedule(static)
  for (int64_t qi = 0; qi < nq; ++qi)
    for (int64_t j = 0; j < n; ++j) out[qi * n + j] = oracle_fmaf_dot(q + qi * ldq, c + j * ldc, dim);
}

typedef struct {
  int32_t id;
  int32_t pos;
} idpos_t;

static int cmp_idpos(const void* x, const void* y) {
  const idpos_t* a = (const idpos_t*)x;
  const idpos_t* b = (const idpos_t*)y;
  if (a->id != b->id) return a->id < b->id ? -1 : 1;
  return a->pos < b->pos ? -1 : (a->pos > b->pos);
}

/* Distinct ids (ascending) and per-id gradient sums.
 * chunk == 0: TF order — one sequential sum 0 + g_p1 + g_p2 + ... over the
 *             id's positions in increasing order (UnsortedSegmentSum CPU).
 * chunk  > 0: the GPU's order — the lookups sorted by (id, position) are cut
 *             into aligned blocks of `chunk`; each segment's piece in a block
 *             is summed sequentially from 0 and the pieces are added in order
 *             starting from 0 (csrc/tt_sparse.hip, block_sum/join kernels).
 * grad row of position p is grad + p*ld.  Returns U. */
int oracle_dedup_sum(const int32_t* ids, int64_t n, const float* grad, int64_t ld, int dim, int chunk,
                     int32_t* uniq, float* sums) {
  idpos_t* v = (idpos_t*)malloc(sizeof(idpos_t) * (size_t)(n > 0 ? n : 1));
  for (int64_t p = 0; p < n; ++p) {
    v[p].id = ids[p];
    v[p].pos = (int32_t)p;
  }
  qsort(v, (size_t)n, sizeof(idpos_t), cmp_idpos);
  int u = 0;
  int64_t i = 0;
  float* part = (float*)malloc(sizeof(float) * (size_t)dim);
  while (i < n) {
    int64_t j = i;
    while (j < n && v[j].id == v[i].id) ++j;
    uniq[u] = v[i].id;
    float* out = sums + (int64_t)u * dim;
    for (int e = 0; e < dim; ++e) out[e] = 0.0f;
    if (chunk <= 0) {
      for (int64_t r = i; r < j; ++r)
        for (int e = 0; e < dim; ++e) out[e] = out[e] + grad[(int64_t)v[r].pos * ld + e];
    } else {
      for (int64_t r0 = i; r0 < j;) {
        int64_t r1 = (r0 / chunk + 1) * chunk;
        if (r1 > j) r1 = j;
        for (int e = 0; e < dim; ++e) part[e] = 0.0f;
        for (int64_t r = r0; r < r1; ++r)
          for (int e = 0; e < dim; ++e) part[e] = part[e] + grad[(int64_t)v[r].pos * ld + e];
        for (int e = 0; e < dim; ++e) out[e] = out[e] + part[e];
        r0 = r1;
      }
    }
    ++u;
    i = j;
  }
  free(part);
  free(v);
  return u;
}

/* ResourceSparseApplyAdagradV2 on distinct rows: table/accum [rows, dim]. */
void oracle_sparse_adagrad_apply(float* table, float* accum, int dim, const int32_t* uniq, const float* sums, int u,
                                 float lr, float eps) {
  for (int q = 0; q < u; ++q) {
    float* w = table + (int64_t)uniq[q] * dim;
    float* a = accum + (int64_t)uniq[q] * dim;
    const float* g = sums + (int64_t)q * dim;
    for (int e = 0; e < dim; ++e) {
      a[e] = a[e] + g[e] * g[e];
      w[e] = w[e] - (lr * g[e]) / (sqrtf(a[e]) + eps);
    }
  }
}
