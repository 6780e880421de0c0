/* ORACLE — test infrastructure, NOT product code.
 *
 * Float64 LightGCN propagation chains at the BASELINE sizes (C3: 50M edges,
 * d=128; C4: 50M, d=64; C5: 500M, d=256), for the full-size parity tests
 * (tests/test_gpu_fullsize.py): the reference's K-layer chain evaluated in
 * float64 on the host from the SAME u0 / i0 the GPU starts from, every layer
 * of it, instead of per product from the GPU's own previous layer.
 *
 *   oracle_csr_perm   stable counting sort of an edge list by one endpoint:
 *                     indptr[n_rows+1] (int64) and perm[E] (int64, input edge
 *                     of each CSR slot, ascending within a row). The caller
 *                     gathers columns and fp32 operator values through perm
 *                     (oracle/ref_numpy.edge_weights: the reference's weight
 *                     expressions, Version-2/lighgcn_cu_pop.py:430-450,
 *                     lightgcn_cu.py:383-397).
 *   oracle_spmm64     y[r] = a*add[r] + sum_e w[e] * x[col[e]]  (float64; w fp32
 *                     values widened), then acc[r] += y[r] when acc is given.
 *                     One torch.sparse.mm of the reference's propagate loop
 *                     (Version-2/lighgcn_cu_pop.py:483-484, lightgcn_cu.py:431,
 *                     434) or of its autograd adjoint (backward_gs/_j of
 *                     oracle/ref_numpy.py), with the layer-mean accumulation
 *                     (:488-489) fused. Rows in parallel (OpenMP), each row's
 *                     sum in CSR order: deterministic for any thread count.
 *
 * Coalesce semantics: duplicate (row, col) pairs stay separate CSR entries;
 * their float64 sum equals the coalesced value to float64 rounding (the
 * synthetic C3-C5 graphs have unique pairs anyway).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int oracle_csr_perm(int64_t E, const int32_t *rows, int64_t n_rows, int64_t *indptr,
                    int64_t *perm) {
  memset(indptr, 0, sizeof(int64_t) * (size_t)(n_rows + 1));
  for (int64_t e = 0; e < E; ++e) {
    const int64_t r = rows[e];
    if (r < 0 || r >= n_rows) return -1;
    indptr[r + 1]++;
  }
  for (int64_t r = 0; r < n_rows; ++r) indptr[r + 1] += indptr[r];
  int64_t *next = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n_rows > 0 ? n_rows : 1));
  if (!next) return -2;
  memcpy(next, indptr, sizeof(int64_t) * (size_t)n_rows);
  for (int64_t e = 0; e < E; ++e) perm[next[rows[e]]++] = e;   /* stable */
  free(next);
  return 0;
}

void oracle_spmm64(int64_t n_rows, const int64_t *indptr, const int32_t *cols,
                   const float *w, const double *x, int64_t ldx, int32_t d, double *y,
                   int64_t ldy, const double *add, int64_t ldadd, double add_scale,
                   double *acc, int64_t ldacc) {
#pragma omp parallel
  {
    double *row = (double *)malloc(sizeof(double) * (size_t)d);
#pragma omp for schedule(dynamic, 256)
    for (int64_t r = 0; r < n_rows; ++r) {
      if (add) {
        const double *a = add + r * ldadd;
        for (int j = 0; j < d; ++j) row[j] = add_scale * a[j];
      } else {
        for (int j = 0; j < d; ++j) row[j] = 0.0;
      }
      for (int64_t e = indptr[r]; e < indptr[r + 1]; ++e) {
        const double we = (double)w[e];
        const double *xs = x + (int64_t)cols[e] * ldx;
        for (int j = 0; j < d; ++j) row[j] += we * xs[j];
      }
      if (y) memcpy(y + r * ldy, row, sizeof(double) * (size_t)d);
      if (acc) {
        double *ac = acc + r * ldacc;
        for (int j = 0; j < d; ++j) ac[j] += row[j];
      }
    }
    free(row);
  }
}
