/* ORACLE — test infrastructure, NOT product code.
 *
 * Full-ranking top-K restatement of evaluate_full_ranking
 * (Version-2/lighgcn_cu_pop.py:690-706): for each evaluated user u,
 *   scores = (uvec * item_emb).sum(1)            (:697)
 *   scores[train_items(u)] = -1e9                (:699-703)
 *   ranked = argsort(scores, descending=True)    (:705)
 * and the top-k of `ranked`. Ties (unspecified in torch.argsort) are broken by
 * item id ascending. The score is restated as the device computes it: one
 * fp32 fma chain per (user, item) over the components in the order
 * 0, d/2, 1, d/2+1, ... (the k order of v_mfma_f32_32x32x2_f32 with lane half
 * h holding components h*d/2 + s), so the device top-k and its scores are
 * compared BIT-exactly. The reference's own summation order (elementwise
 * product, then torch's reduction tree) differs by ulps; tests/test_oracle.py
 * checks this chain against float64 to fp32 rounding.
 * Built by oracle/Makefile with -ffp-contract=off (fmaf only where written).
 */
#include <math.h>
#include <stdint.h>

static int has_item(const int32_t *a, int32_t n, int32_t x) {
  int32_t lo = 0, hi = n;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo < n && a[lo] == x;
}

float oracle_score_chain(const float *a, const float *b, int32_t d) {
  float acc = 0.0f;
  const int32_t h = d / 2;
  for (int32_t s = 0; s < h; ++s) {
    acc = fmaf(a[s], b[s], acc);
    acc = fmaf(a[h + s], b[h + s], acc);
  }
  return acc;
}

void oracle_full_topk(int64_t n_users, const int64_t *users, const int32_t *tr_indptr,
                      const int32_t *tr_indices, const float *uf, int64_t lduf,
                      const float *itf, int64_t ldif, int32_t d, int32_t n_items, int32_t k,
                      int32_t *topk, float *topk_score) {
  for (int64_t b = 0; b < n_users; ++b) {
    const int64_t u = users[b];
    const int32_t rb = tr_indptr[u], re = tr_indptr[u + 1];
    float *tv = topk_score + b * k;
    int32_t *ti = topk + b * k;
    for (int32_t j = 0; j < k; ++j) {
      tv[j] = -INFINITY;
      ti[j] = -1;
    }
    int32_t filled = 0;
    for (int32_t i = 0; i < n_items; ++i) {
      float s = oracle_score_chain(uf + u * lduf, itf + (int64_t)i * ldif, d);
      if (has_item(tr_indices + rb, re - rb, i)) s = -1e9f;
      /* (score desc, item asc): i is larger than every id already held */
      if (filled == k && !(s > tv[k - 1])) continue;
      int32_t p = filled < k ? filled++ : k - 1;
      while (p > 0 && s > tv[p - 1]) {
        tv[p] = tv[p - 1];
        ti[p] = ti[p - 1];
        --p;
      }
      tv[p] = s;
      ti[p] = i;
    }
  }
}
