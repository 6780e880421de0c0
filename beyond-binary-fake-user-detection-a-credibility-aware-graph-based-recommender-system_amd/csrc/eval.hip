// Sampled evaluation: Version-2/lighgcn_cu_pop.py:536-650.
//
// Per evaluated user (one 16-lane group): draw pos uniformly from the user's
// test row; draw n_neg negatives uniformly from [0, I) rejecting test items and
// train items (binary searches in the sorted CSR rows), duplicates allowed as
// in the reference; score the 1+n_neg candidates against the user's final
// embedding; rank them by score descending, ties broken by candidate order
// (stable); write the positive's rank and the top-k_max candidate items.
// A second kernel turns ranks / top-k lists into per-user metric terms for
// each K; a single-workgroup fixed-order reduction sums them.
#include "common.h"

namespace bbgr {

constexpr int EVAL_MAX_CAND = 256;   // 1 + n_neg
constexpr int EVAL_MAX_K = 64;
constexpr int EVAL_NSTAT = 6;        // p, r, ndcg, logpop, selfinfo, hit (group recall)

struct EvalParams {
  long n_users;
  const long *users;
  const int *te_indptr, *te_indices;
  const int *tr_indptr, *tr_indices;
  const float *uf, *itf;
  long lduf, ldif;
  int n_items, n_neg, k_max;
  unsigned long long seed, counter;
  int *pos_rank;
  int *topk;
  int *cand_out;
  int *fail_count;
};

__device__ __forceinline__ bool sorted_has(const int *a, int b, int e, int x) {
  int lo = b, hi = e;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo < e && a[lo] == x;
}

__device__ __forceinline__ float group16_sum_e(float v) {
  v += __shfl_xor(v, 1, 16);
  v += __shfl_xor(v, 2, 16);
  v += __shfl_xor(v, 4, 16);
  v += __shfl_xor(v, 8, 16);
  return v;
}

template <int D>
__global__ __launch_bounds__(256) void eval_sampled_kernel(EvalParams P) {
  constexpr int V = D / 64;
  __shared__ int cand[16][EVAL_MAX_CAND];
  __shared__ float score[16][EVAL_MAX_CAND];
  const int g = threadIdx.x >> 4;
  const int lane = threadIdx.x & 15;
  const long b = (long)blockIdx.x * 16 + g;
  const bool active = b < P.n_users;
  const int nc = 1 + P.n_neg;
  long u = 0;
  int tb = 0, te = 0, rb = 0, re = 0;
  if (active) {
    u = P.users[b];
    tb = P.te_indptr[u];
    te = P.te_indptr[u + 1];
    rb = P.tr_indptr[u];
    re = P.tr_indptr[u + 1];
  }
  // ---- candidates: lane 0 of each group draws pos; lanes split the negatives
  if (active && te > tb) {
    const uint32_t k0 = (uint32_t)P.seed, k1 = (uint32_t)(P.seed >> 32) ^ 0x2545F491u;
    const uint32_t c1 = (uint32_t)b, c2 = (uint32_t)P.counter;
    const uint32_t c3 = (uint32_t)(P.counter >> 32) ^ (uint32_t)((unsigned long long)b >> 32);
    if (lane == 0) {
      const u32x4 r = philox4x32_10(u32x4{0xFFFFFFFFu, c1, c2, c3}, k0, k1);
      int j = (int)(u01_53(r.x, r.y) * (double)(te - tb));
      if (j >= te - tb) j = te - tb - 1;
      cand[g][0] = P.te_indices[tb + j];
    }
    // negative slot s (1..n_neg) is drawn by lane (s-1) % 16 from its own stream
    for (int s = 1 + lane; s < nc; s += 16) {
      int j = -1;
      for (uint32_t draw = 0; draw < (uint32_t)BBGR_NEG_CAP; ++draw) {
        const u32x4 r = philox4x32_10(u32x4{draw, c1, c2 ^ ((uint32_t)s << 16), c3}, k0, k1);
        int x = (int)(u01_53(r.x, r.y) * (double)P.n_items);
        if (x >= P.n_items) x = P.n_items - 1;
        if (sorted_has(P.te_indices, tb, te, x)) continue;     // j in gt_set
        if (sorted_has(P.tr_indices, rb, re, x)) continue;     // user_has_item
        j = x;
        break;
      }
      if (j < 0 && P.fail_count) atomicAdd(P.fail_count, 1);
      cand[g][s] = j;
    }
  }
  __syncthreads();
  const bool work = active && te > tb;   // no early return: every thread reaches each barrier
  if (active && !work && lane == 0) P.pos_rank[b] = -1;   // no test items: not evaluated
  // ---- scores: each lane holds float4 columns of the user row
  float4 fu[V];
  const float4 *pu = reinterpret_cast<const float4 *>(P.uf + u * P.lduf) + lane;
#pragma unroll
  for (int k = 0; k < V; ++k) fu[k] = work ? pu[16 * k] : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int c = 0; work && c < nc; ++c) {
    const int it = cand[g][c];
    float s = -INFINITY;
    if (it >= 0) {
      const float4 *pi = reinterpret_cast<const float4 *>(P.itf + (long)it * P.ldif) + lane;
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const float4 x = pi[16 * k];
        a += fu[k].x * x.x + fu[k].y * x.y + fu[k].z * x.z + fu[k].w * x.w;
      }
      s = group16_sum_e(a);
    }
    if (lane == 0) score[g][c] = s;
  }
  __syncthreads();
  // ---- stable descending rank of every candidate; top-k list and pos rank
  for (int c = lane; work && c < nc; c += 16) {
    const float sc = score[g][c];
    int rank = 0;
    for (int o = 0; o < nc; ++o) {
      const float so = score[g][o];
      rank += (so > sc) || (so == sc && o < c);
    }
    if (c == 0) P.pos_rank[b] = rank;
    if (rank < P.k_max) P.topk[b * P.k_max + rank] = cand[g][c];
    if (P.cand_out) P.cand_out[b * nc + c] = cand[g][c];
  }
}

struct EvalStatParams {
  long n_users;
  const long *users;
  const int *te_indptr;
  const int *pos_rank;
  const int *topk;
  int k_max;
  int n_k;
  int ks[8];
  const float *item_pop;       // train popularity counts (float)
  float self_info_denom;       // total_train + n_items
  const unsigned char *group;  // per evaluated user: bit0 high, bit1 low (nullable)
  float *stats;                // [n_users][n_k][EVAL_NSTAT]
  unsigned char *covered;      // [n_k][n_items] bytes
  int n_items;
};

// Per user and K: precision, recall, ndcg (metrics_at_k with gt = {pos}),
// novelty (avg log(pop+1), avg -log2((pop+1)/(total+I))), hit for groups.
__global__ void eval_stats_kernel(EvalStatParams P) {
  const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= P.n_users) return;
  float *st = P.stats + b * (long)P.n_k * EVAL_NSTAT;
  const int rank = P.pos_rank[b];
  for (int q = 0; q < P.n_k; ++q) {
    float *o = st + q * EVAL_NSTAT;
    if (rank < 0) {
      for (int z = 0; z < EVAL_NSTAT; ++z) o[z] = 0.f;
      continue;
    }
    const int K = P.ks[q];
    const bool hit = rank < K;
    float lp = 0.f, si = 0.f;
    for (int j = 0; j < K; ++j) {
      const int it = P.topk[b * P.k_max + j];
      if (it < 0) continue;
      const float pop = P.item_pop[it];
      lp += logf(pop + 1.0f);
      si += -log2f((pop + 1.0f) / P.self_info_denom);
      P.covered[(long)q * P.n_items + it] = 1;
    }
    o[0] = hit ? 1.0f / (float)K : 0.f;
    o[1] = hit ? 1.0f : 0.f;
    o[2] = hit ? 1.0f / log2f((float)rank + 2.0f) : 0.f;
    o[3] = lp / (float)K;
    o[4] = si / (float)K;
    o[5] = hit ? 1.0f : 0.f;
  }
}

// sums[q][z] over users (+ group sums and counts), fixed order -> deterministic.
// Output layout per K: [p, r, ndcg, logpop, selfinfo, high_r, low_r, high_n, low_n, n, cov]
constexpr int EVAL_NOUT = 11;

__global__ __launch_bounds__(256) void eval_reduce_kernel(EvalStatParams P, float *out) {
  __shared__ double red[256];
  const int q = blockIdx.x / EVAL_NOUT;
  const int z = blockIdx.x % EVAL_NOUT;
  double acc = 0.0;
  if (z < 5) {
    for (long b = threadIdx.x; b < P.n_users; b += 256)
      acc += P.stats[(b * P.n_k + q) * EVAL_NSTAT + z];
  } else if (z <= 8) {
    const int bit = (z == 5 || z == 7) ? 1 : 2;
    for (long b = threadIdx.x; b < P.n_users; b += 256) {
      if (P.pos_rank[b] < 0 || !P.group || !(P.group[b] & bit)) continue;
      acc += (z <= 6) ? P.stats[(b * P.n_k + q) * EVAL_NSTAT + 5] : 1.0;
    }
  } else if (z == 9) {
    for (long b = threadIdx.x; b < P.n_users; b += 256) acc += P.pos_rank[b] >= 0 ? 1.0 : 0.0;
  } else {
    for (long i = threadIdx.x; i < P.n_items; i += 256) acc += P.covered[(long)q * P.n_items + i];
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[q * EVAL_NOUT + z] = (float)red[0];
}

}  // namespace bbgr

using namespace bbgr;

extern "C" int bbgr_eval_sampled(const bbgr_eval_args *a, bbgr_stream_t stream) {
  BBGR_REQUIRE(a, "bbgr_eval_sampled: null args");
  BBGR_REQUIRE(a->n_users >= 0 && a->n_items > 0 && a->n_neg >= 0 &&
                   1 + a->n_neg <= EVAL_MAX_CAND && a->k_max > 0 && a->k_max <= EVAL_MAX_K &&
                   a->n_k > 0 && a->n_k <= 8,
               "bbgr_eval_sampled: sizes out of range (1+n_neg <= 256, k_max <= 64, n_k <= 8)");
  const int d = a->d;
  if (d != 64 && d != 128 && d != 256) {
    set_error("bbgr_eval_sampled: embedding dim %d unsupported (64, 128, 256)", d);
    return BBGR_ERR_UNSUPPORTED;
  }
  if (a->n_users == 0) return BBGR_OK;
  BBGR_REQUIRE(a->users && a->te_indptr && a->te_indices && a->tr_indptr && a->tr_indices &&
                   a->uf && a->itf && a->pos_rank && a->topk && a->stats && a->covered &&
                   a->item_pop && a->sums,
               "bbgr_eval_sampled: null array");
  BBGR_REQUIRE(aligned16(a->uf) && aligned16(a->itf) && (a->lduf & 3) == 0 && (a->ldif & 3) == 0,
               "bbgr_eval_sampled: tables must be 16-byte aligned, ld % 4 == 0");
  for (int q = 0; q < a->n_k; ++q)
    BBGR_REQUIRE(a->ks[q] > 0 && a->ks[q] <= a->k_max, "bbgr_eval_sampled: K > k_max");
  hipStream_t st = as_stream(stream);
  EvalParams P;
  P.n_users = a->n_users;
  P.users = (const long *)a->users;
  P.te_indptr = a->te_indptr;
  P.te_indices = a->te_indices;
  P.tr_indptr = a->tr_indptr;
  P.tr_indices = a->tr_indices;
  P.uf = a->uf;
  P.itf = a->itf;
  P.lduf = a->lduf;
  P.ldif = a->ldif;
  P.n_items = a->n_items;
  P.n_neg = a->n_neg;
  P.k_max = a->k_max;
  P.seed = a->seed;
  P.counter = a->counter;
  P.pos_rank = a->pos_rank;
  P.topk = a->topk;
  P.cand_out = a->cand_out;
  P.fail_count = a->fail_count;
  BBGR_HIP(hipMemsetAsync(a->topk, 0xff, sizeof(int) * (size_t)a->n_users * a->k_max, st));
  const unsigned grid = (unsigned)((a->n_users + 15) / 16);
  switch (d) {
    case 64: hipLaunchKernelGGL(eval_sampled_kernel<64>, dim3(grid), dim3(256), 0, st, P); break;
    case 128: hipLaunchKernelGGL(eval_sampled_kernel<128>, dim3(grid), dim3(256), 0, st, P); break;
    default: hipLaunchKernelGGL(eval_sampled_kernel<256>, dim3(grid), dim3(256), 0, st, P); break;
  }
  BBGR_LAUNCHED("eval_sampled_kernel");
  EvalStatParams S;
  S.n_users = a->n_users;
  S.users = (const long *)a->users;
  S.te_indptr = a->te_indptr;
  S.pos_rank = a->pos_rank;
  S.topk = a->topk;
  S.k_max = a->k_max;
  S.n_k = a->n_k;
  for (int q = 0; q < 8; ++q) S.ks[q] = q < a->n_k ? a->ks[q] : 0;
  S.item_pop = a->item_pop;
  S.self_info_denom = a->self_info_denom;
  S.group = a->group;
  S.stats = a->stats;
  S.covered = a->covered;
  S.n_items = a->n_items;
  BBGR_HIP(hipMemsetAsync(a->covered, 0, (size_t)a->n_k * a->n_items, st));
  hipLaunchKernelGGL(eval_stats_kernel, dim3((unsigned)((a->n_users + 255) / 256)), dim3(256), 0,
                     st, S);
  BBGR_LAUNCHED("eval_stats_kernel");
  hipLaunchKernelGGL(eval_reduce_kernel, dim3((unsigned)(a->n_k * EVAL_NOUT)), dim3(256), 0, st,
                     S, a->sums);
  BBGR_LAUNCHED("eval_reduce_kernel");
  return BBGR_OK;
}
