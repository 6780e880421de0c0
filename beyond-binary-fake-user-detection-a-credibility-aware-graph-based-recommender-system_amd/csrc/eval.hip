// Evaluation.
//
// Sampled protocol, Version-2/lighgcn_cu_pop.py:536-650: per evaluated user
// (one 16-lane group) draw pos uniformly from the test row, draw n_neg
// negatives uniformly from [0, I) rejecting test items and train items
// (binary searches in the sorted CSR rows, LDS copies of short rows),
// duplicates allowed as in the reference; score the 1+n_neg candidates; rank
// them by score descending, ties in candidate order; write the positive's rank
// and the top-k_max candidate items.
//
// Full-ranking protocol, :652-752: every item is scored for every evaluated
// user. That is a U_eval x I x d product: fp32 MFMA (v_mfma_f32_32x32x2_f32,
// exact fp32 fma chains) over LDS-staged 128-item tiles, 256 users per
// workgroup (32 per wave, the user fragment kept in registers for the whole
// sweep). The reference's `scores[train] = -1e9; argsort` is fused: every lane
// keeps the running top-KM of the items it owns in registers (score desc,
// item asc), gated by a per-sub-tile max so almost every tile costs one
// compare; train items are masked on the (rare) insertion path by a monotone
// pointer into the user's sorted train row. While a lane's list has empty
// slots its threshold is -inf, so every item (train items at -1e9 included)
// enters; once full, a raw score at or below the threshold cannot enter
// masked either. A merge kernel combines the per-lane lists (two lane halves
// x item splits) into the user's top-k_max.
//
// Metrics (both protocols): eval_terms_kernel turns ranks / top-K lists into
// per-user P/R/NDCG/novelty/group terms, marks covered items and reduces a
// fixed chunk of users per workgroup; eval_sum_kernel sums the chunks in a
// fixed order and counts covered items. Deterministic bit for bit.
#include <algorithm>
#include <vector>

#include "common.h"

namespace bbgr {

constexpr int EVAL_MAX_CAND = 256;   // 1 + n_neg
constexpr int EVAL_MAX_K = 64;       // sampled k_max
constexpr int EVAL_FULL_MAX_K = 32;  // full-ranking k_max
constexpr int EVAL_NTERM = 10;       // p, r, ndcg, logpop, selfinfo, high_r, low_r, high_n, low_n, n
constexpr int EVAL_NOUT = 11;        // + covered count
constexpr int EVAL_CHUNK = 4096;     // users per eval_terms workgroup (256 threads x 16)
constexpr int ROW_CACHE = 64;        // LDS copy of test / train rows up to this length
constexpr int FULL_THREADS = 512;    // 8 waves: 2 per SIMD hide the check path
constexpr int FULL_USERS = 256;      // users per full-ranking workgroup (8 waves x 32)
constexpr int FULL_TILE = 128;       // items per full-ranking LDS tile
constexpr long FULL_BATCH = 1l << 18;  // users per full-ranking launch
constexpr float TRAIN_MASK = -1e9f;  // Version-2:703 scores[train_items] = -1e9

__device__ __forceinline__ int lower_bound_i32(const int *a, int n, int x) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ bool sorted_has(const int *a, int n, int x) {
  const int lo = lower_bound_i32(a, n, x);
  return lo < n && a[lo] == x;
}

__device__ __forceinline__ float group16_sum_e(float v) {
  v += __shfl_xor(v, 1, 16);
  v += __shfl_xor(v, 2, 16);
  v += __shfl_xor(v, 4, 16);
  v += __shfl_xor(v, 8, 16);
  return v;
}

// ===========================================================================
// Sampled protocol
// ===========================================================================
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
  const int *cand_in;   // candidates supplied (the reference's numpy stream) instead of drawn
};

// MC: LDS candidate capacity per user (128 covers the reference's 1 + 99;
// 256 the ABI maximum). The arrays dominate the workgroup's LDS, so the small
// form fits 6 workgroups per CU instead of 4 (more gathers in flight).
template <int D, int MC>
__global__ __launch_bounds__(256) void eval_sampled_kernel(EvalParams P) {
  constexpr int V = D / 64;
  __shared__ int cand[16][MC];
  __shared__ float score[16][MC];
  __shared__ int rows[16][2][ROW_CACHE];
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
  const int nte = te - tb, ntr = re - rb;
  const bool te_lds = nte <= ROW_CACHE, tr_lds = ntr <= ROW_CACHE;
  for (int j = lane; te_lds && j < nte; j += 16) rows[g][0][j] = P.te_indices[tb + j];
  for (int j = lane; tr_lds && j < ntr; j += 16) rows[g][1][j] = P.tr_indices[rb + j];
  __syncthreads();
  const int *te_row = te_lds ? rows[g][0] : P.te_indices + tb;
  const int *tr_row = tr_lds ? rows[g][1] : P.tr_indices + rb;
  // ---- candidates: supplied (cand_in), or lane 0 of each group draws pos and
  // the lanes split the negatives
  if (active && nte > 0 && P.cand_in) {
    for (int c = lane; c < nc; c += 16) cand[g][c] = P.cand_in[b * nc + c];
  } else if (active && nte > 0) {
    const uint32_t k0 = (uint32_t)P.seed, k1 = (uint32_t)(P.seed >> 32) ^ 0x2545F491u;
    const uint32_t c1 = (uint32_t)b, c2 = (uint32_t)P.counter;
    const uint32_t c3 = (uint32_t)(P.counter >> 32) ^ (uint32_t)((unsigned long long)b >> 32);
    if (lane == 0) {
      const u32x4 r = philox4x32_10(u32x4{0xFFFFFFFFu, c1, c2, c3}, k0, k1);
      int j = (int)(u01_53(r.x, r.y) * (double)nte);
      if (j >= nte) j = nte - 1;
      cand[g][0] = te_row[j];
    }
    // negative slot s (1..n_neg) is drawn by lane (s-1) % 16 from its own stream
    for (int s = 1 + lane; s < nc; s += 16) {
      int j = -1;
      for (uint32_t draw = 0; draw < (uint32_t)BBGR_NEG_CAP; ++draw) {
        const u32x4 r = philox4x32_10(u32x4{draw, c1, c2 ^ ((uint32_t)s << 16), c3}, k0, k1);
        int x = (int)(u01_53(r.x, r.y) * (double)P.n_items);
        if (x >= P.n_items) x = P.n_items - 1;
        if (sorted_has(te_row, nte, x)) continue;     // j in gt_set
        if (sorted_has(tr_row, ntr, x)) continue;     // user_has_item
        j = x;
        break;
      }
      if (j < 0 && P.fail_count) atomicAdd(P.fail_count, 1);
      cand[g][s] = j;
    }
  }
  __syncthreads();
  const bool work = active && nte > 0;   // no early return: every thread reaches each barrier
  if (active && !work && lane == 0) P.pos_rank[b] = -1;   // no test items: not evaluated
  // ---- scores: each lane holds float4 columns of the user row; CF candidate
  // rows in flight per group (each score is its own dot product: the batching
  // does not change any result)
  constexpr int CF = D == 64 ? 8 : 4;
  float4 fu[V];
  const float4 *pu = reinterpret_cast<const float4 *>(P.uf + u * P.lduf) + lane;
#pragma unroll
  for (int k = 0; k < V; ++k) fu[k] = work ? pu[16 * k] : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int c0 = 0; work && c0 < nc; c0 += CF) {
    int it[CF];
    float4 x[CF][V];
#pragma unroll
    for (int q = 0; q < CF; ++q) {
      it[q] = c0 + q < nc ? cand[g][c0 + q] : -1;
      const float4 *pi =
          reinterpret_cast<const float4 *>(P.itf + (long)(it[q] < 0 ? 0 : it[q]) * P.ldif) + lane;
#pragma unroll
      for (int k = 0; k < V; ++k)
        x[q][k] = it[q] >= 0 ? pi[16 * k] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < CF; ++q) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < V; ++k)
        a += fu[k].x * x[q][k].x + fu[k].y * x[q][k].y + fu[k].z * x[q][k].z + fu[k].w * x[q][k].w;
      a = group16_sum_e(a);
      if (lane == 0 && c0 + q < nc) score[g][c0 + q] = it[q] >= 0 ? a : -INFINITY;
    }
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

// ===========================================================================
// Full-ranking protocol
// ===========================================================================
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct FullParams {
  long n_users;               // users in this launch
  const long *users;
  const int *tr_indptr, *tr_indices;
  const float *uf, *itf;
  long lduf, ldif;
  int n_items;
  int split_items;            // items per split (multiple of FULL_TILE)
  int n_splits;
  float *list_score;          // [n_users][n_splits][2][KM]
  int *list_item;
};

// One (score, item) into a sorted register list (score desc, item asc).
template <int KM>
__device__ __forceinline__ void topk_insert(float (&tv)[KM], int (&ti)[KM], float s, int it) {
#pragma unroll
  for (int j = 0; j < KM; ++j) {
    const bool sw = s > tv[j] || (s == tv[j] && it < ti[j]);
    const float t = tv[j];
    const int q = ti[j];
    tv[j] = sw ? s : t;
    ti[j] = sw ? it : q;
    s = sw ? t : s;
    it = sw ? q : it;
  }
}

// Items per LDS tile and per-lane candidate buffer depth, per embedding dim
// (LDS: 2 tiles of TILE x (D+4) floats + CB x 512 float2 <= 160 KB).
template <int D> struct FullShape {
  static constexpr int TILE = D == 64 ? 128 : 64;
  static constexpr int CB = 12;
  static constexpr size_t lds_bytes() {
    return sizeof(float) * 2 * TILE * (D + 4) + sizeof(float2) * CB * FULL_THREADS;
  }
};

template <int D, int KM>
__global__ __launch_bounds__(FULL_THREADS) void eval_full_kernel(FullParams P) {
  constexpr int TILE = FullShape<D>::TILE;
  constexpr int CB = FullShape<D>::CB;
  constexpr int M = TILE / 32;        // 32-item sub-tiles (one accumulator each)
  constexpr int LDT = D + 4;          // padded LDS row (conflict-free b128 reads)
  constexpr int H = D / 2;            // components per lane half
  constexpr int F4 = TILE * D / 4 / FULL_THREADS;   // float4 per thread per tile
  extern __shared__ float smem[];
  float *tile = smem;                                                  // [2][TILE][LDT]
  float2 *cbuf = reinterpret_cast<float2 *>(smem + 2 * TILE * LDT);   // [CB][FULL_THREADS]
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, h = l >> 5;
  const long b = (long)blockIdx.x * FULL_USERS + w * 32 + r;
  const bool valid = b < P.n_users;
  const long u = valid ? P.users[b] : 0;
  const int split = blockIdx.y;
  const int item_lo = split * P.split_items;
  const int item_hi = min(P.n_items, item_lo + P.split_items);
  // user fragment: component h*H + s of user u, for s = 0..H-1
  float ub[H];
  {
    const float4 *pu = reinterpret_cast<const float4 *>(P.uf + u * P.lduf + h * H);
#pragma unroll
    for (int s = 0; s < H / 4; ++s) {
      const float4 v = valid ? pu[s] : make_float4(0.f, 0.f, 0.f, 0.f);
      ub[4 * s] = v.x;
      ub[4 * s + 1] = v.y;
      ub[4 * s + 2] = v.z;
      ub[4 * s + 3] = v.w;
    }
  }
  // train row pointer (monotone; starts at the first train item >= item_lo)
  int tp = 0, tend = 0, nt = INT_MAX;
  if (valid) {
    const int rb = P.tr_indptr[u], re = P.tr_indptr[u + 1];
    tp = rb + lower_bound_i32(P.tr_indices + rb, re - rb, item_lo);
    tend = re;
    nt = tp < tend ? P.tr_indices[tp] : INT_MAX;
  }
  float tv[KM];
  int ti[KM];
#pragma unroll
  for (int j = 0; j < KM; ++j) {
    tv[j] = -INFINITY;
    ti[j] = INT_MAX;
  }
  // Candidates whose raw score beats the (possibly stale) threshold are
  // appended to the lane's LDS buffer in ascending item order; a flush
  // inserts every lane's buffer at once, so the compare-swap insertion runs
  // SIMD-parallel instead of once per passing lane.
  int cnt = 0;
  // (+inf for a lane without a user: nothing ever passes its threshold)
  float thr = valid ? -INFINITY : INFINITY;
  auto flush = [&]() {
    for (int j = 0; j < cnt; ++j) {
      const float2 c = cbuf[j * FULL_THREADS + threadIdx.x];
      float sc = c.x;
      const int it = __float_as_int(c.y);
      if (sc > tv[KM - 1]) {
        while (nt < it) nt = ++tp < tend ? P.tr_indices[tp] : INT_MAX;
        if (nt == it) sc = TRAIN_MASK;
        if (sc > tv[KM - 1]) topk_insert<KM>(tv, ti, sc, it);
      }
    }
    cnt = 0;
    thr = valid ? tv[KM - 1] : INFINITY;
  };
  const int n_tiles = item_hi > item_lo ? (item_hi - item_lo + TILE - 1) / TILE : 0;
  float4 stage[F4];
  auto load_tile = [&](int t) {
    const int i0 = item_lo + t * TILE;
#pragma unroll
    for (int j = 0; j < F4; ++j) {
      const int f = threadIdx.x + FULL_THREADS * j;
      const int row = f / (D / 4), c4 = f % (D / 4);
      const int it = i0 + row;
      stage[j] = it < item_hi ? reinterpret_cast<const float4 *>(P.itf + (long)it * P.ldif)[c4]
                              : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_tile = [&](int buf) {
    float *T = tile + buf * TILE * LDT;
#pragma unroll
    for (int j = 0; j < F4; ++j) {
      const int f = threadIdx.x + FULL_THREADS * j;
      const int row = f / (D / 4), c4 = f % (D / 4);
      *reinterpret_cast<float4 *>(T + row * LDT + 4 * c4) = stage[j];
    }
  };
  // Scores of sub-tiles [lo, hi) of tile T: per sub-tile one chain of H
  // MFMAs over the components in order (the same chain for every tiling).
  // Sub-tiles [plo, phi) (already scored, not written here) have their
  // maxima folded into mxp a few elements per component step, between the
  // MFMAs, so the check's VALU work issues while the matrix pipe is busy.
  f32x16 acc[M];
  float mxp[M];
  constexpr int EPS = 16 / (H / 4);   // max elements folded per component step
  static_assert(EPS >= 1 && EPS * (H / 4) == 16, "the folds must cover the 16 scores");
  auto score_rows = [&](const float *T, int lo, int hi, int plo, int phi) {
#pragma unroll
    for (int m = lo; m < hi; ++m)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[m][e] = 0.f;
#pragma unroll
    for (int m = plo; m < phi; ++m) mxp[m] = acc[m][0];
#pragma unroll
    for (int s4 = 0; s4 < H / 4; ++s4) {
#pragma unroll
      for (int m = plo; m < phi; ++m)
#pragma unroll
        for (int q = 0; q < EPS; ++q)
          if (s4 * EPS + q > 0) mxp[m] = fmaxf(mxp[m], acc[m][s4 * EPS + q]);
      float4 a[M];
#pragma unroll
      for (int m = lo; m < hi; ++m)
        a[m] = *reinterpret_cast<const float4 *>(T + (m * 32 + r) * LDT + h * H + 4 * s4);
      // independent accumulators back to back
#pragma unroll
      for (int m = lo; m < hi; ++m)
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m].x, ub[4 * s4 + 0], acc[m], 0, 0, 0);
#pragma unroll
      for (int m = lo; m < hi; ++m)
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m].y, ub[4 * s4 + 1], acc[m], 0, 0, 0);
#pragma unroll
      for (int m = lo; m < hi; ++m)
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m].z, ub[4 * s4 + 2], acc[m], 0, 0, 0);
#pragma unroll
      for (int m = lo; m < hi; ++m)
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m].w, ub[4 * s4 + 3], acc[m], 0, 0, 0);
    }
  };
  // Sub-tile m's scores against the threshold; acc[m][e] = score of user b,
  // item i0 + 32m + (e&3) + 8(e>>2) + 4h.
  auto scan = [&](int m, int i0, bool folded) {
    float mx = acc[m][0];
    if (folded) {
      mx = mxp[m];
    } else {
#pragma unroll
      for (int e = 1; e < 16; ++e) mx = fmaxf(mx, acc[m][e]);
    }
    if (mx > thr) {
      unsigned pass = 0;
#pragma unroll
      for (int e = 0; e < 16; ++e) pass |= (acc[m][e] > thr ? 1u : 0u) << e;
      while (pass) {
        const int e = __builtin_ctz(pass);
        pass &= pass - 1;
        float sc = acc[m][0];
#pragma unroll
        for (int e2 = 1; e2 < 16; ++e2) sc = e2 == e ? acc[m][e2] : sc;
        const int it = i0 + 32 * m + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (it < item_hi) {
          if (cnt == CB) flush();      // this lane only (early tiles: all lanes together)
          cbuf[cnt * FULL_THREADS + threadIdx.x] = make_float2(sc, __int_as_float(it));
          ++cnt;
        }
      }
    }
    if (__any(cnt > CB - 4)) flush();   // batch the insertions across lanes
  };
  if (n_tiles > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();
  // Software pipeline (KM <= 24): the second half of tile t-1's sub-tiles is
  // checked while the first half of tile t is on the MFMA pipe, the first
  // half of tile t while its second half is. Candidates still reach each
  // lane's buffer in ascending item order. (Before the first tile the pending
  // half holds -inf scores: nothing passes.) The 32-deep list leaves no
  // registers for it and checks each tile after its MFMAs.
  if constexpr (KM <= 24) {
    constexpr int M2 = M / 2;
#pragma unroll
    for (int m = M2; m < M; ++m)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[m][e] = -INFINITY;
    int i_prev = item_lo;
    for (int t = 0; t < n_tiles; ++t) {
      if (t + 1 < n_tiles) load_tile(t + 1);
      const float *T = tile + (t & 1) * TILE * LDT;
      const int i0 = item_lo + t * TILE;
      score_rows(T, 0, M2, M2, M);
#pragma unroll
      for (int m = M2; m < M; ++m) scan(m, i_prev, true);
      score_rows(T, M2, M, 0, M2);
#pragma unroll
      for (int m = 0; m < M2; ++m) scan(m, i0, true);
      i_prev = i0;
      if (t + 1 < n_tiles) store_tile((t + 1) & 1);
      __syncthreads();
    }
#pragma unroll
    for (int m = M2; m < M; ++m) scan(m, i_prev, false);
  } else {
    for (int t = 0; t < n_tiles; ++t) {
      if (t + 1 < n_tiles) load_tile(t + 1);
      const float *T = tile + (t & 1) * TILE * LDT;
      score_rows(T, 0, M, 0, 0);
      const int i0 = item_lo + t * TILE;
#pragma unroll
      for (int m = 0; m < M; ++m) scan(m, i0, false);
      if (t + 1 < n_tiles) store_tile((t + 1) & 1);
      __syncthreads();
    }
  }
  flush();
  if (valid) {
    const long o = ((b * P.n_splits + split) * 2 + h) * KM;
#pragma unroll
    for (int j = 0; j < KM; ++j) {
      P.list_score[o + j] = tv[j];
      P.list_item[o + j] = ti[j];
    }
  }
}

// Per user (one wave): merge the 2 * n_splits sorted lists into the top-k_max.
template <int KM>
__global__ __launch_bounds__(256) void eval_full_merge_kernel(FullParams P, long b0, int k_max,
                                                              int *topk, float *topk_score) {
  const long b = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = threadIdx.x & 63;
  if (b >= P.n_users) return;   // wave-uniform
  const int L = 2 * P.n_splits;
  const long base = b * L * KM;
  int p = 0;
  float hs = -INFINITY;
  int hi = INT_MAX;
  if (l < L) {
    hs = P.list_score[base + l * KM];
    hi = P.list_item[base + l * KM];
  }
  for (int k = 0; k < k_max; ++k) {
    float bs = hs;
    int bi = hi, bl = l;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float os = __shfl_xor(bs, o);
      const int oi = __shfl_xor(bi, o);
      const int ol = __shfl_xor(bl, o);
      const bool take = os > bs || (os == bs && (oi < bi || (oi == bi && ol < bl)));
      bs = take ? os : bs;
      bi = take ? oi : bi;
      bl = take ? ol : bl;
    }
    if (l == 0) {
      topk[(b0 + b) * k_max + k] = bi == INT_MAX ? -1 : bi;
      if (topk_score) topk_score[(b0 + b) * k_max + k] = bi == INT_MAX ? -INFINITY : bs;
    }
    if (l == bl) {
      ++p;
      hs = p < KM ? P.list_score[base + l * KM + p] : -INFINITY;
      hi = p < KM ? P.list_item[base + l * KM + p] : INT_MAX;
    }
  }
}

// ===========================================================================
// Metric terms and the deterministic reduction
// ===========================================================================
struct EvalTermParams {
  long n_users;
  int full;                    // 0 sampled (gt = {pos}, pos_rank), 1 full (gt = test row)
  const long *users;
  const int *te_indptr, *te_indices;
  const int *pos_rank;
  const int *topk;
  int k_max;
  int n_k;
  int ks[8];
  const float *item_pop;       // train popularity counts (float)
  float self_info_denom;       // total_train + n_items
  const unsigned char *group;  // per evaluated user: bit0 high, bit1 low (nullable)
  unsigned char *covered;      // [n_k][n_items] bytes
  int n_items;
  double *partial;             // [n_k][n_chunks][EVAL_NTERM]
  long n_chunks;
};

// Per user and K: metrics_at_k (Version-2:514-531) with gt = {pos} (sampled)
// or the test row (full); novelty over the top-K (:390-405); group recall.
__global__ __launch_bounds__(256) void eval_terms_kernel(EvalTermParams P) {
  __shared__ double red[256];
  const int q = blockIdx.y;
  const int K = P.ks[q];
  double acc[EVAL_NTERM];
#pragma unroll
  for (int z = 0; z < EVAL_NTERM; ++z) acc[z] = 0.0;
  const long base = (long)blockIdx.x * EVAL_CHUNK;
  for (int j = 0; j < EVAL_CHUNK / 256; ++j) {
    const long b = base + j * 256 + threadIdx.x;
    if (b >= P.n_users) break;
    const long u = P.users[b];
    const int tb = P.te_indptr[u], ng = P.te_indptr[u + 1] - tb;
    int hits = 0;
    double dcg = 0.0, idcg = 0.0, n_gt = 1.0;
    if (P.full) {
      if (ng <= 0) continue;
      int nd_gt = 0;   // |gt_set|: distinct test items (rows are sorted)
      for (int j2 = 0; j2 < ng; ++j2)
        nd_gt += j2 == 0 || P.te_indices[tb + j2] != P.te_indices[tb + j2 - 1];
      n_gt = (double)nd_gt;
      for (int j2 = 0; j2 < K; ++j2) {
        const int it = P.topk[b * P.k_max + j2];
        if (it >= 0 && sorted_has(P.te_indices + tb, ng, it)) {
          ++hits;
          dcg += 1.0 / log2((double)j2 + 2.0);
        }
      }
      for (int j2 = 0; j2 < min((int)n_gt, K); ++j2) idcg += 1.0 / log2((double)j2 + 2.0);
    } else {
      const int rank = P.pos_rank[b];
      if (rank < 0) continue;
      hits = rank < K;                       // gt = {pos}, |gt| = 1
      dcg = hits ? 1.0 / log2((double)rank + 2.0) : 0.0;
      idcg = 1.0;
    }
    const double p = (double)hits / K, r = (double)hits / n_gt;
    const double nd = idcg > 0.0 ? dcg / idcg : 0.0;
    double lp = 0.0, si = 0.0;
    int cnt = 0;
    for (int j2 = 0; j2 < K; ++j2) {
      const int it = P.topk[b * P.k_max + j2];
      if (it < 0) continue;
      const double pop = (double)P.item_pop[it];
      lp += log(pop + 1.0);
      si += -log2((pop + 1.0) / (double)P.self_info_denom);
      P.covered[(long)q * P.n_items + it] = 1;
      ++cnt;
    }
    acc[0] += p;
    acc[1] += r;
    acc[2] += nd;
    acc[3] += cnt ? lp / cnt : 0.0;
    acc[4] += cnt ? si / cnt : 0.0;
    const unsigned char gf = P.group ? P.group[b] : 0;
    if (gf & 1) {
      acc[5] += r;
      acc[7] += 1.0;
    }
    if (gf & 2) {
      acc[6] += r;
      acc[8] += 1.0;
    }
    acc[9] += 1.0;
  }
  for (int z = 0; z < EVAL_NTERM; ++z) {
    red[threadIdx.x] = acc[z];
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
      __syncthreads();
    }
    if (threadIdx.x == 0)
      P.partial[((long)q * P.n_chunks + blockIdx.x) * EVAL_NTERM + z] = red[0];
    __syncthreads();
  }
}

// sums[q][0..9] = fixed-order sum of the chunk partials; sums[q][10] = covered.
__global__ __launch_bounds__(256) void eval_sum_kernel(EvalTermParams P, double *sums) {
  __shared__ double red[256];
  const int q = blockIdx.x;
  for (int z = 0; z <= EVAL_NTERM; ++z) {
    double a = 0.0;
    if (z < EVAL_NTERM) {
      for (long c = threadIdx.x; c < P.n_chunks; c += 256)
        a += P.partial[((long)q * P.n_chunks + c) * EVAL_NTERM + z];
    } else {
      const unsigned char *cv = P.covered + (long)q * P.n_items;
      long cnt = 0;
      for (long i = threadIdx.x; i < P.n_items; i += 256) cnt += cv[i];
      a = (double)cnt;
    }
    red[threadIdx.x] = a;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
      __syncthreads();
    }
    if (threadIdx.x == 0) sums[q * EVAL_NOUT + z] = red[0];
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
static int full_km(int k_max) { return k_max <= 16 ? 16 : (k_max <= 24 ? 24 : 32); }

// Item splits so that small user counts still fill the chip (>= 4 workgroups
// per CU), each split at least 4 tiles, at most 32 (merge: 2 lists per split
// on one wave).
static long full_splits(long n_users, int n_items, int cus) {
  const long blocks = (n_users + FULL_USERS - 1) / FULL_USERS;
  const long want = 4l * cus;
  long s = blocks >= want ? 1 : (want + blocks - 1) / blocks;
  const long max_s = (n_items + FULL_TILE * 4 - 1) / (FULL_TILE * 4);
  s = s > max_s ? max_s : s;
  s = s > 32 ? 32 : s;
  return s < 1 ? 1 : s;
}

struct EvalLayout {
  size_t covered, partial, lscore, litem, total;
  long n_chunks, batch, splits;
  int km;
};

static EvalLayout eval_layout(const bbgr_eval_args *a, bool full, int cus) {
  EvalLayout L{};
  L.n_chunks = (a->n_users + EVAL_CHUNK - 1) / EVAL_CHUNK;
  size_t off = 0;
  L.covered = off;
  off = align_up(off + (size_t)a->n_k * a->n_items);
  L.partial = off;
  off = align_up(off + sizeof(double) * (size_t)a->n_k * (L.n_chunks > 0 ? L.n_chunks : 1) *
                           EVAL_NTERM);
  if (full) {
    L.batch = a->n_users < FULL_BATCH ? a->n_users : FULL_BATCH;
    L.splits = full_splits(L.batch, a->n_items, cus);
    L.km = full_km(a->k_max);
    const size_t n = (size_t)(L.batch > 0 ? L.batch : 1) * L.splits * 2 * L.km;
    L.lscore = off;
    off = align_up(off + sizeof(float) * n);
    L.litem = off;
    off = align_up(off + sizeof(int) * n);
  }
  L.total = off;
  return L;
}

static int device_cus() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0)
      cus = p.multiProcessorCount;
  }
  return cus;
}

static int check_common(const bbgr_eval_args *a, const char *who) {
  if (!a) {
    set_error("%s: null args", who);
    return BBGR_ERR_INVALID;
  }
  if (!(a->n_users >= 0 && a->n_items > 0 && a->k_max > 0 && a->n_k > 0 && a->n_k <= 8)) {
    set_error("%s: sizes out of range (n_items > 0, k_max > 0, 1 <= n_k <= 8)", who);
    return BBGR_ERR_INVALID;
  }
  for (int q = 0; q < a->n_k; ++q)
    if (!(a->ks[q] > 0 && a->ks[q] <= a->k_max)) {
      set_error("%s: ks[%d] = %d not in [1, k_max]", who, q, a->ks[q]);
      return BBGR_ERR_INVALID;
    }
  if (a->n_users > 0 &&
      !(a->users && a->te_indptr && a->te_indices && a->tr_indptr && a->tr_indices && a->uf &&
        a->itf && a->topk && a->item_pop && a->sums)) {
    set_error("%s: null array", who);
    return BBGR_ERR_INVALID;
  }
  if (!(aligned16(a->uf) && aligned16(a->itf) && (a->lduf & 3) == 0 && (a->ldif & 3) == 0)) {
    set_error("%s: tables must be 16-byte aligned, ld %% 4 == 0", who);
    return BBGR_ERR_INVALID;
  }
  return BBGR_OK;
}

static int launch_terms(const bbgr_eval_args *a, bool full, const EvalLayout &L, char *ws,
                        hipStream_t st) {
  EvalTermParams S;
  S.n_users = a->n_users;
  S.full = full ? 1 : 0;
  S.users = (const long *)a->users;
  S.te_indptr = a->te_indptr;
  S.te_indices = a->te_indices;
  S.pos_rank = a->pos_rank;
  S.topk = a->topk;
  S.k_max = a->k_max;
  S.n_k = a->n_k;
  for (int q = 0; q < 8; ++q) S.ks[q] = q < a->n_k ? a->ks[q] : 0;
  S.item_pop = a->item_pop;
  S.self_info_denom = a->self_info_denom;
  S.group = a->group;
  S.covered = reinterpret_cast<unsigned char *>(ws + L.covered);
  S.n_items = a->n_items;
  S.partial = reinterpret_cast<double *>(ws + L.partial);
  S.n_chunks = L.n_chunks;
  BBGR_HIP(hipMemsetAsync(S.covered, 0, (size_t)a->n_k * a->n_items, st));
  if (L.n_chunks > 0) {
    hipLaunchKernelGGL(eval_terms_kernel, dim3((unsigned)L.n_chunks, (unsigned)a->n_k),
                       dim3(256), 0, st, S);
    BBGR_LAUNCHED("eval_terms_kernel");
  }
  hipLaunchKernelGGL(eval_sum_kernel, dim3((unsigned)a->n_k), dim3(256), 0, st, S, a->sums);
  BBGR_LAUNCHED("eval_sum_kernel");
  return BBGR_OK;
}

template <int D, int KM>
static int launch_full(const FullParams &P, hipStream_t st) {
  const size_t lds = FullShape<D>::lds_bytes();
  BBGR_HIP(hipFuncSetAttribute((const void *)eval_full_kernel<D, KM>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const dim3 grid((unsigned)((P.n_users + FULL_USERS - 1) / FULL_USERS), (unsigned)P.n_splits);
  hipLaunchKernelGGL((eval_full_kernel<D, KM>), grid, dim3(FULL_THREADS), lds, st, P);
  BBGR_LAUNCHED("eval_full_kernel");
  return BBGR_OK;
}

template <int KM>
static int launch_merge(const FullParams &P, long b0, const bbgr_eval_args *a, hipStream_t st) {
  const unsigned grid = (unsigned)((P.n_users + 3) / 4);
  hipLaunchKernelGGL(eval_full_merge_kernel<KM>, dim3(grid), dim3(256), 0, st, P, b0, a->k_max,
                     a->topk, a->topk_score);
  BBGR_LAUNCHED("eval_full_merge_kernel");
  return BBGR_OK;
}

// ---------------------------------------------------------------------------
// The reference's candidate stream on the host (bbgr_eval_draw_candidates):
// numpy's PCG64 (XSL-RR 128/64: advance the LCG, then output
// rotr64(hi ^ lo, hi >> 58)), its buffered 32-bit outputs (the low half of a
// 64-bit output first, the high half kept for the next call), and
// Generator.integers' scalar int64 path (random_bounded_uint64_fill with
// Lemire's multiply-and-reject; a range of one value draws nothing).
// ---------------------------------------------------------------------------
typedef unsigned __int128 u128;

struct Pcg64 {
  u128 state, inc;
  bool has32;
  uint32_t buf32;

  uint64_t next64() {
    const u128 mult = ((u128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull;
    state = state * mult + inc;
    const uint64_t x = (uint64_t)(state >> 64) ^ (uint64_t)state;
    const unsigned rot = (unsigned)(state >> 122);
    return (x >> rot) | (x << ((-rot) & 63u));
  }
  uint32_t next32() {
    if (has32) {
      has32 = false;
      return buf32;
    }
    const uint64_t v = next64();
    has32 = true;
    buf32 = (uint32_t)(v >> 32);
    return (uint32_t)v;
  }
  // rng.integers(0, n) for an int64 result, n >= 1: off + a value in [0, rng]
  uint64_t bounded(uint64_t rng) {
    if (rng == 0) return 0;
    if (rng <= 0xFFFFFFFFull) {
      if (rng == 0xFFFFFFFFull) return next32();
      const uint32_t excl = (uint32_t)rng + 1u;
      uint64_t m = (uint64_t)next32() * excl;
      uint32_t left = (uint32_t)m;
      if (left < excl) {
        const uint32_t thr = (UINT32_MAX - (uint32_t)rng) % excl;
        while (left < thr) {
          m = (uint64_t)next32() * excl;
          left = (uint32_t)m;
        }
      }
      return m >> 32;
    }
    if (rng == UINT64_MAX) return next64();
    const uint64_t excl = rng + 1;
    u128 m = (u128)next64() * excl;
    uint64_t left = (uint64_t)m;
    if (left < excl) {
      const uint64_t thr = (UINT64_MAX - rng) % excl;
      while (left < thr) {
        m = (u128)next64() * excl;
        left = (uint64_t)m;
      }
    }
    return (uint64_t)(m >> 64);
  }
};

// np.searchsorted(arr, x) (side='left') exactly as numpy's binary search runs
// it, so user_has_item (Version-2:330-336) agrees even on an unsorted row
static inline bool user_has_item_host(const int64_t *arr, int64_t n, int64_t x) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    if (arr[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo < n && arr[lo] == x;
}

// Membership in a SORTED row without data-dependent branches (a rejection is
// rare, so the searches' branches would mispredict on most draws): the same
// answer as any search of a sorted row, hence as user_has_item's.
static inline bool sorted_contains(const int64_t *a, int64_t n, int64_t x) {
  if (n <= 32) {   // short rows: a fixed-length scan (the trip count is the row's)
    bool f = false;
    for (int64_t k = 0; k < n; ++k) f |= a[k] == x;
    return f;
  }
  const int64_t *base = a;
  while (n > 1) {   // the trip count depends on n only; the step is arithmetic
    const int64_t half = n >> 1;
    base += (int64_t)(base[half - 1] < x) * half;
    n -= half;
  }
  return *base == x;
}

static inline bool is_sorted_row(const int64_t *a, int64_t n) {
  for (int64_t k = 1; k < n; ++k)
    if (a[k] < a[k - 1]) return false;
  return true;
}

}  // namespace bbgr

using namespace bbgr;

extern "C" int bbgr_eval_draw_candidates(bbgr_pcg64 *rng, int64_t n_users, const int64_t *users,
                                         const int64_t *te_indptr, const int64_t *te_indices,
                                         const int64_t *tr_indptr, const int64_t *tr_indices,
                                         int64_t n_items, int32_t n_neg, int32_t *cand) {
  BBGR_REQUIRE(rng && n_users >= 0 && n_items > 0 && n_items <= INT32_MAX && n_neg >= 0,
               "bbgr_eval_draw_candidates: bad sizes (n_items in [1, 2^31), n_neg >= 0)");
  BBGR_REQUIRE(n_users == 0 || (users && te_indptr && te_indices && tr_indptr && tr_indices && cand),
               "bbgr_eval_draw_candidates: null array");
  BBGR_REQUIRE((rng->inc_lo & 1ull) == 1ull, "bbgr_eval_draw_candidates: PCG64 increment must be odd");
  Pcg64 g;
  g.state = ((u128)rng->state_hi << 64) | rng->state_lo;
  g.inc = ((u128)rng->inc_hi << 64) | rng->inc_lo;
  g.has32 = rng->has_uint32 != 0;
  g.buf32 = rng->uinteger;
  const int64_t nc = 1 + (int64_t)n_neg;
  std::vector<int64_t> gt;   // the test row, sorted: `j in gt_set`
  for (int64_t b = 0; b < n_users; ++b) {
    const int64_t u = users[b];
    const int64_t tb = te_indptr[u], te = te_indptr[u + 1];
    const int64_t rb = tr_indptr[u], re = tr_indptr[u + 1];
    if (te <= tb) {
      set_error("bbgr_eval_draw_candidates: user %lld has an empty test row", (long long)u);
      return BBGR_ERR_INVALID;
    }
    gt.assign(te_indices + tb, te_indices + te);
    std::sort(gt.begin(), gt.end());
    const int64_t *tr = tr_indices + rb;
    const int64_t ntr = re - rb;
    // a sorted train row (edges_to_user_csr sorts every row) is searched
    // without branches; any other row exactly as numpy's searchsorted runs
    const bool tr_sorted = is_sorted_row(tr, ntr);
    const int64_t *gtp = gt.data();
    const int64_t ngt = (int64_t)gt.size();
    // the reference's while loop ends only if some item passes both tests: each
    // row rejects at most its own values, so a shortfall needs an exact count
    if ((te - tb) + ntr >= n_items) {
      bool any = false;
      for (int64_t j = 0; j < n_items && !any; ++j)
        any = !std::binary_search(gt.begin(), gt.end(), j) && !user_has_item_host(tr, ntr, j);
      if (!any && n_neg > 0) {
        set_error("bbgr_eval_draw_candidates: user %lld has no admissible negative item",
                  (long long)u);
        return BBGR_ERR_INVALID;
      }
    }
    int32_t *out = cand + b * nc;
    out[0] = (int32_t)te_indices[tb + (int64_t)g.bounded((uint64_t)(te - tb - 1))];
    for (int64_t s = 1; s < nc;) {
      const int64_t j = (int64_t)g.bounded((uint64_t)(n_items - 1));
      if (sorted_contains(gtp, ngt, j)) continue;   // j in gt_set
      if (tr_sorted ? sorted_contains(tr, ntr, j) : user_has_item_host(tr, ntr, j)) continue;
      out[s++] = (int32_t)j;
    }
  }
  rng->state_hi = (uint64_t)(g.state >> 64);
  rng->state_lo = (uint64_t)g.state;
  rng->has_uint32 = g.has32 ? 1 : 0;
  rng->uinteger = g.buf32;
  return BBGR_OK;
}

extern "C" int bbgr_eval_sampled(const bbgr_eval_args *a, void *workspace,
                                 size_t *workspace_bytes, bbgr_stream_t stream) {
  if (int rc = check_common(a, "bbgr_eval_sampled")) return rc;
  BBGR_REQUIRE(a->n_neg >= 0 && 1 + a->n_neg <= EVAL_MAX_CAND && a->k_max <= EVAL_MAX_K,
               "bbgr_eval_sampled: 1+n_neg <= 256, k_max <= 64");
  BBGR_REQUIRE(workspace_bytes, "bbgr_eval_sampled: null workspace_bytes");
  const EvalLayout L = eval_layout(a, false, 0);
  if (!workspace) {
    *workspace_bytes = L.total;
    return BBGR_OK;
  }
  if (*workspace_bytes < L.total) {
    set_error("bbgr_eval_sampled: workspace %zu < %zu bytes", *workspace_bytes, L.total);
    return BBGR_ERR_WORKSPACE;
  }
  const int d = a->d;
  if (d != 64 && d != 128 && d != 256) {
    set_error("bbgr_eval_sampled: embedding dim %d unsupported (64, 128, 256)", d);
    return BBGR_ERR_UNSUPPORTED;
  }
  hipStream_t st = as_stream(stream);
  if (a->n_users > 0) {
    BBGR_REQUIRE(a->pos_rank, "bbgr_eval_sampled: null pos_rank");
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
    P.cand_in = a->cand_in;
    BBGR_HIP(hipMemsetAsync(a->topk, 0xff, sizeof(int) * (size_t)a->n_users * a->k_max, st));
    const unsigned grid = (unsigned)((a->n_users + 15) / 16);
    const bool small = 1 + a->n_neg <= 128;
    switch (d) {
      case 64:
        if (small) hipLaunchKernelGGL((eval_sampled_kernel<64, 128>), dim3(grid), dim3(256), 0, st, P);
        else hipLaunchKernelGGL((eval_sampled_kernel<64, 256>), dim3(grid), dim3(256), 0, st, P);
        break;
      case 128:
        if (small) hipLaunchKernelGGL((eval_sampled_kernel<128, 128>), dim3(grid), dim3(256), 0, st, P);
        else hipLaunchKernelGGL((eval_sampled_kernel<128, 256>), dim3(grid), dim3(256), 0, st, P);
        break;
      default:
        if (small) hipLaunchKernelGGL((eval_sampled_kernel<256, 128>), dim3(grid), dim3(256), 0, st, P);
        else hipLaunchKernelGGL((eval_sampled_kernel<256, 256>), dim3(grid), dim3(256), 0, st, P);
        break;
    }
    BBGR_LAUNCHED("eval_sampled_kernel");
  }
  return launch_terms(a, false, L, static_cast<char *>(workspace), st);
}

extern "C" int bbgr_eval_full(const bbgr_eval_args *a, void *workspace, size_t *workspace_bytes,
                              bbgr_stream_t stream) {
  if (int rc = check_common(a, "bbgr_eval_full")) return rc;
  BBGR_REQUIRE(a->k_max <= EVAL_FULL_MAX_K, "bbgr_eval_full: k_max <= 32");
  BBGR_REQUIRE(workspace_bytes, "bbgr_eval_full: null workspace_bytes");
  const int d = a->d;
  if (d != 64 && d != 128) {
    set_error("bbgr_eval_full: embedding dim %d unsupported (64, 128)", d);
    return BBGR_ERR_UNSUPPORTED;
  }
  const EvalLayout L = eval_layout(a, true, device_cus());
  if (!workspace) {
    *workspace_bytes = L.total;
    return BBGR_OK;
  }
  if (*workspace_bytes < L.total) {
    set_error("bbgr_eval_full: workspace %zu < %zu bytes", *workspace_bytes, L.total);
    return BBGR_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  char *ws = static_cast<char *>(workspace);
  for (long b0 = 0; b0 < a->n_users; b0 += L.batch) {
    FullParams P;
    P.n_users = a->n_users - b0 < L.batch ? a->n_users - b0 : L.batch;
    P.users = (const long *)a->users + b0;
    P.tr_indptr = a->tr_indptr;
    P.tr_indices = a->tr_indices;
    P.uf = a->uf;
    P.itf = a->itf;
    P.lduf = a->lduf;
    P.ldif = a->ldif;
    P.n_items = a->n_items;
    P.n_splits = (int)L.splits;
    const long per = (a->n_items + L.splits - 1) / L.splits;
    P.split_items = (int)((per + FULL_TILE - 1) / FULL_TILE * FULL_TILE);
    P.list_score = reinterpret_cast<float *>(ws + L.lscore);
    P.list_item = reinterpret_cast<int *>(ws + L.litem);
    int rc;
    switch (d * 100 + L.km) {
      case 6416: rc = launch_full<64, 16>(P, st); break;
      case 6424: rc = launch_full<64, 24>(P, st); break;
      case 6432: rc = launch_full<64, 32>(P, st); break;
      case 12816: rc = launch_full<128, 16>(P, st); break;
      case 12824: rc = launch_full<128, 24>(P, st); break;
      default: rc = launch_full<128, 32>(P, st); break;
    }
    if (rc) return rc;
    switch (L.km) {
      case 16: rc = launch_merge<16>(P, b0, a, st); break;
      case 24: rc = launch_merge<24>(P, b0, a, st); break;
      default: rc = launch_merge<32>(P, b0, a, st); break;
    }
    if (rc) return rc;
  }
  return launch_terms(a, true, L, ws, st);
}
