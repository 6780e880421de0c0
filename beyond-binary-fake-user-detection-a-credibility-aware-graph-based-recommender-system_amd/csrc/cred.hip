// Credibility-GNN edge weighting: main.py:645-707.
//
// CredModel.ewa_raw            w  = max(beta * clamp(verified, 0, 1) + gamma * align, 0)
// CredModel.normalize_per_dst  w~ = w / (scatter_add(w, dst) + 1e-12)[dst]
// CredModel.aggregate          out = scatter_add(w~ * src_x[src], dst)
//
// The aggregation itself is bbgr_spmm over the destination-row CSR with the
// normalised weights as explicit edge values (its transpose, over the
// source-row CSR, is the backward). The kernels here produce those weights:
//   ewa_raw_kernel     raw weights in input-edge order (coalesced over the
//                      [E][lda] attribute rows);
//   raw_csr_kernel     the same weights in CSR order: the ONE random pass
//                      (each slot gathers its edge's 4-B weight);
//   seg_sum_kernel     per-destination sums on the CSR's load-balance plan
//                      over the CSR-order weights (coalesced): long rows are
//                      cut into chunks (one 256-thread workgroup each,
//                      fixed-order LDS tree), short rows take a 16-lane group;
//                      seg_fixup_kernel adds the chunk partials of split rows
//                      in chunk order -> deterministic;
//   seg_scale_kernel   w~ in CSR order (the SpMM's edge values);
//   edge_scale_kernel  w~ in input-edge order (what the reference returns,
//                      w1t) from the input-order weights and each edge's dst:
//                      coalesced, no scatter. (Without dst: the scatter
//                      through perm in seg_scale_kernel.)
#include "common.h"

namespace bbgr {

struct EwaParams {
  int n_rows;
  int long_threshold;
  int n_chunks;
  const int *indptr;
  const int4 *chunks;
  const int4 *split;
  const int *perm;            // CSR slot -> input edge id
  const float *raw;           // raw weights, input-edge order
  const float *raw_csr;       // raw weights, CSR order
  float *denom;               // [n_rows] per-destination sums
  float *partial;             // [n_chunks] chunk partial sums (split rows)
  float eps;
  float *w_edge;              // normalised, input-edge order (nullable)
  float *w_csr;               // normalised, CSR order (nullable)
};

__global__ void ewa_raw_kernel(long E, const float *attr, long lda, int cv, int ca, float beta,
                               float gamma, float *out) {
#pragma clang fp contract(off)   // two products and a sum, as torch evaluates them
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const float *a = attr + e * lda;
  const float verified = fminf(fmaxf(a[cv], 0.f), 1.f);   // clamp(0, 1)
  const float w = beta * verified + gamma * a[ca];
  out[e] = fmaxf(w, 0.f);                                  // clamp(min=0)
}

__global__ void raw_csr_kernel(long E, const int *perm, const float *raw, float *out) {
  const long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < E) out[k] = raw[perm[k]];   // 4-B gathers from the input-order weights (MALL-sized)
}

__global__ void edge_scale_kernel(long E, const float *raw, const int *dst, const float *denom,
                                  float eps, float *w_edge) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  w_edge[e] = raw[e] / (denom[dst[e]] + eps);
}

__device__ __forceinline__ float group16_sum_c(float v) {
  v += __shfl_xor(v, 1, 16);
  v += __shfl_xor(v, 2, 16);
  v += __shfl_xor(v, 4, 16);
  v += __shfl_xor(v, 8, 16);
  return v;
}

__global__ __launch_bounds__(256) void seg_sum_kernel(EwaParams P) {
  __shared__ float red[256];
  if ((int)blockIdx.x < P.n_chunks) {
    const int4 ch = P.chunks[blockIdx.x];   // row, e_begin, e_end, slot
    float s = 0.f;
    for (int k = ch.y + threadIdx.x; k < ch.z; k += 256) s += P.raw_csr[k];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      if (ch.w < 0) P.denom[ch.x] = red[0];
      else P.partial[ch.w] = red[0];
    }
    return;
  }
  const long r = (long)(blockIdx.x - P.n_chunks) * 16 + (threadIdx.x >> 4);
  const int lane = threadIdx.x & 15;
  if (r >= P.n_rows) return;
  const int b = P.indptr[r], e = P.indptr[r + 1];
  if (e - b > P.long_threshold) return;   // owned by chunk blocks
  float s = 0.f;
  for (int k = b + lane; k < e; k += 16) s += P.raw_csr[k];
  s = group16_sum_c(s);
  if (lane == 0) P.denom[r] = s;
}

__global__ void seg_fixup_kernel(int n_split, EwaParams P) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_split) return;
  const int4 sp = P.split[i];   // row, slot_begin, n_slots
  float s = 0.f;
  for (int j = 0; j < sp.z; ++j) s += P.partial[sp.y + j];
  P.denom[sp.x] = s;
}

__device__ __forceinline__ void scale_slot(const EwaParams &P, int k, float den) {
  const float wt = P.raw_csr[k] / den;   // == raw[perm[k]] / den
  if (P.w_csr) P.w_csr[k] = wt;
  if (P.w_edge) P.w_edge[P.perm[k]] = wt;   // only without dst: scatter
}

__global__ __launch_bounds__(256) void seg_scale_kernel(EwaParams P) {
  if ((int)blockIdx.x < P.n_chunks) {
    const int4 ch = P.chunks[blockIdx.x];
    const float den = P.denom[ch.x] + P.eps;
    for (int k = ch.y + threadIdx.x; k < ch.z; k += 256) scale_slot(P, k, den);
    return;
  }
  const long r = (long)(blockIdx.x - P.n_chunks) * 16 + (threadIdx.x >> 4);
  const int lane = threadIdx.x & 15;
  if (r >= P.n_rows) return;
  const int b = P.indptr[r], e = P.indptr[r + 1];
  if (e - b > P.long_threshold) return;
  const float den = P.denom[r] + P.eps;
  for (int k = b + lane; k < e; k += 16) scale_slot(P, k, den);
}

}  // namespace bbgr

using namespace bbgr;

extern "C" int bbgr_ewa_normalize(const bbgr_csr *csr, const int32_t *perm, const int32_t *dst,
                                  const float *w_in,
                                  const float *edge_attr, int64_t lda, int32_t col_verified,
                                  int32_t col_align, float beta, float gamma, float eps,
                                  float *w_raw, float *w_edge, float *w_csr, void *workspace,
                                  size_t *workspace_bytes, bbgr_stream_t stream) {
  BBGR_REQUIRE(csr && csr->n_rows >= 0 && csr->nnz >= 0 && workspace_bytes,
               "bbgr_ewa_normalize: bad csr / workspace_bytes");
  const long E = csr->nnz;
  // raw weights in input order are needed for w_edge by the coalesced pass
  const bool own_raw = !w_in && !w_raw;
  const size_t a_raw = own_raw ? align_up(4 * (size_t)(E > 0 ? E : 1)) : 0;
  const size_t a_csr = align_up(4 * (size_t)(E > 0 ? E : 1));
  const size_t a_den = align_up(4 * (size_t)(csr->n_rows > 0 ? csr->n_rows : 1));
  const size_t need = a_raw + a_csr + a_den +
                      align_up(4 * (size_t)(csr->n_chunks > 0 ? csr->n_chunks : 1));
  if (!workspace) {
    *workspace_bytes = need;
    return BBGR_OK;
  }
  if (*workspace_bytes < need) {
    set_error("bbgr_ewa_normalize: workspace %zu < %zu bytes", *workspace_bytes, need);
    return BBGR_ERR_WORKSPACE;
  }
  if (csr->n_rows == 0 || E == 0) return BBGR_OK;
  BBGR_REQUIRE(csr->indptr && perm, "bbgr_ewa_normalize: null indptr / perm");
  BBGR_REQUIRE(csr->n_chunks == 0 || (csr->chunks && csr->long_threshold > 0),
               "bbgr_ewa_normalize: csr needs its load-balance plan");
  BBGR_REQUIRE(csr->n_split == 0 || csr->split, "bbgr_ewa_normalize: plan split rows missing");
  BBGR_REQUIRE(w_in || (edge_attr && col_verified >= 0 && col_align >= 0 &&
                        col_verified < lda && col_align < lda),
               "bbgr_ewa_normalize: need w_in or edge_attr with valid columns");
  hipStream_t st = as_stream(stream);
  char *ws = static_cast<char *>(workspace);
  const float *raw = w_in;
  if (!w_in) {
    float *out = own_raw ? reinterpret_cast<float *>(ws) : w_raw;
    hipLaunchKernelGGL(ewa_raw_kernel, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, st, E,
                       edge_attr, (long)lda, col_verified, col_align, beta, gamma, out);
    BBGR_LAUNCHED("ewa_raw_kernel");
    raw = out;
  }
  float *raw_csr = reinterpret_cast<float *>(ws + a_raw);
  hipLaunchKernelGGL(raw_csr_kernel, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, st, E,
                     perm, raw, raw_csr);
  BBGR_LAUNCHED("raw_csr_kernel");
  EwaParams P;
  P.n_rows = csr->n_rows;
  P.long_threshold = csr->n_chunks ? csr->long_threshold : 0x7fffffff;
  P.n_chunks = csr->n_chunks;
  P.indptr = csr->indptr;
  P.chunks = reinterpret_cast<const int4 *>(csr->chunks);
  P.split = reinterpret_cast<const int4 *>(csr->split);
  P.perm = perm;
  P.raw = raw;
  P.raw_csr = raw_csr;
  P.denom = reinterpret_cast<float *>(ws + a_raw + a_csr);
  P.partial = reinterpret_cast<float *>(ws + a_raw + a_csr + a_den);
  P.eps = eps;
  P.w_edge = dst ? nullptr : w_edge;
  P.w_csr = w_csr;
  const unsigned grid = (unsigned)(csr->n_chunks + ((long)csr->n_rows + 15) / 16);
  hipLaunchKernelGGL(seg_sum_kernel, dim3(grid), dim3(256), 0, st, P);
  BBGR_LAUNCHED("seg_sum_kernel");
  if (csr->n_split > 0) {
    hipLaunchKernelGGL(seg_fixup_kernel, dim3((unsigned)((csr->n_split + 255) / 256)),
                       dim3(256), 0, st, csr->n_split, P);
    BBGR_LAUNCHED("seg_fixup_kernel");
  }
  if (P.w_edge || w_csr) {
    hipLaunchKernelGGL(seg_scale_kernel, dim3(grid), dim3(256), 0, st, P);
    BBGR_LAUNCHED("seg_scale_kernel");
  }
  if (dst && w_edge) {
    hipLaunchKernelGGL(edge_scale_kernel, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, st,
                       E, raw, dst, P.denom, eps, w_edge);
    BBGR_LAUNCHED("edge_scale_kernel");
  }
  return BBGR_OK;
}
