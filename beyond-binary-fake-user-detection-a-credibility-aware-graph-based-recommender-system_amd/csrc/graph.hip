// Graph-side device work: CSR build, SpMM load-balance plan, operator scale
// vectors, popularity CDF, positive / pop-mix negative sampler, shuffle.
//
// Reference behaviour restated here (paths relative to the reference root):
//   CSR + coalesce        Version-2/lighgcn_cu_pop.py:309-327, :443, :450
//   operator weights      Version-2/lighgcn_cu_pop.py:429-452
//                         version_1/lightgcn_cu_pop_long_tail_exposure.py:362-396
//                         lightgcn_cu.py:368-399, lightgcn.py:352-372
//   pop_prob              Version-2/lighgcn_cu_pop.py:805-810
//   samplers              Version-2/lighgcn_cu_pop.py:330-376, lightgcn.py:296-300
#include <stdarg.h>

#include <hipcub/hipcub.hpp>

#include "common.h"

namespace bbgr {

static thread_local std::string g_err;

void set_error(const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
}

static int bits_for(uint64_t v) {
  int b = 0;
  while (b < 64 && (v >> b) != 0) ++b;
  return b == 0 ? 1 : b;
}

// ---------------------------------------------------------------------------
// CSR build: radix sort on key = row * n_cols + col (stable), then boundaries.
// ---------------------------------------------------------------------------
__global__ void csr_keys_kernel(long nnz, const int *rows, const int *cols,
                                long n_cols, unsigned long long *keys, int *ids) {
  const long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nnz) return;
  keys[k] = (unsigned long long)rows[k] * (unsigned long long)n_cols +
            (unsigned long long)cols[k];
  ids[k] = (int)k;
}

__global__ void csr_split_kernel(long nnz, const unsigned long long *keys,
                                 unsigned long long n_cols, int n_rows,
                                 int *indptr, int *indices) {
  const long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nnz) return;
  const unsigned long long key = keys[k];
  const long r = (long)(key / n_cols);
  indices[k] = (int)(key - (unsigned long long)r * n_cols);
  const long rprev = k == 0 ? -1 : (long)(keys[k - 1] / n_cols);
  for (long rr = rprev + 1; rr <= r; ++rr) indptr[rr] = (int)k;
  if (k == nnz - 1)
    for (long rr = r + 1; rr <= n_rows; ++rr) indptr[rr] = (int)nnz;
}

__global__ void fill_int_kernel(long n, int *p, int v) {
  const long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) p[k] = v;
}

static inline unsigned blocks_for(long n, int bs = 256) {
  return (unsigned)((n + bs - 1) / bs);
}

// ---------------------------------------------------------------------------
// Plan: chunk counts per row, scans, descriptors.
// ---------------------------------------------------------------------------
__global__ void plan_counts_kernel(int n_rows, const int *indptr, int thr,
                                   int chunk, int *nch, int *sflag) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  const int deg = indptr[r + 1] - indptr[r];
  const int c = plan_chunks(deg, thr, chunk);
  nch[r] = c;
  sflag[r] = c > 1 ? 1 : 0;
}

__global__ void plan_fill_kernel(int n_rows, const int *indptr, const int *nch,
                                 const int *ch_off, const int *sflag,
                                 const int *sp_off, int4 *chunks, int4 *split) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  const int c = nch[r];
  if (c == 0) return;
  const int eb = indptr[r], ee = indptr[r + 1];
  const int base = ch_off[r];
  // equal-size chunks (last one shorter by < c edges)
  const long len = ee - eb;
  for (int j = 0; j < c; ++j) {
    const int b = eb + (int)(len * j / c);
    const int e = eb + (int)(len * (j + 1) / c);
    chunks[base + j] = make_int4(r, b, e, c > 1 ? base + j : -1);
  }
  if (sflag[r]) split[sp_off[r]] = make_int4(r, base, c, 0);
}

// ---------------------------------------------------------------------------
// Operator scale vectors (fp32, same formulas as the reference's numpy code).
// ---------------------------------------------------------------------------
__global__ void user_scales_kernel(int kind, int n_users, const int *indptr_u,
                                   const float *cred, float *deg_u, float *q,
                                   float *s, float *qs) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n_users) return;
  const float deg = (float)(indptr_u[u + 1] - indptr_u[u]);
  float a;
  if (kind == BBGR_OP_SYM) {
    a = deg > 0.f ? 1.0f / sqrtf(deg) : 0.f;  // pow(deg,-0.5), isinf -> 0
  } else {
    a = 1.0f / sqrtf(fmaxf(deg, 1.0f));
  }
  const float c = (cred && kind != BBGR_OP_SYM) ? cred[u] : 1.0f;
  const float qq = c * a;
  if (deg_u) deg_u[u] = deg;
  if (q) q[u] = qq;
  if (s) s[u] = a;
  if (qs) qs[u] = qq * a;
}

__global__ void item_scales_kernel(int kind, int n_items, const int *indptr_i,
                                   float *deg_i, float *p, float *t, float *pt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_items) return;
  const float deg = (float)(indptr_i[i + 1] - indptr_i[i]);
  float b;
  if (kind == BBGR_OP_SYM) {
    b = deg > 0.f ? 1.0f / sqrtf(deg) : 0.f;
  } else {
    b = 1.0f / sqrtf(fmaxf(deg, 1.0f));
    if (kind == BBGR_OP_METHOD_A) {
      // alpha_i = 1/log1p(max(deg_i,1)) computed in double then cast to fp32
      // (np.log1p on float32 input gives float32; difference is < 1 ulp).
      const float alpha = (float)(1.0 / log1p((double)fmaxf(deg, 1.0f)));
      b = b * alpha;
    }
  }
  if (deg_i) deg_i[i] = deg;
  if (p) p[i] = b;
  if (t) t[i] = b;
  if (pt) pt[i] = b * b;
}

// ---------------------------------------------------------------------------
// Popularity CDF.
// ---------------------------------------------------------------------------
__global__ void pop_weight_kernel(int n, const int *indptr_i, double gamma,
                                  double *w) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double deg = (double)(indptr_i[i + 1] - indptr_i[i]);
  w[i] = pow(deg + 1.0, gamma);
}

// Out of place: every thread divides by the scan's last element, so the scan
// output must stay unmodified while any block still reads it (normalising in
// place let the block holding element n-1 overwrite it with 1.0 before other
// blocks had read it).
__global__ void cdf_normalise_kernel(int n, const double *scan, double *cdf) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  cdf[i] = scan[i] / scan[n - 1];
}

// ---------------------------------------------------------------------------
// Sampler.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool row_has(const int *indices, int b, int e,
                                        int item) {
  // np.searchsorted(arr, item) (side='left') then equality test.
  int lo = b, hi = e;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (indices[mid] < item) lo = mid + 1;
    else hi = mid;
  }
  return lo < e && indices[lo] == item;
}

__device__ __forceinline__ int cdf_search(const double *cdf, int n, double u) {
  // np.searchsorted(cdf, u, side='right'): first index with cdf[idx] > u.
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cdf[mid] <= u) lo = mid + 1;
    else hi = mid;
  }
  return lo < n ? lo : n - 1;
}

__global__ void sample_kernel(long batch, const long *users, const int *indptr,
                              const int *indices, int n_items, const double *cdf,
                              float mix_pop, int max_tries, unsigned long long seed,
                              unsigned long long counter0, const long *state, long *pos,
                              long *neg, int *fail_count) {
  const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  // captured steps read this step's counter from the device step state
  const unsigned long long counter = state ? (unsigned long long)state[1] : counter0;
  const long u = users[b];
  const int rb = indptr[u], re = indptr[u + 1];
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const uint32_t c2 = (uint32_t)counter;
  const uint32_t c3 = (uint32_t)(counter >> 32) ^ ((uint32_t)((unsigned long long)b >> 32) * 0x9E3779B9u);
  const uint32_t c1 = (uint32_t)b;
  // positive: uniform within the row
  {
    const u32x4 r = philox4x32_10(u32x4{0xFFFFFFFFu, c1, c2, c3}, k0, k1);
    const int deg = re - rb;
    if (deg == 0) {
      pos[b] = -1;
    } else {
      int j = (int)(u01_53(r.x, r.y) * (double)deg);
      if (j >= deg) j = deg - 1;
      pos[b] = indices[rb + j];
    }
  }
  // negatives
  uint32_t draw = 0;
  for (int t = 0; t < max_tries; ++t, ++draw) {
    const u32x4 r = philox4x32_10(u32x4{draw, c1, c2, c3}, k0, k1);
    const double coin = u01_53(r.x, r.y);
    const double v = u01_53(r.z, r.w);
    int j;
    if (cdf && coin < (double)mix_pop) {
      j = cdf_search(cdf, n_items, v);
    } else {
      j = (int)(v * (double)n_items);
      if (j >= n_items) j = n_items - 1;
    }
    if (!row_has(indices, rb, re, j)) {
      neg[b] = j;
      return;
    }
  }
  for (int t = 0; t < BBGR_NEG_CAP; ++t, ++draw) {
    const u32x4 r = philox4x32_10(u32x4{draw, c1, c2, c3}, k0, k1);
    int j = (int)(u01_53(r.z, r.w) * (double)n_items);
    if (j >= n_items) j = n_items - 1;
    if (!row_has(indices, rb, re, j)) {
      neg[b] = j;
      return;
    }
  }
  neg[b] = -1;
  if (fail_count) atomicAdd(fail_count, 1);
}

__global__ void shuffle_keys_kernel(long n, unsigned long long seed,
                                    unsigned long long counter,
                                    unsigned long long *keys) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const u32x4 r = philox4x32_10(
      u32x4{(uint32_t)i, (uint32_t)((unsigned long long)i >> 32), (uint32_t)counter,
            (uint32_t)(counter >> 32)},
      (uint32_t)seed, (uint32_t)(seed >> 32) ^ 0x5bd1e995u);
  keys[i] = ((unsigned long long)r.x << 32) | r.y;
}

__global__ void gather_scale_kernel(long nnz, const int *indices, const float *scale,
                                    float *out) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < nnz) out[e] = scale[indices[e]];
}

// Vertex order: degree histogram (integer atomics: exact), iota values for
// the descending sort, inverse permutation, id relabelling.
// For every slot s of CSR a (row r, column c): the slot of CSR b (the
// transpose: row c, column-sorted) that holds the same edge; the k-th copy of
// a duplicate pair maps to the k-th copy. One 16-lane group per row of a.
__global__ void transpose_slots_kernel(int n_rows, const int *a_indptr, const int *a_indices,
                                       const int *b_indptr, const int *b_indices, int *out) {
  const long r = (long)blockIdx.x * (blockDim.x / 16) + (threadIdx.x >> 4);
  if (r >= n_rows) return;
  for (int s = a_indptr[r] + (threadIdx.x & 15); s < a_indptr[r + 1]; s += 16) {
    const int c = a_indices[s];
    int k = 0;   // earlier copies of (r, c) in this row (a's columns are sorted)
    while (s - k - 1 >= a_indptr[r] && a_indices[s - k - 1] == c) ++k;
    int lo = b_indptr[c], hi = b_indptr[c + 1];   // first position holding r
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (b_indices[mid] < r) lo = mid + 1;
      else hi = mid;
    }
    out[s] = lo + k;
  }
}

// offs[k] = entries of the ascending list[0..*count) below bounds[k] (lower
// bound); one thread per boundary, the list is read O(log count) times
__global__ void list_offsets_kernel(int n_bounds, const long *bounds, const long *list,
                                    const long *count, long *offs) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_bounds) return;
  const long b = bounds[k];
  long lo = 0, hi = *count;
  while (lo < hi) {
    const long mid = (lo + hi) >> 1;
    if (list[mid] < b) lo = mid + 1;
    else hi = mid;
  }
  offs[k] = lo;
}

// pos[list[j]] = j for j < *count: the compact position of each listed row
__global__ void list_positions_kernel(long n_max, const long *list, const long *count,
                                      int *pos) {
  const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_max || j >= *count) return;
  pos[list[j]] = (int)j;
}

__global__ void degree_count_kernel(long n, const int *ids, int *deg) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) atomicAdd(deg + ids[e], 1);
}

// Replicated counters: workgroup b counts into copy b % DEG_COPIES. Workgroups
// are dispatched round-robin to the 8 XCDs, so each copy takes the atomics
// of one XCD and a power-law id (one item holds ~1 % of a Zipf graph's edges)
// sees 1/8 of the same-address traffic; a second pass sums the copies.
constexpr int DEG_COPIES = 8;
// One atomic per RUN of equal ids in a wave instead of one per id: edge lists
// grouped by one endpoint (a user's edges together, as ingested) made a wave's
// 64 atomics hit a handful of counters, serialised at L2. A lane opens a run
// where its id differs from the previous lane's; the run's first lane adds the
// run length (integers: the counts are exact in any order).
__global__ void degree_count_copies_kernel(long n, const int *ids, int n_bins, int *copies) {
  int *mine = copies + (long)(blockIdx.x % DEG_COPIES) * n_bins;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int id = e < n ? ids[e] : -1;
  const int prev = __shfl(id, lane > 0 ? lane - 1 : 0);
  const bool start = lane == 0 || id != prev;
  const unsigned long long starts = __ballot(start);
  if (start && id >= 0) {
    const unsigned long long later = lane < 63 ? starts >> (lane + 1) : 0ull;
    const int end = later ? lane + __ffsll((long long)later) : 64;   // next run's first lane
    atomicAdd(mine + id, end - lane);
  }
}

__global__ void degree_sum_copies_kernel(int n_bins, const int *copies, int *deg) {
  const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_bins) return;
  int s = 0;
#pragma unroll
  for (int c = 0; c < DEG_COPIES; ++c) s += copies[(long)c * n_bins + j];
  deg[j] = s;
}

__global__ void iota_kernel(int n, int *out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = i;
}

__global__ void invert_perm_kernel(int n, const int *perm, int *rank) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) rank[perm[j]] = j;
}

__global__ void relabel_kernel(long n, const int *ids, const int *map, int *out) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) out[e] = map[ids[e]];
}

struct NonEmpty {
  const int *indptr;
  __host__ __device__ bool operator()(const long &r) const {
    return indptr[r + 1] > indptr[r];
  }
};

struct Flagged {
  const unsigned char *mask;
  __host__ __device__ bool operator()(const long &r) const { return mask[r] != 0; }
};

// bbgr_profile_marker: does nothing; its dispatches mark a trace window
__global__ __launch_bounds__(64) void profile_marker_kernel() {}

}  // namespace bbgr

using namespace bbgr;

// ===========================================================================
// Library entry points
// ===========================================================================
extern "C" int bbgr_abi_version(void) { return BBGR_ABI_VERSION; }

extern "C" const char *bbgr_last_error(void) { return g_err.c_str(); }

extern "C" int bbgr_device_info(int device, int *cu_count, char *arch_name,
                                int arch_name_len) {
  hipDeviceProp_t prop;
  BBGR_HIP(hipGetDeviceProperties(&prop, device));
  if (cu_count) *cu_count = prop.multiProcessorCount;
  if (arch_name && arch_name_len > 0) {
    snprintf(arch_name, (size_t)arch_name_len, "%s", prop.gcnArchName);
  }
  return BBGR_OK;
}

extern "C" int bbgr_sync(bbgr_stream_t stream) {
  BBGR_HIP(hipStreamSynchronize(as_stream(stream)));
  return BBGR_OK;
}

extern "C" int bbgr_profile_marker(int32_t tag, bbgr_stream_t stream) {
  BBGR_REQUIRE(tag >= 1 && tag <= 1024, "bbgr_profile_marker: tag in [1, 1024]");
  hipLaunchKernelGGL(profile_marker_kernel, dim3((unsigned)tag), dim3(64), 0, as_stream(stream));
  BBGR_LAUNCHED("profile_marker_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_csr_build(int64_t nnz, const int32_t *rows,
                              const int32_t *cols, int32_t n_rows,
                              int32_t n_cols, int32_t *indptr, int32_t *indices,
                              int32_t *perm_out, void *workspace,
                              size_t *workspace_bytes, bbgr_stream_t stream) {
  BBGR_REQUIRE(workspace_bytes, "bbgr_csr_build: null workspace_bytes");
  BBGR_REQUIRE(nnz >= 0 && nnz < 2147483647LL, "bbgr_csr_build: nnz out of range");
  BBGR_REQUIRE(n_rows >= 0 && n_cols >= 0, "bbgr_csr_build: negative shape");
  hipStream_t st = as_stream(stream);
  const int end_bit = bits_for((uint64_t)(n_rows > 0 ? n_rows : 1) *
                               (uint64_t)(n_cols > 0 ? n_cols : 1));
  size_t temp = 0;
  BBGR_HIP(hipcub::DeviceRadixSort::SortPairs(
      nullptr, temp, (unsigned long long *)nullptr, (unsigned long long *)nullptr,
      (int *)nullptr, (int *)nullptr, (int)nnz, 0, end_bit, st));
  const size_t off_k1 = 0;
  const size_t off_k2 = align_up(off_k1 + 8 * (size_t)nnz);
  const size_t off_i1 = align_up(off_k2 + 8 * (size_t)nnz);
  const size_t off_i2 = align_up(off_i1 + 4 * (size_t)nnz);
  const size_t off_t = align_up(off_i2 + 4 * (size_t)nnz);
  const size_t need = align_up(off_t + temp);
  if (!workspace) {
    *workspace_bytes = need;
    return BBGR_OK;
  }
  if (*workspace_bytes < need) {
    set_error("bbgr_csr_build: workspace %zu < %zu", *workspace_bytes, need);
    return BBGR_ERR_WORKSPACE;
  }
  BBGR_REQUIRE(indptr, "bbgr_csr_build: null indptr");
  if (nnz == 0) {
    hipLaunchKernelGGL(fill_int_kernel, dim3(blocks_for((long)n_rows + 1)), dim3(256), 0,
                       st, (long)n_rows + 1, indptr, 0);
    BBGR_LAUNCHED("fill_int_kernel");
    return BBGR_OK;
  }
  BBGR_REQUIRE(rows && cols && indices, "bbgr_csr_build: null arrays");
  char *ws = (char *)workspace;
  auto *k1 = (unsigned long long *)(ws + off_k1);
  auto *k2 = (unsigned long long *)(ws + off_k2);
  int *i1 = (int *)(ws + off_i1);
  int *i2 = perm_out ? perm_out : (int *)(ws + off_i2);
  hipLaunchKernelGGL(csr_keys_kernel, dim3(blocks_for(nnz)), dim3(256), 0, st,
                     (long)nnz, rows, cols, (long)n_cols, k1, i1);
  BBGR_LAUNCHED("csr_keys_kernel");
  BBGR_HIP(hipcub::DeviceRadixSort::SortPairs(ws + off_t, temp, k1, k2, i1, i2,
                                              (int)nnz, 0, end_bit, st));
  hipLaunchKernelGGL(csr_split_kernel, dim3(blocks_for(nnz)), dim3(256), 0, st,
                     (long)nnz, k2, (unsigned long long)n_cols, n_rows, indptr,
                     indices);
  BBGR_LAUNCHED("csr_split_kernel");
  return BBGR_OK;
}

static int plan_defaults(const bbgr_csr *csr, int *thr, int *chunk) {
  *thr = csr->long_threshold > 0 ? csr->long_threshold : 256;
  *chunk = csr->chunk_edges > 0 ? csr->chunk_edges : 2048;
  if (*chunk < 16) {
    set_error("plan: chunk_edges %d < 16", *chunk);
    return BBGR_ERR_INVALID;
  }
  return BBGR_OK;
}

// Workspace: nch[n], ch_off[n], sflag[n], sp_off[n], cub temp.
static int plan_scan(const bbgr_csr *csr, void *workspace, size_t *workspace_bytes,
                     hipStream_t st, int **nch, int **ch_off, int **sflag,
                     int **sp_off, bool *query) {
  const int n = csr->n_rows;
  size_t temp = 0;
  BBGR_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, temp, (int *)nullptr,
                                            (int *)nullptr, n > 0 ? n : 1, st));
  const size_t a = align_up(4 * (size_t)(n + 1));
  const size_t need = 4 * a + align_up(temp);
  *query = workspace == nullptr;
  if (!workspace) {
    *workspace_bytes = need;
    return BBGR_OK;
  }
  if (*workspace_bytes < need) {
    set_error("plan: workspace %zu < %zu", *workspace_bytes, need);
    return BBGR_ERR_WORKSPACE;
  }
  int thr, chunk;
  int rc = plan_defaults(csr, &thr, &chunk);
  if (rc) return rc;
  char *ws = (char *)workspace;
  *nch = (int *)ws;
  *ch_off = (int *)(ws + a);
  *sflag = (int *)(ws + 2 * a);
  *sp_off = (int *)(ws + 3 * a);
  if (n == 0) return BBGR_OK;
  hipLaunchKernelGGL(plan_counts_kernel, dim3(blocks_for(n)), dim3(256), 0, st, n,
                     csr->indptr, thr, chunk, *nch, *sflag);
  BBGR_LAUNCHED("plan_counts_kernel");
  BBGR_HIP(hipcub::DeviceScan::ExclusiveSum(ws + 4 * a, temp, *nch, *ch_off, n, st));
  BBGR_HIP(hipcub::DeviceScan::ExclusiveSum(ws + 4 * a, temp, *sflag, *sp_off, n, st));
  return BBGR_OK;
}

extern "C" int bbgr_csr_plan_count(const bbgr_csr *csr, int32_t *n_chunks,
                                   int32_t *n_split, void *workspace,
                                   size_t *workspace_bytes, bbgr_stream_t stream) {
  BBGR_REQUIRE(csr && workspace_bytes && csr->indptr, "bbgr_csr_plan_count: null arg");
  hipStream_t st = as_stream(stream);
  int *nch, *ch_off, *sflag, *sp_off;
  bool query;
  int rc = plan_scan(csr, workspace, workspace_bytes, st, &nch, &ch_off, &sflag,
                     &sp_off, &query);
  if (rc || query) return rc;
  BBGR_REQUIRE(n_chunks && n_split, "bbgr_csr_plan_count: null outputs");
  const int n = csr->n_rows;
  if (n == 0) {
    *n_chunks = 0;
    *n_split = 0;
    return BBGR_OK;
  }
  int h[4];
  BBGR_HIP(hipMemcpyAsync(&h[0], ch_off + n - 1, 4, hipMemcpyDeviceToHost, st));
  BBGR_HIP(hipMemcpyAsync(&h[1], nch + n - 1, 4, hipMemcpyDeviceToHost, st));
  BBGR_HIP(hipMemcpyAsync(&h[2], sp_off + n - 1, 4, hipMemcpyDeviceToHost, st));
  BBGR_HIP(hipMemcpyAsync(&h[3], sflag + n - 1, 4, hipMemcpyDeviceToHost, st));
  BBGR_HIP(hipStreamSynchronize(st));
  *n_chunks = h[0] + h[1];
  *n_split = h[2] + h[3];
  return BBGR_OK;
}

extern "C" int bbgr_csr_plan_build(const bbgr_csr *csr, int32_t *chunks,
                                   int32_t *split, void *workspace,
                                   size_t *workspace_bytes, bbgr_stream_t stream) {
  BBGR_REQUIRE(csr && workspace_bytes && csr->indptr, "bbgr_csr_plan_build: null arg");
  hipStream_t st = as_stream(stream);
  int *nch, *ch_off, *sflag, *sp_off;
  bool query;
  int rc = plan_scan(csr, workspace, workspace_bytes, st, &nch, &ch_off, &sflag,
                     &sp_off, &query);
  if (rc || query) return rc;
  const int n = csr->n_rows;
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(csr->n_chunks == 0 || chunks, "bbgr_csr_plan_build: null chunks");
  BBGR_REQUIRE(csr->n_split == 0 || split, "bbgr_csr_plan_build: null split");
  hipLaunchKernelGGL(plan_fill_kernel, dim3(blocks_for(n)), dim3(256), 0, st, n,
                     csr->indptr, nch, ch_off, sflag, sp_off, (int4 *)chunks,
                     (int4 *)split);
  BBGR_LAUNCHED("plan_fill_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_operator_scales(int32_t kind, int32_t n_users,
                                    int32_t n_items, const int32_t *indptr_u,
                                    const int32_t *indptr_i, const float *cred,
                                    float *deg_u, float *deg_i, float *p,
                                    float *q, float *s, float *t, float *pt,
                                    float *qs, bbgr_stream_t stream) {
  BBGR_REQUIRE(kind >= BBGR_OP_GS && kind <= BBGR_OP_SYM,
               "bbgr_operator_scales: unknown operator kind");
  BBGR_REQUIRE(indptr_u && indptr_i, "bbgr_operator_scales: null indptr");
  hipStream_t st = as_stream(stream);
  if (n_users > 0) {
    hipLaunchKernelGGL(user_scales_kernel, dim3(blocks_for(n_users)), dim3(256), 0,
                       st, kind, n_users, indptr_u, cred, deg_u, q, s, qs);
    BBGR_LAUNCHED("user_scales_kernel");
  }
  if (n_items > 0) {
    hipLaunchKernelGGL(item_scales_kernel, dim3(blocks_for(n_items)), dim3(256), 0,
                       st, kind, n_items, indptr_i, deg_i, p, t, pt);
    BBGR_LAUNCHED("item_scales_kernel");
  }
  return BBGR_OK;
}

extern "C" int bbgr_pop_cdf(int32_t n_items, const int32_t *indptr_i,
                            double gamma, double *cdf, void *workspace,
                            size_t *workspace_bytes, bbgr_stream_t stream) {
  BBGR_REQUIRE(workspace_bytes && n_items > 0, "bbgr_pop_cdf: bad args");
  hipStream_t st = as_stream(stream);
  size_t temp = 0;
  BBGR_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, temp, (double *)nullptr,
                                            (double *)nullptr, n_items, st));
  const size_t a = align_up(8 * (size_t)n_items);
  const size_t need = 2 * a + align_up(temp);
  if (!workspace) {
    *workspace_bytes = need;
    return BBGR_OK;
  }
  if (*workspace_bytes < need) {
    set_error("bbgr_pop_cdf: workspace %zu < %zu", *workspace_bytes, need);
    return BBGR_ERR_WORKSPACE;
  }
  BBGR_REQUIRE(indptr_i && cdf, "bbgr_pop_cdf: null arrays");
  char *ws = (char *)workspace;
  double *w = (double *)ws;
  double *scan = (double *)(ws + a);
  hipLaunchKernelGGL(pop_weight_kernel, dim3(blocks_for(n_items)), dim3(256), 0, st,
                     n_items, indptr_i, gamma, w);
  BBGR_LAUNCHED("pop_weight_kernel");
  BBGR_HIP(hipcub::DeviceScan::InclusiveSum(ws + 2 * a, temp, w, scan, n_items, st));
  hipLaunchKernelGGL(cdf_normalise_kernel, dim3(blocks_for(n_items)), dim3(256), 0,
                     st, n_items, (const double *)scan, cdf);
  BBGR_LAUNCHED("cdf_normalise_kernel");
  return BBGR_OK;
}

static int sample_launch(int64_t batch, const int64_t *users, const int32_t *indptr,
                         const int32_t *indices, int32_t n_items, const double *cdf,
                         float mix_pop, int32_t max_tries, uint64_t seed, uint64_t counter,
                         const int64_t *state, int64_t *pos, int64_t *neg,
                         int32_t *fail_count, bbgr_stream_t stream) {
  BBGR_REQUIRE(batch >= 0 && n_items > 0 && max_tries >= 0, "bbgr_sample: bad sizes");
  if (batch == 0) return BBGR_OK;
  BBGR_REQUIRE(users && indptr && indices && pos && neg, "bbgr_sample: null arrays");
  hipLaunchKernelGGL(sample_kernel, dim3(blocks_for(batch)), dim3(256), 0,
                     as_stream(stream), (long)batch, (const long *)users, indptr,
                     indices, n_items, cdf, mix_pop, max_tries,
                     (unsigned long long)seed, (unsigned long long)counter,
                     (const long *)state, (long *)pos, (long *)neg, fail_count);
  BBGR_LAUNCHED("sample_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_sample(int64_t batch, const int64_t *users,
                           const int32_t *indptr, const int32_t *indices,
                           int32_t n_items, const double *cdf, float mix_pop,
                           int32_t max_tries, uint64_t seed, uint64_t counter,
                           int64_t *pos, int64_t *neg, int32_t *fail_count,
                           bbgr_stream_t stream) {
  return sample_launch(batch, users, indptr, indices, n_items, cdf, mix_pop, max_tries, seed,
                       counter, nullptr, pos, neg, fail_count, stream);
}

extern "C" int bbgr_sample_dev(int64_t batch, const int64_t *users,
                               const int32_t *indptr, const int32_t *indices,
                               int32_t n_items, const double *cdf, float mix_pop,
                               int32_t max_tries, uint64_t seed, const int64_t *state,
                               int64_t *pos, int64_t *neg, int32_t *fail_count,
                               bbgr_stream_t stream) {
  BBGR_REQUIRE(state, "bbgr_sample_dev: null state");
  return sample_launch(batch, users, indptr, indices, n_items, cdf, mix_pop, max_tries, seed,
                       0, state, pos, neg, fail_count, stream);
}

extern "C" int bbgr_shuffle(int64_t n, const int64_t *in, int64_t *out,
                            uint64_t seed, uint64_t counter, void *workspace,
                            size_t *workspace_bytes, bbgr_stream_t stream) {
  BBGR_REQUIRE(workspace_bytes && n >= 0 && n < 2147483647LL, "bbgr_shuffle: bad args");
  hipStream_t st = as_stream(stream);
  size_t temp = 0;
  BBGR_HIP(hipcub::DeviceRadixSort::SortPairs(
      nullptr, temp, (unsigned long long *)nullptr, (unsigned long long *)nullptr,
      (long *)nullptr, (long *)nullptr, (int)(n > 0 ? n : 1), 0, 64, st));
  const size_t a = align_up(8 * (size_t)(n > 0 ? n : 1));
  const size_t need = 2 * a + align_up(temp);
  if (!workspace) {
    *workspace_bytes = need;
    return BBGR_OK;
  }
  if (*workspace_bytes < need) {
    set_error("bbgr_shuffle: workspace %zu < %zu", *workspace_bytes, need);
    return BBGR_ERR_WORKSPACE;
  }
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(in && out, "bbgr_shuffle: null arrays");
  char *ws = (char *)workspace;
  auto *k1 = (unsigned long long *)ws;
  auto *k2 = (unsigned long long *)(ws + a);
  hipLaunchKernelGGL(shuffle_keys_kernel, dim3(blocks_for(n)), dim3(256), 0, st,
                     (long)n, (unsigned long long)seed, (unsigned long long)counter,
                     k1);
  BBGR_LAUNCHED("shuffle_keys_kernel");
  BBGR_HIP(hipcub::DeviceRadixSort::SortPairs(ws + 2 * a, temp, k1, k2,
                                              (const long *)in, (long *)out, (int)n,
                                              0, 64, st));
  return BBGR_OK;
}

extern "C" int bbgr_gather_scale(int64_t nnz, const int32_t *indices,
                                 const float *scale, float *out,
                                 bbgr_stream_t stream) {
  BBGR_REQUIRE(nnz >= 0, "bbgr_gather_scale: negative nnz");
  if (nnz == 0) return BBGR_OK;
  BBGR_REQUIRE(indices && scale && out, "bbgr_gather_scale: null arrays");
  hipLaunchKernelGGL(gather_scale_kernel, dim3(blocks_for(nnz)), dim3(256), 0,
                     as_stream(stream), (long)nnz, indices, scale, out);
  BBGR_LAUNCHED("gather_scale_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_transpose_slots(const bbgr_csr *a, const bbgr_csr *b, int32_t *out,
                                    bbgr_stream_t stream) {
  BBGR_REQUIRE(a && b && out, "bbgr_transpose_slots: null args");
  BBGR_REQUIRE(a->n_rows == b->n_cols && a->n_cols == b->n_rows && a->nnz == b->nnz,
               "bbgr_transpose_slots: b is not the transpose of a");
  if (a->n_rows == 0 || a->nnz == 0) return BBGR_OK;
  hipLaunchKernelGGL(transpose_slots_kernel, dim3((unsigned)((a->n_rows + 15) / 16)), dim3(256),
                     0, as_stream(stream), (int)a->n_rows, a->indptr, a->indices, b->indptr,
                     b->indices, out);
  BBGR_LAUNCHED("transpose_slots_kernel");
  return BBGR_OK;
}

__global__ void invert_slots_kernel(long n, const int *perm, int *inv) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) inv[perm[t]] = (int)t;
}

__global__ void compose_slots_kernel(long n, const int *perm_a, const int *inv_b, int *out) {
  const long s = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < n) out[s] = inv_b[perm_a[s]];
}

extern "C" int bbgr_slots_from_perms(int64_t nnz, const int32_t *perm_a, const int32_t *perm_b,
                                     int32_t *out, int32_t *scratch, bbgr_stream_t stream) {
  BBGR_REQUIRE(nnz >= 0 && nnz < 2147483647LL, "bbgr_slots_from_perms: nnz out of range");
  if (nnz == 0) return BBGR_OK;
  BBGR_REQUIRE(perm_a && perm_b && out && scratch, "bbgr_slots_from_perms: null arrays");
  BBGR_REQUIRE(out != scratch, "bbgr_slots_from_perms: out and scratch alias");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(invert_slots_kernel, dim3(blocks_for(nnz)), dim3(256), 0, st, (long)nnz,
                     perm_b, scratch);
  BBGR_LAUNCHED("invert_slots_kernel");
  hipLaunchKernelGGL(compose_slots_kernel, dim3(blocks_for(nnz)), dim3(256), 0, st, (long)nnz,
                     perm_a, scratch, out);
  BBGR_LAUNCHED("compose_slots_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_nonempty_rows(int32_t n_rows, const int32_t *indptr,
                                  int64_t *out, int64_t *count, void *workspace,
                                  size_t *workspace_bytes, bbgr_stream_t stream) {
  BBGR_REQUIRE(workspace_bytes && n_rows >= 0, "bbgr_nonempty_rows: bad args");
  hipStream_t st = as_stream(stream);
  hipcub::CountingInputIterator<long> it(0);
  NonEmpty sel{indptr};
  size_t temp = 0;
  BBGR_HIP(hipcub::DeviceSelect::If(nullptr, temp, it, (long *)nullptr,
                                    (long *)nullptr, n_rows > 0 ? n_rows : 1, sel, st));
  const size_t need = align_up(temp);
  if (!workspace) {
    *workspace_bytes = need;
    return BBGR_OK;
  }
  if (*workspace_bytes < need) {
    set_error("bbgr_nonempty_rows: workspace %zu < %zu", *workspace_bytes, need);
    return BBGR_ERR_WORKSPACE;
  }
  BBGR_REQUIRE(indptr && out && count, "bbgr_nonempty_rows: null arrays");
  if (n_rows == 0) {
    BBGR_HIP(hipMemsetAsync(count, 0, 8, st));
    return BBGR_OK;
  }
  BBGR_HIP(hipcub::DeviceSelect::If(workspace, temp, it, (long *)out, (long *)count,
                                    n_rows, sel, st));
  return BBGR_OK;
}

extern "C" int bbgr_mask_to_list(int64_t n, const uint8_t *mask, int64_t *out,
                                 int64_t *count, void *workspace, size_t *workspace_bytes,
                                 bbgr_stream_t stream) {
  BBGR_REQUIRE(workspace_bytes && n >= 0 && n < (int64_t)1 << 31,
               "bbgr_mask_to_list: bad args");
  hipStream_t st = as_stream(stream);
  hipcub::CountingInputIterator<long> it(0);
  Flagged sel{mask};
  size_t temp = 0;
  BBGR_HIP(hipcub::DeviceSelect::If(nullptr, temp, it, (long *)nullptr, (long *)nullptr,
                                    n > 0 ? (int)n : 1, sel, st));
  const size_t need = align_up(temp);
  if (!workspace) {
    *workspace_bytes = need;
    return BBGR_OK;
  }
  if (*workspace_bytes < need) {
    set_error("bbgr_mask_to_list: workspace %zu < %zu", *workspace_bytes, need);
    return BBGR_ERR_WORKSPACE;
  }
  BBGR_REQUIRE(mask && out && count, "bbgr_mask_to_list: null arrays");
  if (n == 0) {
    BBGR_HIP(hipMemsetAsync(count, 0, 8, st));
    return BBGR_OK;
  }
  BBGR_HIP(hipcub::DeviceSelect::If(workspace, temp, it, (long *)out, (long *)count, (int)n,
                                    sel, st));
  return BBGR_OK;
}

extern "C" int bbgr_list_offsets(int32_t n_bounds, const int64_t *bounds, const int64_t *list,
                                 const int64_t *count, int64_t *offs, bbgr_stream_t stream) {
  BBGR_REQUIRE(n_bounds >= 0, "bbgr_list_offsets: bad args");
  if (n_bounds == 0) return BBGR_OK;
  BBGR_REQUIRE(bounds && list && count && offs, "bbgr_list_offsets: null arrays");
  hipLaunchKernelGGL(list_offsets_kernel, dim3((unsigned)((n_bounds + 63) / 64)), dim3(64), 0,
                     as_stream(stream), (int)n_bounds, (const long *)bounds, (const long *)list,
                     (const long *)count, (long *)offs);
  BBGR_LAUNCHED("list_offsets_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_list_positions(int64_t n_max, const int64_t *list, const int64_t *count,
                                   int32_t *pos, bbgr_stream_t stream) {
  BBGR_REQUIRE(n_max >= 0 && n_max < (int64_t)1 << 31, "bbgr_list_positions: bad args");
  if (n_max == 0) return BBGR_OK;
  BBGR_REQUIRE(list && count && pos, "bbgr_list_positions: null arrays");
  hipLaunchKernelGGL(list_positions_kernel, dim3((unsigned)((n_max + 255) / 256)), dim3(256), 0,
                     as_stream(stream), (long)n_max, (const long *)list, (const long *)count,
                     (int *)pos);
  BBGR_LAUNCHED("list_positions_kernel");
  return BBGR_OK;
}

// deg[key[j]] = count[j] for the j < *n_runs runs of the sorted ids.
__global__ void degree_runs_kernel(int n_max, const unsigned *key, const int *count,
                                   const int *n_runs, int n_bins, int *deg) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_max || j >= *n_runs) return;
  const unsigned k = key[j];
  if (k < (unsigned)n_bins) deg[k] = count[j];
}

// Large id lists are counted by sorting instead of atomics: 50M ids with
// power-law repeats (Zipf items: the hottest holds ~1 % of the edges) or over
// 5M counters far beyond L2 (users) ran 1.9-2.7 ms per side with the per-XCD
// atomic copies (C4, round 4); a radix sort of the ids (ceil(log2 n) bits,
// ~3 passes), a run-length encode and one scatter of the run lengths are
// HBM-streaming passes instead. Counts are exact either way.
constexpr long DEG_SORT_MIN = 1L << 22;

struct DegreeSortWs {
  size_t keys, uniq, cnt, runs, temp, total;
};

static DegreeSortWs degree_sort_ws(long n_ids, int n, int end_bit) {
  DegreeSortWs w = {};
  size_t t_sort = 0, t_rle = 0;
  // size queries (no launch; the sizes are what they return)
  (void)hipcub::DeviceRadixSort::SortKeys(nullptr, t_sort, (const unsigned *)nullptr,
                                          (unsigned *)nullptr, (int)n_ids, 0, end_bit);
  (void)hipcub::DeviceRunLengthEncode::Encode(nullptr, t_rle, (const unsigned *)nullptr,
                                              (unsigned *)nullptr, (int *)nullptr, (int *)nullptr,
                                              (int)n_ids);
  w.keys = align_up(4 * (size_t)n_ids);
  w.uniq = align_up(4 * (size_t)n);
  w.cnt = align_up(4 * (size_t)n);
  w.runs = align_up(8);
  w.temp = align_up(t_sort > t_rle ? t_sort : t_rle);
  w.total = w.keys + w.uniq + w.cnt + w.runs + w.temp;
  return w;
}

extern "C" int bbgr_degree_count_ws(int64_t n_ids, const int32_t *ids, int32_t n,
                                    int32_t *degree, void *workspace, size_t *workspace_bytes,
                                    bbgr_stream_t stream) {
  BBGR_REQUIRE(workspace_bytes && n_ids >= 0 && n >= 0 && n_ids < (1LL << 31),
               "bbgr_degree_count_ws: bad args");
  const bool by_sort = n_ids >= DEG_SORT_MIN && n > 0;
  int end_bit = 1;
  while (end_bit < 32 && (1ull << end_bit) < (unsigned long long)n) ++end_bit;
  const DegreeSortWs sw = by_sort ? degree_sort_ws(n_ids, n, end_bit) : DegreeSortWs{};
  const size_t need = by_sort ? sw.total : (size_t)DEG_COPIES * 4 * (size_t)(n > 0 ? n : 1);
  if (!workspace) {
    *workspace_bytes = need;
    return BBGR_OK;
  }
  if (*workspace_bytes < need) {
    set_error("bbgr_degree_count_ws: workspace %zu < %zu", *workspace_bytes, need);
    return BBGR_ERR_WORKSPACE;
  }
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(degree && (n_ids == 0 || ids), "bbgr_degree_count_ws: null arrays");
  hipStream_t st = as_stream(stream);
  if (by_sort) {   // (ids are in [0, n): the caller's contract, as for the atomics)
    char *ws = static_cast<char *>(workspace);
    unsigned *keys = reinterpret_cast<unsigned *>(ws);
    unsigned *uniq = reinterpret_cast<unsigned *>(ws + sw.keys);
    int *cnt = reinterpret_cast<int *>(ws + sw.keys + sw.uniq);
    int *runs = reinterpret_cast<int *>(ws + sw.keys + sw.uniq + sw.cnt);
    void *temp = ws + sw.keys + sw.uniq + sw.cnt + sw.runs;
    size_t t = sw.temp;
    BBGR_HIP(hipcub::DeviceRadixSort::SortKeys(temp, t, reinterpret_cast<const unsigned *>(ids),
                                               keys, (int)n_ids, 0, end_bit, st));
    t = sw.temp;
    BBGR_HIP(hipcub::DeviceRunLengthEncode::Encode(temp, t, keys, uniq, cnt, runs, (int)n_ids,
                                                   st));
    BBGR_HIP(hipMemsetAsync(degree, 0, 4 * (size_t)n, st));
    hipLaunchKernelGGL(degree_runs_kernel, dim3(blocks_for(n)), dim3(256), 0, st, (int)n,
                       (const unsigned *)uniq, (const int *)cnt, (const int *)runs, (int)n,
                       degree);
    BBGR_LAUNCHED("degree_runs_kernel");
    return BBGR_OK;
  }
  int *copies = static_cast<int *>(workspace);
  BBGR_HIP(hipMemsetAsync(copies, 0, need, st));
  if (n_ids > 0) {
    hipLaunchKernelGGL(degree_count_copies_kernel, dim3(blocks_for(n_ids)), dim3(256), 0, st,
                       (long)n_ids, ids, (int)n, copies);
    BBGR_LAUNCHED("degree_count_copies_kernel");
  }
  hipLaunchKernelGGL(degree_sum_copies_kernel, dim3(blocks_for(n)), dim3(256), 0, st, (int)n,
                     (const int *)copies, degree);
  BBGR_LAUNCHED("degree_sum_copies_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_degree_count(int64_t n_ids, const int32_t *ids, int32_t n,
                                 int32_t *degree, bbgr_stream_t stream) {
  BBGR_REQUIRE(n_ids >= 0 && n >= 0, "bbgr_degree_count: negative size");
  hipStream_t st = as_stream(stream);
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(degree && (n_ids == 0 || ids), "bbgr_degree_count: null arrays");
  BBGR_HIP(hipMemsetAsync(degree, 0, 4 * (size_t)n, st));
  if (n_ids == 0) return BBGR_OK;
  hipLaunchKernelGGL(degree_count_kernel, dim3(blocks_for(n_ids)), dim3(256), 0, st,
                     (long)n_ids, ids, degree);
  BBGR_LAUNCHED("degree_count_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_degree_order(int32_t n, const int32_t *degree, int32_t *perm,
                                 int32_t *rank, void *workspace, size_t *workspace_bytes,
                                 bbgr_stream_t stream) {
  BBGR_REQUIRE(workspace_bytes && n >= 0, "bbgr_degree_order: bad args");
  hipStream_t st = as_stream(stream);
  const int m = n > 0 ? n : 1;
  size_t temp = 0;
  BBGR_HIP(hipcub::DeviceRadixSort::SortPairsDescending(
      nullptr, temp, (const unsigned *)nullptr, (unsigned *)nullptr, (const int *)nullptr,
      (int *)nullptr, m, 0, 32, st));
  const size_t off_k = 0;
  const size_t off_v = align_up(off_k + 4 * (size_t)m);
  const size_t off_t = align_up(off_v + 4 * (size_t)m);
  const size_t need = align_up(off_t + temp);
  if (!workspace) {
    *workspace_bytes = need;
    return BBGR_OK;
  }
  if (*workspace_bytes < need) {
    set_error("bbgr_degree_order: workspace %zu < %zu", *workspace_bytes, need);
    return BBGR_ERR_WORKSPACE;
  }
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(degree && perm && rank, "bbgr_degree_order: null arrays");
  char *ws = (char *)workspace;
  unsigned *k_out = (unsigned *)(ws + off_k);
  int *iota = (int *)(ws + off_v);
  hipLaunchKernelGGL(iota_kernel, dim3(blocks_for(n)), dim3(256), 0, st, n, iota);
  BBGR_LAUNCHED("iota_kernel");
  // radix sort is stable: equal degrees keep ascending input id
  BBGR_HIP(hipcub::DeviceRadixSort::SortPairsDescending(
      ws + off_t, temp, (const unsigned *)degree, k_out, (const int *)iota, (int *)perm, n, 0,
      32, st));
  hipLaunchKernelGGL(invert_perm_kernel, dim3(blocks_for(n)), dim3(256), 0, st, n,
                     (const int *)perm, (int *)rank);
  BBGR_LAUNCHED("invert_perm_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_relabel(int64_t n, const int32_t *ids, const int32_t *map, int32_t *out,
                            bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0, "bbgr_relabel: negative size");
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(ids && map && out, "bbgr_relabel: null arrays");
  hipLaunchKernelGGL(relabel_kernel, dim3(blocks_for(n)), dim3(256), 0, as_stream(stream),
                     (long)n, ids, map, out);
  BBGR_LAUNCHED("relabel_kernel");
  return BBGR_OK;
}
