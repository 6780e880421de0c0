// Training-step kernels: fused BPR forward/backward, deterministic loss
// reduction, Adam (torch.optim.Adam semantics), row zero / row axpy.
//
// Reference: LightGCN.bpr_loss  Version-2/lighgcn_cu_pop.py:495-508
//            (lightgcn.py:333-349; lightgcn_cu.py:632-648 adds L_fair)
//            opt.step()          Version-2/lighgcn_cu_pop.py:863 (Adam, :793)
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace bbgr {

struct BprParams {
  long batch, n_users, n_items;
  const long *users, *pos, *neg;
  const float *uf, *itf, *ue, *ie;
  long lduf, ldif, ldue, ldie;
  const float *pop;
  float reg, lambda_fair, inv_b;
  float *parts;
  const float *dloss;
  float *g_uf, *g_if, *g_ue, *g_ie;
  long ldguf, ldgif, ldgue, ldgie;
  float *contrib;
  long ldc;
  float *scores_out;      // partial (s+, s-, r) over this table's columns
  const float *scores;    // complete (s+, s-, r) (all-reduced over column shards)
};

__device__ __forceinline__ float group16_sum(float v) {
  v += __shfl_xor(v, 1, 16);
  v += __shfl_xor(v, 2, 16);
  v += __shfl_xor(v, 4, 16);
  v += __shfl_xor(v, 8, 16);
  return v;
}

__device__ __forceinline__ float dot4(float4 a, float4 b) {
  return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}

__device__ __forceinline__ void atomic_axpy4(float *dst, float a, float4 x) {
  atomicAdd(dst + 0, a * x.x);
  atomicAdd(dst + 1, a * x.y);
  atomicAdd(dst + 2, a * x.z);
  atomicAdd(dst + 3, a * x.w);
}

__device__ __forceinline__ void atomic_axpby4(float *dst, float a, float4 x,
                                              float b, float4 y) {
  atomicAdd(dst + 0, a * x.x + b * y.x);
  atomicAdd(dst + 1, a * x.y + b * y.y);
  atomicAdd(dst + 2, a * x.z + b * y.z);
  atomicAdd(dst + 3, a * x.w + b * y.w);
}

// One 16-lane group per (user, pos, neg) triple.
template <int D>
__global__ __launch_bounds__(256) void bpr_kernel(BprParams P) {
  constexpr int V = RowShape<D>::V;
  constexpr int LANES = RowShape<D>::LANES;
  const long b = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int lane = threadIdx.x & 15;
  if (b >= P.batch) return;
  const long u = P.users[b], ip = P.pos[b], in = P.neg[b];
  if (u < 0 || u >= P.n_users || ip < 0 || ip >= P.n_items || in < 0 || in >= P.n_items) {
    if (P.scores_out && lane == 0) {
      P.scores_out[3 * b + 0] = 0.f;
      P.scores_out[3 * b + 1] = 0.f;
      P.scores_out[3 * b + 2] = 0.f;
    }
    if (P.scores_out) return;
    if (P.parts && lane == 0) {
      P.parts[3 * b + 0] = 0.f;
      P.parts[3 * b + 1] = 0.f;
      P.parts[3 * b + 2] = 0.f;
    }
    if (P.contrib && lane < LANES) {
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int k = 0; k < V; ++k)
          reinterpret_cast<float4 *>(P.contrib + (r * P.batch + b) * P.ldc)[lane + 16 * k] = z;
    }
    return;  // whole group leaves together
  }
  const bool act = lane < LANES;   // narrow rows: the first d/4 lanes hold the row
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 fu[V], fp[V], fn[V];
  const float4 *pu = reinterpret_cast<const float4 *>(P.uf + u * P.lduf) + lane;
  const float4 *pp = reinterpret_cast<const float4 *>(P.itf + ip * P.ldif) + lane;
  const float4 *pn = reinterpret_cast<const float4 *>(P.itf + in * P.ldif) + lane;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    fu[k] = act ? pu[16 * k] : z4;
    fp[k] = act ? pp[16 * k] : z4;
    fn[k] = act ? pn[16 * k] : z4;
  }
  float sp = 0.f, sn = 0.f;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    sp += dot4(fu[k], fp[k]);
    sn += dot4(fu[k], fn[k]);
  }
  sp = group16_sum(sp);
  sn = group16_sum(sn);
  const bool need_reg = P.parts || P.g_ue || P.g_ie || P.scores_out;
  float4 eu[V], ep[V], en[V];
  if (need_reg) {
    const float4 *qu = reinterpret_cast<const float4 *>(P.ue + u * P.ldue) + lane;
    const float4 *qp = reinterpret_cast<const float4 *>(P.ie + ip * P.ldie) + lane;
    const float4 *qn = reinterpret_cast<const float4 *>(P.ie + in * P.ldie) + lane;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      eu[k] = act ? qu[16 * k] : z4;
      ep[k] = act ? qp[16 * k] : z4;
      en[k] = act ? qn[16 * k] : z4;
    }
  }
  float r_full = 0.f;
  if (P.parts || P.scores_out) {
    float r = 0.f;
#pragma unroll
    for (int k = 0; k < V; ++k) r += dot4(eu[k], eu[k]) + dot4(ep[k], ep[k]) + dot4(en[k], en[k]);
    r_full = group16_sum(r);
  }
  if (P.scores_out) {   // column shard: this table's share of (s+, s-, r) only
    if (lane == 0) {
      P.scores_out[3 * b + 0] = sp;
      P.scores_out[3 * b + 1] = sn;
      P.scores_out[3 * b + 2] = r_full;
    }
    return;
  }
  if (P.scores) {       // column shard: the complete sums over every shard
    sp = P.scores[3 * b + 0];
    sn = P.scores[3 * b + 1];
    r_full = P.scores[3 * b + 2];
  }
  const float x = sp - sn;
  const float sig = 1.0f / (1.0f + expf(-x));
  if (P.parts) {
    const float r = r_full;
    if (lane == 0) {
      P.parts[3 * b + 0] = -logf(sig + 1e-12f);
      P.parts[3 * b + 1] = r;
      P.parts[3 * b + 2] = P.pop ? P.pop[ip] * sp : 0.f;
    }
  }
  if (!(P.g_uf || P.g_if || P.g_ue || P.g_ie || P.contrib)) return;
  const float G = (P.dloss ? *P.dloss : 1.0f) * P.inv_b;
  // d/dx [-log(sigmoid(x) + 1e-12)] = -sigmoid'(x) / (sigmoid(x) + 1e-12)
  const float gx = -(sig * (1.0f - sig)) / (sig + 1e-12f) * G;
  const float gpos = gx + (P.pop ? P.lambda_fair * P.pop[ip] * G : 0.f);
  const float gneg = -gx;
  if (!act) return;   // narrow rows: lanes past the row write nothing
  if (P.contrib) {   // deterministic mode: per-triple rows, summed by scatter_add_rows
    float4 *cu = reinterpret_cast<float4 *>(P.contrib + b * P.ldc) + lane;
    float4 *cp = reinterpret_cast<float4 *>(P.contrib + (P.batch + b) * P.ldc) + lane;
    float4 *cn = reinterpret_cast<float4 *>(P.contrib + (2 * P.batch + b) * P.ldc) + lane;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      cu[16 * k] = make_float4(gpos * fp[k].x + gneg * fn[k].x, gpos * fp[k].y + gneg * fn[k].y,
                               gpos * fp[k].z + gneg * fn[k].z, gpos * fp[k].w + gneg * fn[k].w);
      cp[16 * k] = make_float4(gpos * fu[k].x, gpos * fu[k].y, gpos * fu[k].z, gpos * fu[k].w);
      cn[16 * k] = make_float4(gneg * fu[k].x, gneg * fu[k].y, gneg * fu[k].z, gneg * fu[k].w);
    }
  } else if (P.g_uf) {
    float *d = P.g_uf + u * P.ldguf + 4 * lane;
#pragma unroll
    for (int k = 0; k < V; ++k) atomic_axpby4(d + 64 * k, gpos, fp[k], gneg, fn[k]);
  }
  if (P.g_if && !P.contrib) {
    float *dp = P.g_if + ip * P.ldgif + 4 * lane;
    float *dn = P.g_if + in * P.ldgif + 4 * lane;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      atomic_axpy4(dp + 64 * k, gpos, fu[k]);
      atomic_axpy4(dn + 64 * k, gneg, fu[k]);
    }
  }
  const float gr = 2.0f * P.reg * G;
  if (P.g_ue) {
    float *d = P.g_ue + u * P.ldgue + 4 * lane;
#pragma unroll
    for (int k = 0; k < V; ++k) atomic_axpy4(d + 64 * k, gr, eu[k]);
  }
  if (P.g_ie) {
    float *dp = P.g_ie + ip * P.ldgie + 4 * lane;
    float *dn = P.g_ie + in * P.ldgie + 4 * lane;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      atomic_axpy4(dp + 64 * k, gr, ep[k]);
      atomic_axpy4(dn + 64 * k, gr, en[k]);
    }
  }
}

// One workgroup, fixed summation order -> deterministic loss.
__global__ __launch_bounds__(256) void bpr_reduce_kernel(long batch,
                                                         const float *parts,
                                                         float reg, float lam,
                                                         float *loss) {
  __shared__ float s0[256], s1[256], s2[256];
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  for (long b = threadIdx.x; b < batch; b += 256) {
    a0 += parts[3 * b + 0];
    a1 += parts[3 * b + 1];
    a2 += parts[3 * b + 2];
  }
  s0[threadIdx.x] = a0;
  s1[threadIdx.x] = a1;
  s2[threadIdx.x] = a2;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      s0[threadIdx.x] += s0[threadIdx.x + w];
      s1[threadIdx.x] += s1[threadIdx.x + w];
      s2[threadIdx.x] += s2[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float inv = 1.0f / (float)batch;
    loss[0] = s0[0] * inv + reg * (s1[0] * inv) + lam * (s2[0] * inv);
  }
}

// torch.optim.Adam (single-tensor/foreach math), float4 vectorised; the
// per-element update is adam_elem (common.h), shared with the fused epilogue.
// Step t from device memory (captured steps): the bias corrections come from
// the host-built table, so the constants equal the host's bit for bit.
__device__ __forceinline__ AdamConsts device_step_consts(AdamConsts c, float lr,
                                                         const float *bc, const long *state) {
  if (state) {
    const long t = clamp_step(state);
    c.step = lr / bc[2 * (t - 1)];
    c.bc2s = bc[2 * (t - 1) + 1];
  }
  return c;
}

// Each workgroup owns contiguous tiles of 256 x ADAM_TILE float4 per stream
// (thread t on float4 t, t + 256, ...), all loads of a tile issued before the
// math, every stream read and written non-temporally (each byte is touched
// once), one tile per workgroup (no grid cap). Measured on the C4 tables
// (tools/adam_variants.hip, 28 B/param): 5M x 64 1.643 -> 1.439 ms (5.45 ->
// 6.23 TB/s) for 4-float4 tiles and a 4096-workgroup cap against the
// grid-stride one-float4 form; on a second box the uncapped grid took another
// 6-8 % (users 1.702 -> 1.568 / 1.595 ms with 4 / 2 float4 per stream, items
// 0.317 -> 0.309 / 0.297 ms); the same bits.
#define ADAM_TILE 2
__global__ __launch_bounds__(256) void adam_kernel(long n4, float4 *p, const float4 *g,
                                                   float4 *m, float4 *v, AdamConsts c0,
                                                   float gs, float lr, const float *bc,
                                                   const long *state) {
  const AdamConsts c = device_step_consts(c0, lr, bc, state);
  constexpr long tile = 256L * ADAM_TILE;
  for (long t0 = (long)blockIdx.x * tile; t0 < n4; t0 += (long)gridDim.x * tile) {
    float4 pp[ADAM_TILE], gg[ADAM_TILE], mm[ADAM_TILE], vv[ADAM_TILE];
#pragma unroll
    for (int u = 0; u < ADAM_TILE; ++u) {
      const long k = t0 + u * 256 + threadIdx.x;
      if (k < n4) {
        pp[u] = ld_nt(p + k);
        gg[u] = ld_nt(g + k);
        mm[u] = ld_nt(m + k);
        vv[u] = ld_nt(v + k);
      }
    }
#pragma unroll
    for (int u = 0; u < ADAM_TILE; ++u) {
      const long k = t0 + u * 256 + threadIdx.x;
      if (k < n4) {
        adam_elem(pp[u].x, gs * gg[u].x, mm[u].x, vv[u].x, c);
        adam_elem(pp[u].y, gs * gg[u].y, mm[u].y, vv[u].y, c);
        adam_elem(pp[u].z, gs * gg[u].z, mm[u].z, vv[u].z, c);
        adam_elem(pp[u].w, gs * gg[u].w, mm[u].w, vv[u].w, c);
        st_nt(p + k, pp[u]);
        st_nt(m + k, mm[u]);
        st_nt(v + k, vv[u]);
      }
    }
  }
}

__global__ void adam_tail_kernel(long n, long start, float *p, const float *g, float *m,
                                 float *v, AdamConsts c0, float gs, float lr, const float *bc,
                                 const long *state) {
  const long i = start + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const AdamConsts c = device_step_consts(c0, lr, bc, state);
  adam_elem(p[i], gs * g[i], m[i], v[i], c);
}

// bbgr_step_begin: state = {t, counter, next counter}; one lane.
__global__ void step_begin_kernel(long *state) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const long t = state[0], next = state[2];
  state[0] = t + 1;
  state[1] = next;
  state[2] = next + 1;
}

__global__ void rows_zero_kernel(long n, const long *idx, float *t, long ld,
                                 int d) {
  const long k = (long)blockIdx.x * (blockDim.x / 16) + (threadIdx.x >> 4);
  if (k >= n || idx[k] < 0) return;
  float *row = t + idx[k] * ld;
  for (int c = threadIdx.x & 15; c < d; c += 16) row[c] = 0.f;
}

__global__ void mark_rows_kernel(long n, const long *idx, unsigned char v,
                                 unsigned char *mask, long n_rows) {
  const long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const long r = idx[k];
  if (r >= 0 && r < n_rows) mask[r] = v;   // -1 = sampler "no item"; out of range: skipped
}

// one 16-lane group per listed row; duplicate writes store the same value
__global__ void mark_neighbors_kernel(long n, const long *rows, const int *indptr,
                                      const int *indices, unsigned char v,
                                      unsigned char *mask) {
  const long k = (long)blockIdx.x * (blockDim.x / 16) + (threadIdx.x >> 4);
  if (k >= n || rows[k] < 0) return;
  const long r = rows[k];
  for (int e = indptr[r] + (threadIdx.x & 15); e < indptr[r + 1]; e += 16)
    mask[indices[e]] = v;
}

// Flag row r in a byte mask; true if this call set it first. A byte already
// seen set needs no atomic: within the launch bytes only go 0 -> 1, so a set
// byte is final, and a stale 0 just takes the atomic path (hub items recur
// in most batch users' rows; their words would serialise the atomics).
__device__ __forceinline__ bool mark_first(long r, unsigned char *mask) {
  if (mask[r] != 0) return false;
  unsigned *w = reinterpret_cast<unsigned *>(mask + (r & ~3L));
  const unsigned sh = 8u * (unsigned)(r & 3);
  return (atomicOr(w, 1u << sh) & (0xffu << sh)) == 0u;
}

// The rows a workgroup flags first are collected in LDS and appended to the
// list with ONE global atomic add on the count per workgroup (one counter
// shared by every wave of the launch was the bottleneck: 69 us for a C4
// batch's neighbourhood against 5 us for the plain marking). Overflow past
// the LDS buffer appends directly.
constexpr int MARK_LDS = 2048;

struct MarkListLds {
  long buf[MARK_LDS];
  int n;
  unsigned long long base;
};

__device__ __forceinline__ void mark_list_push(MarkListLds &s, long r, long *list,
                                               unsigned long long *count) {
  const int k = atomicAdd(&s.n, 1);
  if (k < MARK_LDS) s.buf[k] = r;
  else list[atomicAdd(count, 1ull)] = r;
}

__device__ __forceinline__ void mark_list_flush(MarkListLds &s, long *list,
                                                unsigned long long *count) {
  __syncthreads();
  const int m = s.n < MARK_LDS ? s.n : MARK_LDS;
  if (threadIdx.x == 0 && m > 0) s.base = atomicAdd(count, (unsigned long long)m);
  __syncthreads();
  for (int i = threadIdx.x; i < m; i += blockDim.x) list[s.base + i] = s.buf[i];
}

__global__ __launch_bounds__(256) void mark_list_rows_kernel(long n, const long *idx,
                                                             unsigned char *mask, long n_rows,
                                                             long *list,
                                                             unsigned long long *count) {
  __shared__ MarkListLds s;
  if (threadIdx.x == 0) s.n = 0;
  __syncthreads();
  const long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long r = k < n ? idx[k] : -1;
  if (r >= 0 && r < n_rows && mark_first(r, mask)) mark_list_push(s, r, list, count);
  mark_list_flush(s, list, count);
}

// one 16-lane group per listed row, its edges 16 at a time
__global__ __launch_bounds__(256) void mark_list_neighbors_kernel(
    long n, const long *rows, const int *indptr, const int *indices, unsigned char *mask,
    long *list, unsigned long long *count) {
  __shared__ MarkListLds s;
  if (threadIdx.x == 0) s.n = 0;
  __syncthreads();
  const long k = (long)blockIdx.x * (blockDim.x / 16) + (threadIdx.x >> 4);
  const long r = k < n ? rows[k] : -1;
  if (r >= 0) {
    const int ee = indptr[r + 1];
    for (int e = indptr[r] + (int)(threadIdx.x & 15); e < ee; e += 16) {
      const long c = indices[e];
      if (mark_first(c, mask)) mark_list_push(s, c, list, count);
    }
  }
  mark_list_flush(s, list, count);
}

// slot bitmap of the listed rows' edges in the TRANSPOSE CSR: for every edge e
// of row rows[k], bit tmap[e] of bits is set (set != 0, atomic OR) or its
// whole word cleared (set == 0; a later launch, so no OR races the store)
__global__ void mark_slots_kernel(long n, const long *rows, const int *indptr, const int *tmap,
                                  unsigned *bits, int set) {
  const long k = (long)blockIdx.x * (blockDim.x / 16) + (threadIdx.x >> 4);
  if (k >= n || rows[k] < 0) return;
  const long r = rows[k];
  for (int e = indptr[r] + (threadIdx.x & 15); e < indptr[r + 1]; e += 16) {
    const int sl = tmap[e];
    if (set) atomicOr(bits + (sl >> 5), 1u << (sl & 31));
    else bits[sl >> 5] = 0u;
  }
}

// bbgr_batch_begin / bbgr_batch_end: one 16-lane group per batch entry b.
struct BatchParams {
  long B, U, I;
  const long *users, *pos, *neg;
  const int *indptr, *indices;
  unsigned char *mask_u, *mask_i;
  long *list;
  unsigned long long *count;
  const int *tmap;
  unsigned *bits;
  float *g_u, *g_i, *g_side;
  long ld_gu, ld_gi, ld_side;
  int d;
};

__device__ __forceinline__ void batch_flag_item(const BatchParams &P, MarkListLds &s, long r) {
  if (P.list) {
    if (mark_first(r, P.mask_i)) mark_list_push(s, r, P.list, P.count);
  } else {
    P.mask_i[r] = 1;
  }
}

__global__ __launch_bounds__(256) void batch_begin_kernel(BatchParams P) {
  __shared__ MarkListLds s;
  if (threadIdx.x == 0) s.n = 0;
  __syncthreads();
  const long b = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int lane = threadIdx.x & 15;
  if (b < P.B) {
    // every lane's loads issue before its first returning atomic: the pos /
    // neg rows ride on the last two lanes (a user's first 14 edges are on the
    // others), the slot bit is set without waiting on a return, and only the
    // mask's first-setter test waits
    const long u = P.users[b];
    const long pn = lane == 14 ? P.pos[b] : lane == 15 ? P.neg[b] : -1;
    const bool uok = u >= 0 && u < P.U;
    int e = 0, ee = 0;
    if (uok && P.indptr) {
      e = P.indptr[u] + lane;
      ee = P.indptr[u + 1];
    }
    if (lane == 0 && uok) P.mask_u[u] = 1;
    if (pn >= 0 && pn < P.I) batch_flag_item(P, s, pn);
    for (; e < ee; e += 16) {
      const long c = P.indices[e];
      if (P.bits) {
        const int sl = P.tmap[e];
        atomicOr(P.bits + (sl >> 5), 1u << (sl & 31));
      }
      batch_flag_item(P, s, c);
    }
  }
  if (P.list) mark_list_flush(s, P.list, P.count);   // block-uniform
}

// bbgr_rows_mark: one 16-lane group per listed user (lane 0: its masks, all
// lanes: its graph row's neighbours) and per four listed items (lanes 12-15),
// two LDS lists (users, frontier) flushed with one count add each
struct RowsMarkParams {
  long nu, ni, U, I;
  const long *users, *items, *urank, *irank;
  const int *indptr, *indices;
  unsigned char *mu, *mi, *fr, *mu_in, *mi_in;
  long *ulist, *flist;
  unsigned long long *ucount, *fcount;
};

__global__ __launch_bounds__(256) void rows_mark_kernel(RowsMarkParams P) {
  __shared__ MarkListLds su, sf;
  if (threadIdx.x == 0) su.n = sf.n = 0;
  __syncthreads();
  const long k = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int lane = threadIdx.x & 15;
  const long it = 4 * k + (lane - 12);   // lanes 12-15: items 4k .. 4k + 3
  const long i = lane >= 12 && it < P.ni ? P.items[it] : -1;
  const long u = k < P.nu ? P.users[k] : -1;
  const bool uok = u >= 0 && u < P.U;
  const long ur = uok ? (P.urank ? P.urank[u] : u) : -1;
  if (i >= 0 && i < P.I) {
    const long ir = P.irank ? P.irank[i] : i;
    if (P.mi_in) P.mi_in[i] = 1;
    P.mi[ir] = 1;
    if (mark_first(ir, P.fr)) mark_list_push(sf, ir, P.flist, P.fcount);
  }
  if (uok) {
    if (lane == 0) {
      if (P.mu_in) P.mu_in[u] = 1;
      if (mark_first(ur, P.mu)) mark_list_push(su, ur, P.ulist, P.ucount);
    }
    if (P.indptr) {
      const int ee = P.indptr[ur + 1];
      for (int e = P.indptr[ur] + lane; e < ee; e += 16) {
        const long c = P.indices[e];
        if (mark_first(c, P.fr)) mark_list_push(sf, c, P.flist, P.fcount);
      }
    }
  }
  mark_list_flush(su, P.ulist, P.ucount);   // block-uniform
  mark_list_flush(sf, P.flist, P.fcount);
}

__device__ __forceinline__ void zero_row(float *t, long ld, long r, int d, int lane) {
  if (!t) return;
  float4 *row = reinterpret_cast<float4 *>(t + r * ld);
  for (int c = lane; c < d / 4; c += 16) row[c] = make_float4(0.f, 0.f, 0.f, 0.f);
}

__global__ __launch_bounds__(256) void batch_end_kernel(BatchParams P) {
  const long b = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int lane = threadIdx.x & 15;
  if (b == 0 && lane == 0 && P.count) *P.count = 0ull;
  if (b >= P.B) return;
  const long u = P.users[b];
  const bool uok = u >= 0 && u < P.U;
  if (uok) {
    zero_row(P.g_u, P.ld_gu, u, P.d, lane);
    if (lane == 0) P.mask_u[u] = 0;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const long r = h == 0 ? P.pos[b] : P.neg[b];
    if (r < 0 || r >= P.I) continue;
    zero_row(P.g_i, P.ld_gi, r, P.d, lane);
    zero_row(P.g_side, P.ld_side, r, P.d, lane);
    if (lane == 0) P.mask_i[r] = 0;
  }
  if (uok && P.indptr) {
    const int ee = P.indptr[u + 1];
    for (int e = P.indptr[u] + lane; e < ee; e += 16) {
      P.mask_i[P.indices[e]] = 0;
      if (P.bits) P.bits[P.tmap[e] >> 5] = 0u;
    }
  }
}

// every neighbour of a row flagged in row_mask (indexed through row_map when
// given: CSR row r is flagged by row_mask[row_map[r]]) is set to v in mask
__global__ void mark_neighbors_of_mask_kernel(long n_rows, const unsigned char *row_mask,
                                              const int *row_map, const int *indptr,
                                              const int *indices, unsigned char v,
                                              unsigned char *mask) {
  const long r = (long)blockIdx.x * (blockDim.x / 16) + (threadIdx.x >> 4);
  if (r >= n_rows || !row_mask[row_map ? (long)row_map[r] : r]) return;
  for (int e = indptr[r] + (threadIdx.x & 15); e < indptr[r + 1]; e += 16)
    mask[indices[e]] = v;
}

// mask[r] = 1 if row r of x holds a nonzero (a -0.0 counts as zero: skipping
// a signed-zero source row leaves every sum unchanged), else 0; with a CSR,
// every neighbour of a flagged row is also set in nbr. One 16-lane group per
// row; VEC: float4 loads (d, ldx multiples of 4, x 16-byte aligned).
template <bool VEC>
__global__ __launch_bounds__(256) void row_support_kernel(long n_rows, int d, const float *x,
                                                          long ldx, unsigned char *mask,
                                                          const int *indptr, const int *indices,
                                                          unsigned char *nbr) {
  const long r = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int lane = threadIdx.x & 15;
  bool nz = false;
  if (r < n_rows) {
    const float *row = x + r * ldx;
    if (VEC) {
      for (int c = lane * 4; c < d; c += 64) {
        const float4 v = *reinterpret_cast<const float4 *>(row + c);
        nz |= (v.x != 0.f) | (v.y != 0.f) | (v.z != 0.f) | (v.w != 0.f);
      }
    } else {
      for (int c = lane; c < d; c += 16) nz |= row[c] != 0.f;
    }
  }
  const unsigned long long b = __ballot(nz);
  const bool any = ((b >> (threadIdx.x & 48)) & 0xFFFFull) != 0;
  if (r >= n_rows) return;
  if (lane == 0) mask[r] = any ? 1 : 0;
  if (any && indptr)
    for (int e = indptr[r] + lane; e < indptr[r + 1]; e += 16) nbr[indices[e]] = 1;
}

__global__ void rows_axpy_kernel(long n, const long *idx, float alpha,
                                 const float *src, long lds, float *dst, long ldd,
                                 int d) {
  const long k = (long)blockIdx.x * (blockDim.x / 16) + (threadIdx.x >> 4);
  if (k >= n || idx[k] < 0) return;
  const long r = idx[k];
  for (int c = threadIdx.x & 15; c < d; c += 16)
    atomicAdd(dst + r * ldd + c, alpha * src[r * lds + c]);
}

// bbgr_first_slot: first[ids[k]] = min k (atomic minimum: order-free), then
// slot[k] = first[ids[k]], then first[ids[k]] = INT32_MAX again.
__global__ void first_slot_min_kernel(long n, const long *ids, long n_rows, int *first) {
  const long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const long r = ids[k];
  if (r >= 0 && r < n_rows) atomicMin(first + r, (int)k);
}
__global__ void first_slot_read_kernel(long n, const long *ids, long n_rows, const int *first,
                                       long *slot) {
  const long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const long r = ids[k];
  slot[k] = (r >= 0 && r < n_rows) ? (long)first[r] : k;
}
__global__ void first_slot_reset_kernel(long n, const long *ids, long n_rows, int *first) {
  const long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const long r = ids[k];
  if (r >= 0 && r < n_rows) first[r] = 0x7fffffff;
}

// bbgr_ego_slots: the first_slot passes of a (user, pos, neg) batch at once.
// Thread t < B handles user t, thread B + j item j of cat(pos, neg).
__device__ __forceinline__ long clamp_row(long r, long n) { return r < 0 ? 0 : (r >= n ? n - 1 : r); }

__global__ void ego_slots_min_kernel(long B, const long *users, const long *pos, const long *neg,
                                     long U, long I, int *first_u, int *first_i, long *iu,
                                     long *ii) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 3 * B) return;
  if (t < B) {
    const long r = clamp_row(users[t], U);
    iu[t] = r;
    atomicMin(first_u + r, (int)t);
  } else {
    const long j = t - B;
    const long r = clamp_row(j < B ? pos[j] : neg[j - B], I);
    ii[j] = r;
    atomicMin(first_i + r, (int)j);
  }
}
__global__ void ego_slots_read_kernel(long B, const long *users, const long *pos, const long *neg,
                                      long U, long I, const int *first_u, const int *first_i,
                                      const long *iu, const long *ii, long *cu, long *sp,
                                      long *sn) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 3 * B) return;
  if (t < B) {
    const long u = users[t], p = pos[t], n = neg[t];
    const bool ok = u >= 0 && u < U && p >= 0 && p < I && n >= 0 && n < I;
    cu[t] = ok ? (long)first_u[iu[t]] : -1;
  } else {
    const long j = t - B;
    const long s = first_i[ii[j]];
    if (j < B) sp[j] = s; else sn[j - B] = s;
  }
}
__global__ void ego_slots_reset_kernel(long B, int *first_u, int *first_i, const long *iu,
                                       const long *ii) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 3 * B) return;
  if (t < B) first_u[iu[t]] = 0x7fffffff;
  else first_i[ii[t - B]] = 0x7fffffff;
}

// bbgr_ego_rows: the ego-L2 rows in first-slot form. ego_count_kernel counts
// each first slot's occurrences among the valid triples (int atomics: one per
// occurrence, not d float atomics); ego_rows_kernel gives every slot s (one
// 16-lane group each) y = gr * e added n times from +0.0 and re-zeroes its
// count. All addends of a row are the same y, so the atomics' sum in any
// order is this sequential sum, bit for bit.
__global__ void ego_count_kernel(long B, const long *cu, const long *sp, const long *sn,
                                 int *counts) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B || cu[t] < 0) return;
  atomicAdd(counts + cu[t], 1);
  atomicAdd(counts + B + sp[t], 1);
  atomicAdd(counts + B + sn[t], 1);
}

template <int D>
__global__ __launch_bounds__(256) void ego_rows_kernel(long B, const long *iu, const long *ii,
                                                       const float *ue, long ldue,
                                                       const float *ie, long ldie,
                                                       const float *dloss, float inv_b,
                                                       float reg, int *counts, float *g_u,
                                                       long ldgu, float *g_i, long ldgi,
                                                       float scale, int *counts_u_out) {
  constexpr int V = D / 64;
  const long s = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int lane = threadIdx.x & 15;
  if (s >= 3 * B) return;
  const int n = counts[s];
  const bool user = s < B;
  if (user && counts_u_out && lane == 0) counts_u_out[s] = n;
  float4 *dst = reinterpret_cast<float4 *>(user ? g_u + s * ldgu : g_i + (s - B) * ldgi) + lane;
  float4 acc[V];
#pragma unroll
  for (int k = 0; k < V; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n > 0) {
    // bbgr_bpr's G and gr, in its order
    const float G = (dloss ? *dloss : 1.0f) * inv_b;
    const float gr = 2.0f * reg * G;
    const float4 *src = reinterpret_cast<const float4 *>(
                            user ? ue + iu[s] * ldue : ie + ii[s - B] * ldie) + lane;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float4 e = src[16 * k];
      const float4 y = make_float4(__fmul_rn(gr, e.x), __fmul_rn(gr, e.y), __fmul_rn(gr, e.z),
                                   __fmul_rn(gr, e.w));
      for (int j = 0; j < n; ++j)
        acc[k] = make_float4(__fadd_rn(acc[k].x, y.x), __fadd_rn(acc[k].y, y.y),
                             __fadd_rn(acc[k].z, y.z), __fadd_rn(acc[k].w, y.w));
    }
    if (lane == 0) counts[s] = 0;
    if (scale != 1.0f)   // (x * 1 == x, -0 included: the unscaled rows are these)
#pragma unroll
      for (int k = 0; k < V; ++k)
        acc[k] = make_float4(__fmul_rn(acc[k].x, scale), __fmul_rn(acc[k].y, scale),
                             __fmul_rn(acc[k].z, scale), __fmul_rn(acc[k].w, scale));
  }
#pragma unroll
  for (int k = 0; k < V; ++k) dst[16 * k] = acc[k];
}

__global__ void graph_rows_kernel(long n, const long *ids, long n_rows, const long *rank,
                                  long *out) {
  const long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const long r = ids[k];
  out[k] = (r >= 0 && r < n_rows) ? (rank ? rank[r] : r) : -1;
}

// dst[idx[k]] = src[idx[k]] (idx < 0 skipped; repeats write the same row).
__global__ __launch_bounds__(256) void rows_copy_kernel(long n, const long *idx,
                                                        const float4 *src, long lds4,
                                                        float4 *dst, long ldd4, int d4) {
  const long k = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
  if (k >= n) return;
  const long r = idx[k];
  if (r < 0) return;
  for (int c = threadIdx.x & 15; c < d4; c += 16) dst[r * ldd4 + c] = src[r * lds4 + c];
}

// dst[idx[k]] += (0 + src[k]) for distinct idx: a one-addend segment of
// scatter_segments_kernel (acc = 0 + x, then dst + acc), bit for bit.
__global__ __launch_bounds__(256) void rows_add_unique_kernel(long n, const long *idx,
                                                              const float4 *src, long lds4,
                                                              float4 *dst, long ldd4, int d4,
                                                              long n_dst) {
  const long k = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
  if (k >= n) return;
  const long r = idx[k];
  if (r < 0 || r >= n_dst) return;
  const float4 *in = src + k * lds4;
  float4 *out = dst + r * ldd4;
  for (int c = threadIdx.x & 15; c < d4; c += 16) {
    const float4 x = in[c];
    const float4 a = make_float4(0.f + x.x, 0.f + x.y, 0.f + x.z, 0.f + x.w);
    const float4 o = out[c];
    out[c] = make_float4(o.x + a.x, o.y + a.y, o.z + a.z, o.w + a.w);
  }
}

// dst[rows[f]] += (0 + src[f] + src[k2] + ... ) over each leader f's
// occurrences (slot[k] == f, ascending k; counts[f] of them): the sums of a
// stable sort's segments (scatter_segments_kernel) without the sort, the
// slots of invalid triples (zero rows) left out (+0.0 changes no such sum).
// A batch of distinct rows (counts 1) reads no slot past its own; a repeated
// row scans forward 16 slots a load until its count is found.
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

__global__ __launch_bounds__(256) void rows_add_slots_kernel(long n, const long *slot,
                                                             const int *counts, const long *rows,
                                                             const float4 *src, long lds4,
                                                             float4 *dst, long ldd4, int d4,
                                                             long n_dst) {
  const long f = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int lane = threadIdx.x & 15;
  // a leader: some valid slot points at f (f itself, or an invalid triple's
  // slot holding the first occurrence of the clamped id; slot[f] == -1 then)
  if (f >= n || counts[f] <= 0) return;   // group-uniform
  const long r = rows[f];
  if (r < 0 || r >= n_dst) return;
  const int c = counts[f];
  for (int col = lane; col - lane < d4; col += 16) {   // (every lane runs the scan's ballots)
    const bool on = col < d4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (on) acc = add4(acc, src[f * lds4 + col]);
    int found = slot[f] == f ? 1 : 0;   // (counts count the valid slots only)
    for (long k0 = f + 1; found < c && k0 < n; k0 += 16) {
      const long kk = k0 + lane;
      const bool hit = kk < n && slot[kk] == f;
      unsigned m = (unsigned)((__ballot(hit) >> (threadIdx.x & 48)) & 0xffffull);
      while (m) {
        const int j = __ffs(m) - 1;
        m &= m - 1u;
        if (on) acc = add4(acc, src[(k0 + j) * lds4 + col]);
        ++found;
      }
    }
    if (on) dst[r * ldd4 + col] = add4(dst[r * ldd4 + col], acc);
  }
}

// dst[k, :] = src[idx[k], :] (zero row for idx < 0); float4 per lane, one
// 16-lane group per row: the compaction of frontier rows for the sparse
// multi-GPU exchange.
__global__ __launch_bounds__(256) void rows_gather_kernel(long n, const long *idx,
                                                          const float4 *src, long lds4,
                                                          float4 *dst, long ldd4, int d4) {
  const long k = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
  if (k >= n) return;
  const long r = idx[k];
  float4 *out = dst + k * ldd4;
  if (r < 0) {
    for (int c = threadIdx.x & 15; c < d4; c += 16) out[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  const float4 *in = src + r * lds4;
  for (int c = threadIdx.x & 15; c < d4; c += 16) out[c] = in[c];
}

// ---- deterministic index_add_ (bbgr_scatter_add_rows) ----------------------
__global__ void scatter_keys_kernel(long n, const long *idx, long n_dst, unsigned *keys,
                                    int *vals) {
  const long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const long r = idx[k];
  keys[k] = (r >= 0 && r < n_dst) ? (unsigned)r : (unsigned)n_dst;   // n_dst = skip
  vals[k] = (int)k;
}

// One 16-lane group per sorted position; the group at the start of a run of
// equal keys sums the run's source rows in (stable) ascending-k order and adds
// the total to the destination row once. The run is read 16 positions at a
// time (lane j loads key / source index t0 + j; the run's part of the window
// is a prefix, its length a ballot), then up to 8 of its rows are gathered
// before they are added in order: a hot destination (a popular item drawn
// many times as a negative) no longer costs one dependent load chain per
// element. The additions are the same, in the same order (bitwise). src2
// (nullable): the run is summed over src, then the same sum continues over
// src2's rows of the run — one ascending sum over [src; src2], as if the two
// tables were concatenated with their index lists (bbgr_scatter_apply).
template <int D>
__global__ __launch_bounds__(256) void scatter_segments_kernel(long n, const unsigned *keys,
                                                               const int *vals,
                                                               const float *src, long lds,
                                                               const float *src2, long lds2,
                                                               float *dst, long ldd,
                                                               unsigned skip) {
  constexpr int V = RowShape<D>::V;
  constexpr int G = 8;   // rows in flight
  const long s = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int lane = threadIdx.x & 15;
  if (s >= n) return;   // group-uniform
  const unsigned key = keys[s];
  if (key == skip || (s > 0 && keys[s - 1] == key)) return;   // group-uniform
  const bool cols = lane < RowShape<D>::LANES;
  float4 acc[V];
#pragma unroll
  for (int k = 0; k < V; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int pass = 0; pass < 2; ++pass) {
  const float *sp = pass ? src2 : src;
  const long lp = pass ? lds2 : lds;
  if (!sp) break;
  for (long t0 = s;; t0 += 16) {
    const long tj = t0 + lane;
    const bool in = tj < n && keys[tj] == key;
    const int vj = in ? vals[tj] : 0;
    const unsigned m = (unsigned)((__ballot(in) >> (threadIdx.x & 48)) & 0xffffull);
    const int cnt = __popc(m);   // keys are sorted: the run's lanes are a prefix
    for (int j0 = 0; j0 < cnt; j0 += G) {
      float4 x[G][V];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int v = __shfl(vj, j0 + g, 16);
        if (cols && j0 + g < cnt) {
          const float4 *row = reinterpret_cast<const float4 *>(sp + (long)v * lp) + lane;
#pragma unroll
          for (int k = 0; k < V; ++k) x[g][k] = row[16 * k];
        }
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        if (j0 + g < cnt) {
#pragma unroll
          for (int k = 0; k < V; ++k)
            acc[k] = make_float4(acc[k].x + x[g][k].x, acc[k].y + x[g][k].y,
                                 acc[k].z + x[g][k].z, acc[k].w + x[g][k].w);
        }
      }
    }
    if (cnt < 16) break;
  }
  }
  if (!cols) return;
  float4 *out = reinterpret_cast<float4 *>(dst + (long)key * ldd) + lane;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const float4 o = out[16 * k];
    out[16 * k] = make_float4(o.x + acc[k].x, o.y + acc[k].y, o.z + acc[k].z, o.w + acc[k].w);
  }
}

}  // namespace bbgr

using namespace bbgr;

// the plan of a scatter over n rows: [k1 | k2 | v1 | v2 | sort scratch], the
// sorted (key, position) pairs in k2 / v2
static size_t scatter_plan_bytes(int64_t n, int64_t n_dst, int *end_bit_out, size_t *temp_out,
                                 hipStream_t st) {
  int end_bit = 1;   // keys are in [0, n_dst] (n_dst marks skipped rows)
  while (end_bit < 32 && (1ull << end_bit) <= (unsigned long long)n_dst) ++end_bit;
  size_t temp = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (unsigned *)nullptr, (unsigned *)nullptr,
                                           (int *)nullptr, (int *)nullptr,
                                           (int)(n > 0 ? n : 1), 0, end_bit, st);
  if (end_bit_out) *end_bit_out = end_bit;
  if (temp_out) *temp_out = temp;
  return 4 * align_up(4 * (size_t)(n > 0 ? n : 1)) + align_up(temp);
}

extern "C" int bbgr_scatter_plan(int64_t n, const int64_t *idx, int64_t n_dst, void *plan,
                                 size_t *plan_bytes, bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0 && n < (1ll << 31) && n_dst >= 0 && n_dst < 0xFFFFFFFFll && plan_bytes,
               "bbgr_scatter_plan: bad sizes");
  hipStream_t st = as_stream(stream);
  int end_bit = 1;
  size_t temp = 0;
  const size_t need = scatter_plan_bytes(n, n_dst, &end_bit, &temp, st);
  if (!plan) {
    *plan_bytes = need;
    return BBGR_OK;
  }
  if (*plan_bytes < need) {
    set_error("bbgr_scatter_plan: plan %zu < %zu bytes", *plan_bytes, need);
    return BBGR_ERR_WORKSPACE;
  }
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(idx, "bbgr_scatter_plan: null idx");
  const size_t a = align_up(4 * (size_t)n);
  char *ws = static_cast<char *>(plan);
  unsigned *k1 = reinterpret_cast<unsigned *>(ws), *k2 = reinterpret_cast<unsigned *>(ws + a);
  int *v1 = reinterpret_cast<int *>(ws + 2 * a), *v2 = reinterpret_cast<int *>(ws + 3 * a);
  hipLaunchKernelGGL(scatter_keys_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     (long)n, (const long *)idx, (long)n_dst, k1, v1);
  BBGR_LAUNCHED("scatter_keys_kernel");
  BBGR_HIP(hipcub::DeviceRadixSort::SortPairs(ws + 4 * a, temp, k1, k2, v1, v2, (int)n, 0,
                                              end_bit, st));
  return BBGR_OK;
}

extern "C" int bbgr_scatter_apply(int64_t n, int64_t n_dst, const void *plan, const float *src,
                                  int64_t ldsrc, const float *src2, int64_t ldsrc2, float *dst,
                                  int64_t lddst, int32_t d, bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0 && n < (1ll << 31) && n_dst >= 0 && n_dst < 0xFFFFFFFFll,
               "bbgr_scatter_apply: bad sizes");
  if (!supported_width(d)) {
    set_error("bbgr_scatter_apply: d = %d unsupported (8, 16, 32, 64, 128, 256)", d);
    return BBGR_ERR_UNSUPPORTED;
  }
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(plan && src && dst, "bbgr_scatter_apply: null arrays");
  BBGR_REQUIRE(aligned16(src) && aligned16(dst) && ldsrc >= d && lddst >= d &&
                   (ldsrc & 3) == 0 && (lddst & 3) == 0 &&
                   (!src2 || (aligned16(src2) && ldsrc2 >= d && (ldsrc2 & 3) == 0)),
               "bbgr_scatter_apply: tables must be 16-byte aligned, ld >= d, ld % 4 == 0");
  hipStream_t st = as_stream(stream);
  const size_t a = align_up(4 * (size_t)n);
  const char *ws = static_cast<const char *>(plan);
  const unsigned *k2 = reinterpret_cast<const unsigned *>(ws + a);
  const int *v2 = reinterpret_cast<const int *>(ws + 3 * a);
  const unsigned grid = (unsigned)((n + 15) / 16);
#define BBGR_SEGMENTS(DD)                                                                        \
  hipLaunchKernelGGL(scatter_segments_kernel<DD>, dim3(grid), dim3(256), 0, st, (long)n, k2, v2, \
                     src, (long)ldsrc, src2, (long)ldsrc2, dst, (long)lddst, (unsigned)n_dst)
  switch (d) {
    case 8: BBGR_SEGMENTS(8); break;
    case 16: BBGR_SEGMENTS(16); break;
    case 32: BBGR_SEGMENTS(32); break;
    case 64: BBGR_SEGMENTS(64); break;
    case 128: BBGR_SEGMENTS(128); break;
    default: BBGR_SEGMENTS(256); break;
  }
#undef BBGR_SEGMENTS
  BBGR_LAUNCHED("scatter_segments_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_scatter_add_rows(int64_t n, const int64_t *idx, const float *src,
                                     int64_t ldsrc, float *dst, int64_t lddst, int32_t d,
                                     int64_t n_dst, void *workspace, size_t *workspace_bytes,
                                     bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0 && n < (1ll << 31) && n_dst >= 0 && n_dst < 0xFFFFFFFFll && workspace_bytes,
               "bbgr_scatter_add_rows: bad sizes");
  if (!supported_width(d)) {
    set_error("bbgr_scatter_add_rows: d = %d unsupported (8, 16, 32, 64, 128, 256)", d);
    return BBGR_ERR_UNSUPPORTED;
  }
  const size_t need = scatter_plan_bytes(n, n_dst, nullptr, nullptr, as_stream(stream));
  if (!workspace) {
    *workspace_bytes = need;
    return BBGR_OK;
  }
  if (*workspace_bytes < need) {
    set_error("bbgr_scatter_add_rows: workspace %zu < %zu bytes", *workspace_bytes, need);
    return BBGR_ERR_WORKSPACE;
  }
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(idx && src && dst, "bbgr_scatter_add_rows: null arrays");
  BBGR_REQUIRE(aligned16(src) && aligned16(dst) && ldsrc >= d && lddst >= d &&
                   (ldsrc & 3) == 0 && (lddst & 3) == 0,
               "bbgr_scatter_add_rows: tables must be 16-byte aligned, ld >= d, ld % 4 == 0");
  size_t have = *workspace_bytes;
  const int rc = bbgr_scatter_plan(n, idx, n_dst, workspace, &have, stream);
  if (rc != BBGR_OK) return rc;
  return bbgr_scatter_apply(n, n_dst, workspace, src, ldsrc, nullptr, 0, dst, lddst, d, stream);
}

extern "C" int bbgr_bpr(const bbgr_bpr_args *a, bbgr_stream_t stream) {
  BBGR_REQUIRE(a, "bbgr_bpr: null args");
  BBGR_REQUIRE(a->batch >= 0, "bbgr_bpr: negative batch");
  if (a->batch == 0) return BBGR_OK;
  const int d = a->d;
  if (!supported_width(d)) {
    set_error("bbgr_bpr: embedding dim %d unsupported (8, 16, 32, 64, 128, 256)", d);
    return BBGR_ERR_UNSUPPORTED;
  }
  BBGR_REQUIRE(a->users && a->pos && a->neg && a->uf && a->itf,
               "bbgr_bpr: null index/table");
  BBGR_REQUIRE(a->n_users > 0 && a->n_items > 0, "bbgr_bpr: n_users/n_items must be set");
  const bool need_reg = a->parts || a->g_ue || a->g_ie || a->scores_out;
  BBGR_REQUIRE(!need_reg || (a->ue && a->ie), "bbgr_bpr: ego tables required");
  BBGR_REQUIRE(!(a->scores_out && a->scores), "bbgr_bpr: scores_out and scores exclude each other");
  BprParams P;
  P.batch = a->batch;
  P.n_users = a->n_users;
  P.n_items = a->n_items;
  P.users = (const long *)a->users;
  P.pos = (const long *)a->pos;
  P.neg = (const long *)a->neg;
  P.uf = a->uf; P.lduf = a->lduf;
  P.itf = a->itf; P.ldif = a->ldif;
  P.ue = a->ue; P.ldue = a->ldue;
  P.ie = a->ie; P.ldie = a->ldie;
  P.pop = a->pop;
  P.reg = a->reg;
  P.lambda_fair = a->lambda_fair;
  P.inv_b = 1.0f / (float)a->batch;
  P.parts = a->parts;
  P.dloss = a->dloss;
  P.g_uf = a->g_uf; P.ldguf = a->ldguf;
  P.g_if = a->g_if; P.ldgif = a->ldgif;
  P.g_ue = a->g_ue; P.ldgue = a->ldgue;
  P.g_ie = a->g_ie; P.ldgie = a->ldgie;
  P.contrib = a->contrib; P.ldc = a->ldcontrib;
  P.scores_out = a->scores_out;
  P.scores = a->scores;
  const long lds[] = {P.lduf, P.ldif, P.ldue, P.ldie, P.ldguf, P.ldgif, P.ldgue, P.ldgie, P.ldc};
  const void *ptrs[] = {P.uf, P.itf, P.ue, P.ie, P.g_uf, P.g_if, P.g_ue, P.g_ie, P.contrib};
  for (int k = 0; k < 9; ++k) {
    if (!ptrs[k]) continue;
    BBGR_REQUIRE(aligned16(ptrs[k]) && lds[k] >= d && (lds[k] & 3) == 0,
                 "bbgr_bpr: tables must be 16-byte aligned with ld >= d, ld % 4 == 0");
  }
  const unsigned grid = (unsigned)((a->batch + 15) / 16);
  hipStream_t st = as_stream(stream);
  switch (d) {
    case 8: hipLaunchKernelGGL(bpr_kernel<8>, dim3(grid), dim3(256), 0, st, P); break;
    case 16: hipLaunchKernelGGL(bpr_kernel<16>, dim3(grid), dim3(256), 0, st, P); break;
    case 32: hipLaunchKernelGGL(bpr_kernel<32>, dim3(grid), dim3(256), 0, st, P); break;
    case 64: hipLaunchKernelGGL(bpr_kernel<64>, dim3(grid), dim3(256), 0, st, P); break;
    case 128: hipLaunchKernelGGL(bpr_kernel<128>, dim3(grid), dim3(256), 0, st, P); break;
    default: hipLaunchKernelGGL(bpr_kernel<256>, dim3(grid), dim3(256), 0, st, P); break;
  }
  BBGR_LAUNCHED("bpr_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_bpr_reduce(int64_t batch, const float *parts, float reg,
                               float lambda_fair, float *loss,
                               bbgr_stream_t stream) {
  BBGR_REQUIRE(batch > 0 && parts && loss, "bbgr_bpr_reduce: bad args");
  hipLaunchKernelGGL(bpr_reduce_kernel, dim3(1), dim3(256), 0, as_stream(stream),
                     (long)batch, parts, reg, lambda_fair, loss);
  BBGR_LAUNCHED("bpr_reduce_kernel");
  return BBGR_OK;
}

static int adam_launch(int64_t n, float *param, const float *grad, float *exp_avg,
                       float *exp_avg_sq, float lr, float beta1, float beta2, float eps,
                       float weight_decay, float grad_scale, float bias_correction1,
                       float bias_correction2_sqrt, const float *bc, const long *state,
                       hipStream_t st) {
  const AdamConsts c = adam_consts(lr, beta1, beta2, eps, weight_decay, bias_correction1,
                                   bias_correction2_sqrt);
  const bool vec = aligned16(param) && aligned16(grad) && aligned16(exp_avg) &&
                   aligned16(exp_avg_sq);
  const long n4 = vec ? n / 4 : 0;
  if (n4 > 0) {
    long blocks = (n4 + 256 * ADAM_TILE - 1) / (256 * ADAM_TILE);
    if (blocks > (1L << 30)) blocks = 1L << 30;   // the kernel strides past it
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, st, n4,
                       (float4 *)param, (const float4 *)grad, (float4 *)exp_avg,
                       (float4 *)exp_avg_sq, c, grad_scale, lr, bc, state);
    BBGR_LAUNCHED("adam_kernel");
  }
  const long start = n4 * 4;
  if (start < n) {
    hipLaunchKernelGGL(adam_tail_kernel, dim3((unsigned)((n - start + 255) / 256)),
                       dim3(256), 0, st, (long)n, start, param, grad, exp_avg,
                       exp_avg_sq, c, grad_scale, lr, bc, state);
    BBGR_LAUNCHED("adam_tail_kernel");
  }
  return BBGR_OK;
}

extern "C" int bbgr_adam(int64_t n, float *param, const float *grad,
                         float *exp_avg, float *exp_avg_sq, float lr, float beta1,
                         float beta2, float eps, float weight_decay, float grad_scale,
                         float bias_correction1, float bias_correction2_sqrt,
                         bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0, "bbgr_adam: negative n");
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(param && grad && exp_avg && exp_avg_sq, "bbgr_adam: null tensor");
  return adam_launch(n, param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay,
                     grad_scale, bias_correction1, bias_correction2_sqrt, nullptr, nullptr,
                     as_stream(stream));
}

extern "C" int bbgr_adam_dev(int64_t n, float *param, const float *grad, float *exp_avg,
                             float *exp_avg_sq, float lr, float beta1, float beta2,
                             float eps, float weight_decay, float grad_scale,
                             const float *bc_table, const int64_t *state,
                             bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0, "bbgr_adam_dev: negative n");
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(param && grad && exp_avg && exp_avg_sq && bc_table && state,
               "bbgr_adam_dev: null tensor / table / state");
  return adam_launch(n, param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay,
                     grad_scale, 1.f, 1.f, bc_table, (const long *)state, as_stream(stream));
}

extern "C" int bbgr_step_begin(int64_t *state, bbgr_stream_t stream) {
  BBGR_REQUIRE(state, "bbgr_step_begin: null state");
  hipLaunchKernelGGL(step_begin_kernel, dim3(1), dim3(64), 0, as_stream(stream), (long *)state);
  BBGR_LAUNCHED("step_begin_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_rows_zero(int64_t n, const int64_t *idx, float *table,
                              int64_t ld, int32_t d, bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0 && d > 0 && ld >= d, "bbgr_rows_zero: bad sizes");
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(idx && table, "bbgr_rows_zero: null arrays");
  hipLaunchKernelGGL(rows_zero_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0,
                     as_stream(stream), (long)n, (const long *)idx, table, (long)ld, d);
  BBGR_LAUNCHED("rows_zero_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_mark_rows(int64_t n, const int64_t *idx, uint8_t value,
                              uint8_t *mask, int64_t n_rows, bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0 && n_rows >= 0, "bbgr_mark_rows: negative n / n_rows");
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(idx && mask, "bbgr_mark_rows: null arrays");
  hipLaunchKernelGGL(mark_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     as_stream(stream), (long)n, (const long *)idx, value, mask, (long)n_rows);
  BBGR_LAUNCHED("mark_rows_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_mark_neighbors(int64_t n, const int64_t *rows,
                                   const int32_t *indptr, const int32_t *indices,
                                   uint8_t value, uint8_t *mask, bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0, "bbgr_mark_neighbors: negative n");
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(rows && indptr && indices && mask, "bbgr_mark_neighbors: null arrays");
  hipLaunchKernelGGL(mark_neighbors_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0,
                     as_stream(stream), (long)n, (const long *)rows, indptr, indices, value,
                     mask);
  BBGR_LAUNCHED("mark_neighbors_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_mark_list(int64_t n, const int64_t *rows, const int32_t *indptr,
                              const int32_t *indices, uint8_t *mask, int64_t n_rows,
                              int64_t *list, int64_t *count, bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0 && n_rows >= 0, "bbgr_mark_list: negative n / n_rows");
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(rows && mask && list && count && (!indptr || indices),
               "bbgr_mark_list: null arrays");
  BBGR_REQUIRE(((uintptr_t)mask & 3) == 0, "bbgr_mark_list: mask must be 4-byte aligned");
  hipStream_t st = as_stream(stream);
  if (!indptr) {
    hipLaunchKernelGGL(mark_list_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       st, (long)n, (const long *)rows, mask, (long)n_rows, (long *)list,
                       (unsigned long long *)count);
    BBGR_LAUNCHED("mark_list_rows_kernel");
  } else {
    hipLaunchKernelGGL(mark_list_neighbors_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256),
                       0, st, (long)n, (const long *)rows, indptr, indices, mask, (long *)list,
                       (unsigned long long *)count);
    BBGR_LAUNCHED("mark_list_neighbors_kernel");
  }
  return BBGR_OK;
}

extern "C" int bbgr_mark_slots(int64_t n, const int64_t *rows, const int32_t *indptr,
                               const int32_t *tmap, uint32_t *bits, int32_t set,
                               bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0, "bbgr_mark_slots: negative n");
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(rows && indptr && tmap && bits, "bbgr_mark_slots: null arrays");
  hipLaunchKernelGGL(mark_slots_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0,
                     as_stream(stream), (long)n, (const long *)rows, indptr, tmap, bits, (int)set);
  BBGR_LAUNCHED("mark_slots_kernel");
  return BBGR_OK;
}

// one thread per 32-bit word: 32 byte loads as eight 4-byte loads
__global__ __launch_bounds__(256) void mask_pack_kernel(long n, const unsigned char *mask,
                                                        unsigned *bits) {
  const long w = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long b0 = w * 32;
  if (b0 >= n) return;
  unsigned v = 0;
  if (b0 + 32 <= n && (reinterpret_cast<uintptr_t>(mask) & 3) == 0) {
    const unsigned *q = reinterpret_cast<const unsigned *>(mask + b0);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const unsigned x = q[k];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if ((x >> (8 * j)) & 0xffu) v |= 1u << (4 * k + j);
    }
  } else {
    for (int j = 0; j < 32 && b0 + j < n; ++j)
      if (mask[b0 + j]) v |= 1u << j;
  }
  bits[w] = v;
}

extern "C" int bbgr_mask_pack(int64_t n, const uint8_t *mask, uint32_t *bits,
                              bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0, "bbgr_mask_pack: bad size");
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(mask && bits, "bbgr_mask_pack: null arrays");
  const long words = (long)((n + 31) / 32);
  hipLaunchKernelGGL(mask_pack_kernel, dim3((unsigned)((words + 255) / 256)), dim3(256), 0,
                     as_stream(stream), (long)n, mask, bits);
  BBGR_LAUNCHED("mask_pack_kernel");
  return BBGR_OK;
}

static int batch_params(const bbgr_batch_args *a, BatchParams &P) {
  BBGR_REQUIRE(a && a->batch >= 0 && a->n_users > 0 && a->n_items > 0, "bbgr_batch: bad sizes");
  BBGR_REQUIRE(a->batch == 0 || (a->users && a->pos && a->neg && a->mask_u && a->mask_i),
               "bbgr_batch: null arrays");
  BBGR_REQUIRE(!a->user_indptr == !a->user_indices, "bbgr_batch: user CSR half given");
  BBGR_REQUIRE(!a->list == !a->count, "bbgr_batch: list and count go together");
  BBGR_REQUIRE(!a->slot_bits == !a->slot_map && (!a->slot_bits || a->user_indptr),
               "bbgr_batch: slot_bits needs slot_map and the user CSR");
  BBGR_REQUIRE(!(a->g_u || a->g_i || a->g_side) || (a->d > 0 && a->d % 4 == 0),
               "bbgr_batch: gradient rows need d % 4 == 0");
  for (const float *t : {a->g_u, a->g_i, a->g_side})
    BBGR_REQUIRE(!t || aligned16(t), "bbgr_batch: gradient tables must be 16-byte aligned");
  BBGR_REQUIRE((a->ld_gu & 3) == 0 && (a->ld_gi & 3) == 0 && (a->ld_side & 3) == 0,
               "bbgr_batch: ld % 4 == 0");
  P.B = a->batch;
  P.U = a->n_users;
  P.I = a->n_items;
  P.users = (const long *)a->users;
  P.pos = (const long *)a->pos;
  P.neg = (const long *)a->neg;
  P.indptr = a->user_indptr;
  P.indices = a->user_indices;
  P.mask_u = a->mask_u;
  P.mask_i = a->mask_i;
  P.list = (long *)a->list;
  P.count = (unsigned long long *)a->count;
  P.tmap = a->slot_map;
  P.bits = a->slot_bits;
  P.g_u = a->g_u;
  P.g_i = a->g_i;
  P.g_side = a->g_side;
  P.ld_gu = a->ld_gu;
  P.ld_gi = a->ld_gi;
  P.ld_side = a->ld_side;
  P.d = a->d;
  return BBGR_OK;
}

extern "C" int bbgr_batch_begin(const bbgr_batch_args *a, bbgr_stream_t stream) {
  BatchParams P;
  if (int rc = batch_params(a, P)) return rc;
  if (P.B == 0) return BBGR_OK;
  hipLaunchKernelGGL(batch_begin_kernel, dim3((unsigned)((P.B + 15) / 16)), dim3(256), 0,
                     as_stream(stream), P);
  BBGR_LAUNCHED("batch_begin_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_rows_mark(const bbgr_rows_mark_args *a, bbgr_stream_t stream) {
  BBGR_REQUIRE(a && a->n_users_listed >= 0 && a->n_items_listed >= 0 && a->n_users > 0 &&
                   a->n_items > 0,
               "bbgr_rows_mark: bad sizes");
  if (a->n_users_listed == 0 && a->n_items_listed == 0) return BBGR_OK;
  BBGR_REQUIRE((a->n_users_listed == 0 || (a->users && a->mask_u && a->user_list &&
                                           a->user_count)) &&
                   (a->n_items_listed == 0 || (a->items && a->mask_i)) && a->frontier &&
                   a->frontier_list && a->frontier_count,
               "bbgr_rows_mark: null arrays");
  BBGR_REQUIRE(!a->user_indptr || a->user_indices, "bbgr_rows_mark: user CSR half given");
  BBGR_REQUIRE(((uintptr_t)a->frontier & 3) == 0 && ((uintptr_t)a->mask_u & 3) == 0,
               "bbgr_rows_mark: mask_u / frontier must be 4-byte aligned");
  RowsMarkParams P;
  P.nu = a->n_users_listed;
  P.ni = a->n_items_listed;
  P.U = a->n_users;
  P.I = a->n_items;
  P.users = (const long *)a->users;
  P.items = (const long *)a->items;
  P.urank = (const long *)a->user_rank;
  P.irank = (const long *)a->item_rank;
  P.indptr = a->user_indptr;
  P.indices = a->user_indices;
  P.mu = a->mask_u;
  P.mi = a->mask_i;
  P.fr = a->frontier;
  P.mu_in = a->mask_u_in;
  P.mi_in = a->mask_i_in;
  P.ulist = (long *)a->user_list;
  P.flist = (long *)a->frontier_list;
  P.ucount = (unsigned long long *)a->user_count;
  P.fcount = (unsigned long long *)a->frontier_count;
  const long groups = P.nu > (P.ni + 3) / 4 ? P.nu : (P.ni + 3) / 4;
  hipLaunchKernelGGL(rows_mark_kernel, dim3((unsigned)((groups + 15) / 16)), dim3(256), 0,
                     as_stream(stream), P);
  BBGR_LAUNCHED("rows_mark_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_batch_end(const bbgr_batch_args *a, bbgr_stream_t stream) {
  BatchParams P;
  if (int rc = batch_params(a, P)) return rc;
  if (P.B == 0 && !P.count) return BBGR_OK;
  const long blocks = P.B > 0 ? (P.B + 15) / 16 : 1;   // (B == 0: the count reset alone)
  hipLaunchKernelGGL(batch_end_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream),
                     P);
  BBGR_LAUNCHED("batch_end_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_mark_neighbors_of_mask(int64_t n_rows, const uint8_t *row_mask,
                                           const int32_t *row_map, const int32_t *indptr,
                                           const int32_t *indices, uint8_t value,
                                           uint8_t *mask, bbgr_stream_t stream) {
  BBGR_REQUIRE(n_rows >= 0, "bbgr_mark_neighbors_of_mask: negative n_rows");
  if (n_rows == 0) return BBGR_OK;
  BBGR_REQUIRE(row_mask && indptr && indices && mask,
               "bbgr_mark_neighbors_of_mask: null arrays");
  hipLaunchKernelGGL(mark_neighbors_of_mask_kernel, dim3((unsigned)((n_rows + 15) / 16)),
                     dim3(256), 0, as_stream(stream), (long)n_rows, row_mask, row_map, indptr,
                     indices, value, mask);
  BBGR_LAUNCHED("mark_neighbors_of_mask_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_row_support(int64_t n_rows, int32_t d, const float *x, int64_t ldx,
                                uint8_t *mask, const int32_t *indptr, const int32_t *indices,
                                uint8_t *nbr_mask, bbgr_stream_t stream) {
  BBGR_REQUIRE(n_rows >= 0 && d > 0 && ldx >= d, "bbgr_row_support: bad sizes");
  if (n_rows == 0) return BBGR_OK;
  BBGR_REQUIRE(x && mask, "bbgr_row_support: null arrays");
  BBGR_REQUIRE(!indptr || (indices && nbr_mask), "bbgr_row_support: CSR without indices / nbr_mask");
  const bool vec = d % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)x & 15) == 0;
  const dim3 grid((unsigned)((n_rows + 15) / 16));
  if (vec)
    hipLaunchKernelGGL(row_support_kernel<true>, grid, dim3(256), 0, as_stream(stream),
                       (long)n_rows, (int)d, x, (long)ldx, mask, indptr, indices, nbr_mask);
  else
    hipLaunchKernelGGL(row_support_kernel<false>, grid, dim3(256), 0, as_stream(stream),
                       (long)n_rows, (int)d, x, (long)ldx, mask, indptr, indices, nbr_mask);
  BBGR_LAUNCHED("row_support_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_rows_axpy(int64_t n, const int64_t *idx, float alpha,
                              const float *src, int64_t ldsrc, float *dst,
                              int64_t lddst, int32_t d, bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0 && d > 0 && ldsrc >= d && lddst >= d, "bbgr_rows_axpy: bad sizes");
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(idx && src && dst, "bbgr_rows_axpy: null arrays");
  hipLaunchKernelGGL(rows_axpy_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0,
                     as_stream(stream), (long)n, (const long *)idx, alpha, src,
                     (long)ldsrc, dst, (long)lddst, d);
  BBGR_LAUNCHED("rows_axpy_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_first_slot(int64_t n, const int64_t *ids, int64_t n_rows, int32_t *first,
                               int64_t *slot, bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0 && n < (1LL << 31) && n_rows >= 0, "bbgr_first_slot: bad sizes");
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(ids && first && slot, "bbgr_first_slot: null arrays");
  hipStream_t st = as_stream(stream);
  const unsigned g = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(first_slot_min_kernel, dim3(g), dim3(256), 0, st, (long)n,
                     (const long *)ids, (long)n_rows, first);
  BBGR_LAUNCHED("first_slot_min_kernel");
  hipLaunchKernelGGL(first_slot_read_kernel, dim3(g), dim3(256), 0, st, (long)n,
                     (const long *)ids, (long)n_rows, (const int *)first, (long *)slot);
  BBGR_LAUNCHED("first_slot_read_kernel");
  hipLaunchKernelGGL(first_slot_reset_kernel, dim3(g), dim3(256), 0, st, (long)n,
                     (const long *)ids, (long)n_rows, first);
  BBGR_LAUNCHED("first_slot_reset_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_ego_slots(int64_t B, const int64_t *users, const int64_t *pos,
                              const int64_t *neg, int64_t n_users, int64_t n_items,
                              int32_t *first_u, int32_t *first_i, int64_t *iu, int64_t *ii,
                              int64_t *cu, int64_t *sp, int64_t *sn, bbgr_stream_t stream) {
  BBGR_REQUIRE(B >= 0 && 3 * B < (1LL << 31) && n_users > 0 && n_items > 0,
               "bbgr_ego_slots: bad sizes");
  if (B == 0) return BBGR_OK;
  BBGR_REQUIRE(users && pos && neg && first_u && first_i && iu && ii && cu && sp && sn,
               "bbgr_ego_slots: null arrays");
  hipStream_t st = as_stream(stream);
  const unsigned g = (unsigned)((3 * B + 255) / 256);
  const long *u = (const long *)users, *p = (const long *)pos, *n = (const long *)neg;
  hipLaunchKernelGGL(ego_slots_min_kernel, dim3(g), dim3(256), 0, st, (long)B, u, p, n,
                     (long)n_users, (long)n_items, first_u, first_i, (long *)iu, (long *)ii);
  BBGR_LAUNCHED("ego_slots_min_kernel");
  hipLaunchKernelGGL(ego_slots_read_kernel, dim3(g), dim3(256), 0, st, (long)B, u, p, n,
                     (long)n_users, (long)n_items, (const int *)first_u, (const int *)first_i,
                     (const long *)iu, (const long *)ii, (long *)cu, (long *)sp, (long *)sn);
  BBGR_LAUNCHED("ego_slots_read_kernel");
  hipLaunchKernelGGL(ego_slots_reset_kernel, dim3(g), dim3(256), 0, st, (long)B, first_u,
                     first_i, (const long *)iu, (const long *)ii);
  BBGR_LAUNCHED("ego_slots_reset_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_ego_rows(int64_t B, int32_t d, const int64_t *cu, const int64_t *sp,
                             const int64_t *sn, const int64_t *iu, const int64_t *ii,
                             const float *ue, int64_t ldue, const float *ie, int64_t ldie,
                             const float *dloss, float reg, int32_t *counts, float *g_u,
                             int64_t ldgu, float *g_i, int64_t ldgi, float scale,
                             int32_t *counts_u_out, bbgr_stream_t stream) {
  BBGR_REQUIRE(B >= 0 && 3 * B < (1LL << 31), "bbgr_ego_rows: bad batch");
  if (d != 64 && d != 128 && d != 256) {
    set_error("bbgr_ego_rows: embedding dim %d unsupported (64, 128, 256)", d);
    return BBGR_ERR_UNSUPPORTED;
  }
  if (B == 0) return BBGR_OK;
  BBGR_REQUIRE(cu && sp && sn && iu && ii && ue && ie && counts && g_u && g_i,
               "bbgr_ego_rows: null arrays");
  BBGR_REQUIRE(aligned16(ue) && aligned16(ie) && aligned16(g_u) && aligned16(g_i) &&
                   (ldue & 3) == 0 && (ldie & 3) == 0 && (ldgu & 3) == 0 && (ldgi & 3) == 0,
               "bbgr_ego_rows: tables must be 16-byte aligned, ld % 4 == 0");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(ego_count_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st,
                     (long)B, (const long *)cu, (const long *)sp, (const long *)sn, counts);
  BBGR_LAUNCHED("ego_count_kernel");
  const dim3 g((unsigned)((3 * B + 15) / 16));
  const float inv_b = 1.0f / (float)B;
#define BBGR_EGO_ROWS(DD)                                                                   \
  hipLaunchKernelGGL(ego_rows_kernel<DD>, g, dim3(256), 0, st, (long)B, (const long *)iu, \
                     (const long *)ii, ue, (long)ldue, ie, (long)ldie, dloss, inv_b, reg,   \
                     counts, g_u, (long)ldgu, g_i, (long)ldgi, scale, counts_u_out)
  switch (d) {
    case 64: BBGR_EGO_ROWS(64); break;
    case 128: BBGR_EGO_ROWS(128); break;
    default: BBGR_EGO_ROWS(256); break;
  }
#undef BBGR_EGO_ROWS
  BBGR_LAUNCHED("ego_rows_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_graph_rows(int64_t n, const int64_t *ids, int64_t n_rows, const int64_t *rank,
                               int64_t *out, bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0 && n_rows >= 0, "bbgr_graph_rows: bad sizes");
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(ids && out, "bbgr_graph_rows: null arrays");
  hipLaunchKernelGGL(graph_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     as_stream(stream), (long)n, (const long *)ids, (long)n_rows,
                     (const long *)rank, (long *)out);
  BBGR_LAUNCHED("graph_rows_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_rows_copy(int64_t n, const int64_t *idx, const float *src,
                              int64_t ldsrc, float *dst, int64_t lddst, int32_t d,
                              bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0 && d > 0 && (d & 3) == 0 && ldsrc >= d && lddst >= d &&
                   (ldsrc & 3) == 0 && (lddst & 3) == 0,
               "bbgr_rows_copy: bad sizes (d, ld multiples of 4, ld >= d)");
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(idx && src && dst && aligned16(src) && aligned16(dst),
               "bbgr_rows_copy: null or unaligned arrays");
  hipLaunchKernelGGL(rows_copy_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0,
                     as_stream(stream), (long)n, (const long *)idx,
                     reinterpret_cast<const float4 *>(src), (long)ldsrc / 4,
                     reinterpret_cast<float4 *>(dst), (long)lddst / 4, d / 4);
  BBGR_LAUNCHED("rows_copy_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_rows_add_unique(int64_t n, const int64_t *idx, const float *src,
                                    int64_t ldsrc, float *dst, int64_t lddst, int32_t d,
                                    int64_t n_dst, bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0 && n_dst >= 0 && d > 0 && (d & 3) == 0 && ldsrc >= d && lddst >= d &&
                   (ldsrc & 3) == 0 && (lddst & 3) == 0,
               "bbgr_rows_add_unique: bad sizes (d, ld multiples of 4, ld >= d)");
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(idx && src && dst && aligned16(src) && aligned16(dst),
               "bbgr_rows_add_unique: null or unaligned arrays");
  hipLaunchKernelGGL(rows_add_unique_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0,
                     as_stream(stream), (long)n, (const long *)idx,
                     reinterpret_cast<const float4 *>(src), (long)ldsrc / 4,
                     reinterpret_cast<float4 *>(dst), (long)lddst / 4, d / 4, (long)n_dst);
  BBGR_LAUNCHED("rows_add_unique_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_rows_add_slots(int64_t n, const int64_t *slot, const int32_t *counts,
                                   const int64_t *rows, const float *src, int64_t ldsrc,
                                   float *dst, int64_t lddst, int32_t d, int64_t n_dst,
                                   bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0 && n_dst >= 0 && d > 0 && (d & 3) == 0 && ldsrc >= d && lddst >= d &&
                   (ldsrc & 3) == 0 && (lddst & 3) == 0,
               "bbgr_rows_add_slots: bad sizes (d, ld multiples of 4, ld >= d)");
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(slot && counts && rows && src && dst && aligned16(src) && aligned16(dst),
               "bbgr_rows_add_slots: null or unaligned arrays");
  hipLaunchKernelGGL(rows_add_slots_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0,
                     as_stream(stream), (long)n, (const long *)slot, counts, (const long *)rows,
                     reinterpret_cast<const float4 *>(src), (long)ldsrc / 4,
                     reinterpret_cast<float4 *>(dst), (long)lddst / 4, d / 4, (long)n_dst);
  BBGR_LAUNCHED("rows_add_slots_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_rows_gather(int64_t n, const int64_t *idx, const float *src,
                                int64_t ldsrc, float *dst, int64_t lddst, int32_t d,
                                bbgr_stream_t stream) {
  BBGR_REQUIRE(n >= 0 && d > 0 && (d & 3) == 0 && ldsrc >= d && lddst >= d &&
                   (ldsrc & 3) == 0 && (lddst & 3) == 0,
               "bbgr_rows_gather: bad sizes (d, ld multiples of 4, ld >= d)");
  if (n == 0) return BBGR_OK;
  BBGR_REQUIRE(idx && src && dst && aligned16(src) && aligned16(dst),
               "bbgr_rows_gather: null or unaligned arrays");
  hipLaunchKernelGGL(rows_gather_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0,
                     as_stream(stream), (long)n, (const long *)idx,
                     reinterpret_cast<const float4 *>(src), (long)ldsrc / 4,
                     reinterpret_cast<float4 *>(dst), (long)lddst / 4, d / 4);
  BBGR_LAUNCHED("rows_gather_kernel");
  return BBGR_OK;
}
