// Fused CSR-SpMM for the LightGCN propagation (gfx950).
//
// Replaces torch.sparse.mm(M, X) at Version-2/lighgcn_cu_pop.py:483-484,
// lightgcn_cu.py:431,434, lightgcn.py:323 (and the autograd backward of each,
// which is the same product on the transposed CSR), fused with the layer-mean
// accumulation of Version-2/lighgcn_cu_pop.py:488-489.
//
// Work decomposition (HBM/gather-bound, no MFMA):
//   * one 16-lane group owns one output row; each lane holds D/64 float4 of the
//     row, so a group reads a whole source row (D*4 bytes) with one coalesced
//     16-B-per-lane load per float4 column block; a wave gathers 4 rows per
//     load instruction and keeps 16/V rows in flight per group.
//   * rows with deg > long_threshold are cut into chunks of <= chunk_edges
//     edges; each chunk is one 256-thread workgroup (16 groups on contiguous
//     edge sub-ranges, fixed-order LDS reduction). Chunk blocks come first in
//     the grid so the heavy (power-law) rows start early.
//   * rows cut into >1 chunk write per-chunk partials (write-through) and take
//     an arrival ticket; the last-arriving chunk workgroup of the row sums the
//     partials in chunk order and runs the epilogue, inside the same launch.
//     Every reduction order is fixed: the result is bitwise deterministic (no
//     floating-point atomics).
#include <stdarg.h>
#include <stdlib.h>

#include <cstring>

#include "common.h"

namespace bbgr {

struct SpmmParams {
  int n_rows;
  int long_threshold;
  int n_chunks;
  const int *indptr;
  const int *indices;
  const int4 *chunks;
  const int4 *split;
  const float *x;
  long ldx;
  const float *edge_val;
  const float *col_scale;
  float col_scale_s;
  float *y;
  long ldy;
  const float *y_scale;
  float y_scale_s;
  const float *add;
  long ldadd;
  const float *add_scale;
  float add_scale_s;
  const float *acc_in;
  long ldacc_in;
  float *acc_out;
  long ldacc_out;
  const float *acc_scale;
  float acc_scale_s;
  float gamma;
  float *partial;
  const unsigned char *src_mask;
  const unsigned char *row_mask;
  const unsigned char *acc_mask;
  const unsigned char *add_mask;
  const long *row_list;
  long n_row_list;
  int row_begin, row_end;      // short rows computed: [row_begin, row_end)
  int pair_rows;               // two short rows per 16-lane group (gather_pair)
  int chunk_begin;             // first long-row chunk of this launch
  int nt_from;                 // source rows >= nt_from: streaming loads (args.stream_from)
  int nt_out_from;             // output rows >= nt_out_from: streaming stores (args.stream_out_from)
  int chunk_edges;             // plan chunk size (a split row has ceil(deg / chunk_edges) chunks)
  int *arrivals;               // per-chunk arrival counters (after the partials), zero between launches
  // fused Adam on the y-row value (bbgr_spmm_args.adam_*)
  float *adam_p, *adam_m, *adam_v;
  long adam_ld;
  AdamConsts adam;
  float adam_lr;
  const float *adam_bc;        // device step state (nullable): bias corrections by step t
  const long *adam_state;
  // row maps of the epilogue's tables (nullable; args.y_map / acc_map / add_map):
  // CSR row r reads / writes row map[r] of y (and the fused Adam's rows), of
  // acc_in / acc_out, of add; the masks of those tables index the same rows
  const int *y_map, *acc_map, *add_map;
  const int *acc_in_map;       // acc_in's own row map (args.acc_in_map; NULL: acc_map's)
  const unsigned *src_bits;    // slot bitmap of live edges (args.src_bits; d >= 64)
  const long *row_count;       // device length of row_list (args.row_count; nullable)
  const float *adam_g;         // fused Adam's own gradient table (args.adam_grad; nullable)
  long adam_g_ld;
  float adam_g_scale;
  const int *adam_map;         // the fused Adam's row map (args.adam_map; NULL: y_map's)
  int adam_mrow;               // moments at the launch row (args.adam_moments_unmapped)
  int *tag_out;                // tagged-index copy written by a full launch (args.tag_out)
  const unsigned char *tag_mask;
  float *adam_mirror;          // caller-order copy of the updated param rows (args.adam_mirror)
  const unsigned *src_mask_bits;   // src_mask packed one bit per row (args.src_mask_bits)
};

// Per-edge liveness of source row c. The packed form (bbgr_mask_pack) puts 1024
// rows in a 128-B line instead of 128: the degree-ordered hub columns most
// edges point at share a few lines, so a wave's 64 lookups need fewer L2
// requests and hit L1 more often. Same liveness, so bitwise the byte test.
__device__ __forceinline__ bool src_live(const SpmmParams &P, int c) {
  if (P.src_mask_bits) return (P.src_mask_bits[c >> 5] >> (c & 31)) & 1u;
  return P.src_mask[c] != 0;
}

// src_live for two lanes' sources at once (a, b < 0: no edge): both loads are
// issued before either result is used; a dead source becomes -1
__device__ __forceinline__ void src_live2(const SpmmParams &P, int &a, int &b) {
  if (P.src_mask_bits) {
    const unsigned wa = a >= 0 ? P.src_mask_bits[a >> 5] : 0u;
    const unsigned wb = b >= 0 ? P.src_mask_bits[b >> 5] : 0u;
    if (!((wa >> (a & 31)) & 1u)) a = -1;
    if (!((wb >> (b & 31)) & 1u)) b = -1;
  } else {
    const unsigned char ma = a >= 0 ? P.src_mask[a] : (unsigned char)0;
    const unsigned char mb = b >= 0 ? P.src_mask[b] : (unsigned char)0;
    if (!ma) a = -1;
    if (!mb) b = -1;
  }
}

// Tagged column indices (ABI 10): a full launch over a CSR can write a copy of
// its column indices with bit 31 set where the column is dead in tag_mask
// (TAG_WRITE); a masked launch over the same CSR then reads liveness from the
// index itself (TAG_READ: indices = the copy, no src_mask load), which takes
// the mask byte's dependent load out of every batch's index -> gather chain.
constexpr int TAG_NONE = 0, TAG_WRITE = 1, TAG_READ = 2;

// The writer loads the mask byte of an edge's column right after the index
// and stores the tagged index only after the batch's gathers are issued, so
// the dependent mask load never stalls the gather chain (stored before the
// gathers, its wait exposed an L2 round trip per batch: +0.26 ms per C4 user
// product). col < 0: no edge in this lane.
__device__ __forceinline__ int tag_of(const SpmmParams &P, int col) {
  return col < 0 ? 0 : (int)P.tag_mask[col];
}
__device__ __forceinline__ void tag_store(const SpmmParams &P, long e, int col, int live) {
  __builtin_nontemporal_store(live ? col : (int)((unsigned)col | 0x80000000u), P.tag_out + e);
}

__device__ __forceinline__ float4 f4_fma(float a, float4 x, float4 y) {
  return make_float4(fmaf(a, x.x, y.x), fmaf(a, x.y, y.y), fmaf(a, x.z, y.z),
                     fmaf(a, x.w, y.w));
}
__device__ __forceinline__ float4 f4_add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 f4_mul(float a, float4 x) {
  return make_float4(a * x.x, a * x.y, a * x.z, a * x.w);
}

// Column indices and per-edge values are read once per launch (200 MB each at
// C4). Streaming (non-temporal) loads for them, so they would not displace
// gathered rows from L2 / the Infinity Cache, measured slower (round 4 A/B,
// tools/probes/gpu_ab_nt_index.sh: C4 step 16.72 -> 16.84 ms, masked user
// product 1.115 -> 1.136 ms on one box): default-policy loads
// (BBGR_NT_INDEX=1 builds the streamed form).
#ifndef BBGR_NT_INDEX
#define BBGR_NT_INDEX 0
#endif
template <typename T>
__device__ __forceinline__ T ld_edge(const T *p) {
  if constexpr (BBGR_NT_INDEX != 0) return ld_nt(p);
  return *p;
}

// Per-width tuning (measured with tools/ab_spmm.sh A/B builds; every value
// can be overridden with -D for such builds):
//   row_u        source rows in flight per 16-lane group, one-row kernels
//   row_waves    occupancy the one-row kernels are compiled for (0 = compiler)
//   pair_u       source rows in flight PER ROW, two-row kernels (full / masked)
//   pair_waves   occupancy of the two-row kernels (full / masked)
// d = 64: more rows in flight per CU beat deeper per-row batches.
#ifndef BBGR_ROW_U
#define BBGR_ROW_U 8
#endif
#ifndef BBGR_ROW_WAVES
#define BBGR_ROW_WAVES 0
#endif
// occupancy target of the UNWEIGHTED (WMODE 0) one-row kernels: without one
// the compiler takes 106 SGPRs, which admits only 6 workgroups per CU
// (MI355X_MICROARCH.md, residency), at 7 / 8 waves 94 / 78 SGPRs and no spill;
// the weighted forms spill at 8 (round 3's slower 8-wave A/B)
#ifndef BBGR_ROW_WAVES0
#define BBGR_ROW_WAVES0 0
#endif
// Two-row kernels at the 8-wave target hold at most 64 VGPRs: with 4 rows in
// flight per row they spilled (12 / 24 B per lane in the full / masked form,
// round 5: every 16-edge batch wrote and re-read its spill slots through L2,
// 5-12.5M extra 64-B write requests per C4 launch, TCC_WRITE 25.0M / 32.5M
// against the 20.0M of the output rows, profiles/round5/r5c_*). 2 / 3 rows in flight
// per row fit without spilling (55 / 59 VGPRs) and the many rows of a user
// table keep the CU busy anyway: C4 full user products 1.556 -> 1.47-1.48
// ms, the src-masked backward user product 1.14 -> 0.92 ms, step 17.00 ->
// 16.51-16.55 ms (profiles/round5/r5e_ab_spills.txt). The sums are unchanged bit for
// bit (each row still adds its edges in CSR order).
// tests/test_kernel_resources.py keeps every product kernel spill-free.
#ifndef BBGR_PAIR_U
#define BBGR_PAIR_U 2
#endif
#ifndef BBGR_PAIR_U_MASKED
#define BBGR_PAIR_U_MASKED 3
#endif
#ifndef BBGR_PAIR_WAVES
#define BBGR_PAIR_WAVES 0
#endif
#ifndef BBGR_PAIR_WAVES_MASKED
#define BBGR_PAIR_WAVES_MASKED 0
#endif
// the unweighted (WMODE 0) masked two-row kernel at 8 waves (59 VGPRs with 3
// rows in flight per row, no spill; round 3 measured the 8-wave target 0.984
// -> 0.886 ms for the src-masked backward user product, tools/ab_spmm.sh);
// the weighted forms keep the compiler's choice
#ifndef BBGR_PAIR_WAVES_MASKED0
#define BBGR_PAIR_WAVES_MASKED0 8
#endif
// ... and the unweighted full two-row kernel (62 -> 63 VGPRs, 7 -> 8 waves, no
// spill): C4 full user products 1.484 -> 1.451 ms per launch (round 3 A/B;
// the weighted forms spill at 8; an 8-wave target on the one-row kernels
// measured slower, item products 1.816 -> 1.829 ms)
// the unweighted d = 64 slot-bitmap kernel (spmm_bits_kernel): the 8-wave
// target spilled 16 B per lane after the single-live-edge path (round 4);
// the compiler's choice (67 VGPRs, 7 waves) measures the same 0.094-0.097 ms
#ifndef BBGR_BITS_WAVES0
#define BBGR_BITS_WAVES0 0
#endif
#ifndef BBGR_PAIR_WAVES0
#define BBGR_PAIR_WAVES0 8
#endif
// d = 128
#ifndef BBGR_ROW_U128
#define BBGR_ROW_U128 8
#endif
#ifndef BBGR_ROW_WAVES128
#define BBGR_ROW_WAVES128 0
#endif
#ifndef BBGR_PAIR_U128
#define BBGR_PAIR_U128 4
#endif
#ifndef BBGR_PAIR_WAVES128
#define BBGR_PAIR_WAVES128 0
#endif
// d = 256
#ifndef BBGR_ROW_U256
#define BBGR_ROW_U256 4
#endif
#ifndef BBGR_ROW_WAVES256
#define BBGR_ROW_WAVES256 0
#endif
#ifndef BBGR_PAIR_U256
#define BBGR_PAIR_U256 2
#endif
#ifndef BBGR_SLOT_ROUNDS32   // narrow short rows: 8-edge index rounds per load round
#define BBGR_SLOT_ROUNDS32 1
#endif
#ifndef BBGR_NARROW_WAVES32   // occupancy target of the 32-column kernels (0: none)
#define BBGR_NARROW_WAVES32 0
#endif
#ifndef BBGR_NARROW_MASKED_WAVES32   // ... of the 32-column masked kernel (no edge values)
#define BBGR_NARROW_MASKED_WAVES32 8
#endif
#ifndef BBGR_NARROW_WAVES16
#define BBGR_NARROW_WAVES16 0
#endif
#ifndef BBGR_NARROW_MASKED_WAVES16
#define BBGR_NARROW_MASKED_WAVES16 0
#endif
#ifndef BBGR_SLOT_ROUNDS16
#define BBGR_SLOT_ROUNDS16 2
#endif
#ifndef BBGR_PAIR_WAVES256
#define BBGR_PAIR_WAVES256 0
#endif

template <int D> struct Tune {   // narrow rows (8, 16, 32): one-row kernels only
  static constexpr int row_u = 0;
  static constexpr int row_waves0 = 0;
  static constexpr int row_waves = D == 32 ? BBGR_NARROW_WAVES32 : D == 16 ? BBGR_NARROW_WAVES16 : 0;
  static constexpr int masked_waves =
      D == 32 ? BBGR_NARROW_MASKED_WAVES32 : D == 16 ? BBGR_NARROW_MASKED_WAVES16 : 0;
  static constexpr int pair_u = 0, pair_u_masked = 0;
  static constexpr int pair_waves = 0, pair_waves_masked = 0, pair_waves_masked0 = 0;
  static constexpr int pair_waves0 = 0;
};
template <> struct Tune<64> {
  static constexpr int row_u = BBGR_ROW_U, row_waves = BBGR_ROW_WAVES;
  static constexpr int row_waves0 = BBGR_ROW_WAVES0;
  static constexpr int masked_waves = row_waves;
  static constexpr int pair_u = BBGR_PAIR_U, pair_u_masked = BBGR_PAIR_U_MASKED;
  static constexpr int pair_waves = BBGR_PAIR_WAVES, pair_waves_masked = BBGR_PAIR_WAVES_MASKED;
  static constexpr int pair_waves_masked0 = BBGR_PAIR_WAVES_MASKED0;
  static constexpr int pair_waves0 = BBGR_PAIR_WAVES0;
};
template <> struct Tune<128> {
  static constexpr int row_u = BBGR_ROW_U128, row_waves = BBGR_ROW_WAVES128;
  static constexpr int row_waves0 = row_waves;
  static constexpr int masked_waves = row_waves;
  static constexpr int pair_u = BBGR_PAIR_U128, pair_u_masked = BBGR_PAIR_U128;
  static constexpr int pair_waves = BBGR_PAIR_WAVES128, pair_waves_masked = BBGR_PAIR_WAVES128;
  static constexpr int pair_waves_masked0 = pair_waves_masked, pair_waves0 = pair_waves;
};
template <> struct Tune<256> {
  static constexpr int row_u = BBGR_ROW_U256, row_waves = BBGR_ROW_WAVES256;
  static constexpr int row_waves0 = row_waves;
  static constexpr int masked_waves = row_waves;
  static constexpr int pair_u = BBGR_PAIR_U256, pair_u_masked = BBGR_PAIR_U256;
  static constexpr int pair_waves = BBGR_PAIR_WAVES256, pair_waves_masked = BBGR_PAIR_WAVES256;
  static constexpr int pair_waves_masked0 = pair_waves_masked, pair_waves0 = pair_waves;
};
#define BBGR_WAVES(n) __attribute__((amdgpu_waves_per_eu((n) ? (n) : 1, (n) ? (n) : 10)))

// Bits [e, e + 64) of a slot bitmap (3 words of padding past the end).
__device__ __forceinline__ unsigned long long slot_bits64(const unsigned *bits, int e) {
  const int w = e >> 5, sh = e & 31;
  const unsigned long long x =
      (unsigned long long)bits[w] | ((unsigned long long)bits[w + 1] << 32);
  return sh ? (x >> sh) | ((unsigned long long)bits[w + 2] << (64 - sh)) : x;
}

// Stable compaction of a 16-lane group's live edges (my >= 0) onto its first
// lanes: afterwards lane j holds the j-th live edge of the batch in CSR order
// (index and weight), and the live count is returned. A slot-bitmap batch
// (about 1 live edge in 16 at C4) is then gathered in ceil(live / U) load
// rounds instead of ceil(16 / U) mostly idle ones: C4 first backward item
// product 0.111 -> 0.106 ms. The plain src-masked kernels do not use it: there
// 41 % of the edges are live, and the permute's latency in every batch's
// dependent chain (index -> mask -> permute -> gather) cost more than the
// idle slots (masked user product 0.913 -> 0.98-0.99 ms, round 4 A/B, on a
// build that spilled). They walk the ballot's live-lane bit set instead
// (kPairCompact / kRowCompact: a find-first-bit per pick, no permute): C4
// src-masked user product 0.90 -> 0.88 ms, C3 (d = 128) 1.437 -> 1.347 ms
// (profiles/round6/r6ae_compact_walk_ab.txt).
// The skipped edges would each add +0.0 to a sum that started at +0.0 and so
// is never -0.0: s + 0.0 == s, results are unchanged bit for bit.
// ds_permute (forward permute) sends every lane's pair to its rank among the
// live (or, after them, the dead) lanes of its group: a permutation, so each
// lane receives exactly one. Called with the whole wave converged.
template <int WMODE>
__device__ __forceinline__ int compact_live(int &my, float &mw) {
  const unsigned long long b = __ballot(my >= 0);
  const int base = threadIdx.x & 48;
  const int l = threadIdx.x & 15;
  const unsigned lm = (unsigned)((b >> base) & 0xffffull);
  const unsigned below = (1u << l) - 1u;
  const int nlive = __popc(lm);
  const int p = my >= 0 ? __popc(lm & below) : nlive + __popc(~lm & below);
  const int to = (base + p) << 2;
  my = __builtin_amdgcn_ds_permute(to, my);
  if (WMODE != 0) mw = __int_as_float(__builtin_amdgcn_ds_permute(to, __float_as_int(mw)));
  return nlive;
}

#ifndef BBGR_ROW_COMPACT
#define BBGR_ROW_COMPACT 1
#endif
constexpr bool kRowCompact = BBGR_ROW_COMPACT != 0;

// Sum w_e * x[col_e] over edges [eb, ee) into acc (one 16-lane group).
template <int D, int WMODE, bool MASKED, bool BITS = false, int TAG = TAG_NONE>
__device__ __forceinline__ void gather_range(const SpmmParams &P, int eb, int ee,
                                             int lane, float4 (&acc)[D / 64]) {
  constexpr int V = D / 64;
  constexpr int U = Tune<D>::row_u;   // source rows in flight per group per batch
  for (int e0 = eb; e0 < ee; e0 += 16) {
    int n = min(16, ee - e0);
    unsigned live = 0xffffu;   // slot-bitmap mode: this batch's live edges
    if constexpr (MASKED && BITS) {
      // liveness from the bitmap, 64 edges per test: a dead window costs one
      // (cached) 12-byte load instead of 64 index + mask loads; the live
      // edges are exactly src_mask's, in the same order (bitwise identical)
      unsigned long long win = slot_bits64(P.src_bits, e0);
      const int span = ee - e0;
      if (span < 64) win &= (1ull << span) - 1ull;
      if (win == 0ull) {
        e0 += 48;   // + 16 by the loop: the next 64-edge window
        continue;
      }
      live = (unsigned)(win & 0xffffull);
      if (live == 0u) continue;
    }
    int my = -1;
    float mw = 0.f;
    if (lane < n && ((live >> lane) & 1u)) {
      my = ld_edge(P.indices + e0 + lane);
      // exact-zero source row (a tagged index carries it in its sign)
      if (MASKED && !BITS && TAG != TAG_READ && P.src_mask && !src_live(P, my)) my = -1;
      if (my >= 0) {
        if (WMODE == 1) mw = ld_edge(P.edge_val + e0 + lane);
        if (WMODE == 2) mw = P.col_scale[my] * P.col_scale_s;
      }
    }
    int tm = 0;
    if constexpr (TAG == TAG_WRITE) tm = tag_of(P, my);
    // src-masked batches walk their live lanes' bit set as gather_pair does
    // (kRowCompact): ceil(live / U) load rounds, no permute in the chain
    unsigned rem = 0u;
    if constexpr (MASKED && !BITS && kRowCompact) rem = n >= 16 ? 0xffffu : (1u << n) - 1u;
    if constexpr (MASKED && BITS) {   // live edges first (sparse: ~1 of 16 live)
      n = compact_live<WMODE>(my, mw);
    } else if (MASKED && (TAG == TAG_READ || P.src_mask)) {   // skip 16-edge batches with no live source (group-uniform)
      const unsigned long long lv = __ballot(my >= 0);
      const unsigned lm = (unsigned)((lv >> (threadIdx.x & 48)) & 0xffffull);
      if (lm == 0) continue;
      if constexpr (kRowCompact) {
        rem = lm;
        n = __popc(lm);
      }
    }
    for (int j0 = 0; j0 < n; j0 += U) {
      float4 v[U][V];
      int sl[U];   // the lanes of this round's edges
#pragma unroll
      for (int j = 0; j < U; ++j) {
        sl[j] = j0 + j;
        if constexpr (MASKED && !BITS && kRowCompact) {
          sl[j] = __builtin_ctz(rem | 0x10000u);   // (16: past the set, never read)
          rem &= rem - 1u;
        }
        const int c = __shfl(my, sl[j], 16);
        if (j0 + j < n && (!MASKED || c >= 0)) {
          const float4 *src =
              reinterpret_cast<const float4 *>(P.x + (long)c * P.ldx) + lane;
          if (c >= P.nt_from) {
#pragma unroll
            for (int k = 0; k < V; ++k) v[j][k] = ld_nt(src + 16 * k);
          } else {
#pragma unroll
            for (int k = 0; k < V; ++k) v[j][k] = src[16 * k];
          }
        } else {
#pragma unroll
          for (int k = 0; k < V; ++k) v[j][k] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int j = 0; j < U; ++j) {
        if (WMODE == 0) {
#pragma unroll
          for (int k = 0; k < V; ++k) acc[k] = f4_add(acc[k], v[j][k]);
        } else {
          const float w = __shfl(mw, sl[j], 16);
#pragma unroll
          for (int k = 0; k < V; ++k) acc[k] = f4_fma(w, v[j][k], acc[k]);
        }
      }
    }
    if constexpr (TAG == TAG_WRITE) {
      if (lane < n) tag_store(P, (long)e0 + lane, my, tm);
    }
  }
}

// Narrow rows (D = 8, 16, 32; column-sharded tables): the 16-lane group
// still owns one output row and loads 16 column indices at a time, but L =
// D/4 lanes cover one gathered row, so S = 16/L edges are gathered per load
// round and each lane keeps R = L loads in flight per 16-edge batch. Lane
// (slot, sub) accumulates edges slot, slot+S, ... of every batch; the S slot
// sums are added by a fixed xor tree at the end (deterministic; every lane
// then holds its sub-column block of the row sum).
template <int D, int WMODE, bool MASKED>
__device__ __forceinline__ void gather_range_narrow(const SpmmParams &P, int eb, int ee,
                                                    int lane, float4 &acc) {
  constexpr int L = D / 4;
  constexpr int S = 16 / L;
  constexpr int R = L;
  const int slot = lane / L, sub = lane - slot * L;
  for (int e0 = eb; e0 < ee; e0 += 16) {
    const int n = min(16, ee - e0);
    int my = -1;
    float mw = 0.f;
    if (lane < n) {
      my = P.indices[e0 + lane];
      if (MASKED && P.src_mask && !src_live(P, my)) my = -1;
      if (my >= 0) {
        if (WMODE == 1) mw = P.edge_val[e0 + lane];
        if (WMODE == 2) mw = P.col_scale[my] * P.col_scale_s;
      }
    }
    if (MASKED && P.src_mask) {
      const unsigned long long live = __ballot(my >= 0);
      if (((live >> (threadIdx.x & 48)) & 0xffffull) == 0) continue;
    }
    float4 v[R];
    float w[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int e = r * S + slot;
      const int c = __shfl(my, e, 16);
      w[r] = WMODE == 0 ? 1.f : __shfl(mw, e, 16);
      if (e < n && (!MASKED || c >= 0)) {
        const float4 *src = reinterpret_cast<const float4 *>(P.x + (long)c * P.ldx) + sub;
        v[r] = c >= P.nt_from ? ld_nt(src) : *src;
      } else {
        v[r] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) acc = WMODE == 0 ? f4_add(acc, v[r]) : f4_fma(w[r], v[r], acc);
  }
#pragma unroll
  for (int off = L; off < 16; off <<= 1) {
    acc.x += __shfl_xor(acc.x, off, 16);
    acc.y += __shfl_xor(acc.y, off, 16);
    acc.z += __shfl_xor(acc.z, off, 16);
    acc.w += __shfl_xor(acc.w, off, 16);
  }
}

// Narrow short rows (D = 8, 16, 32): S = 16/L rows per 16-lane group, one
// per L-lane slot, walked independently (a slot leaves its loop when its row
// ends), so a wave keeps 64/L rows in flight: one row per group left these
// launches bound by the per-row latency chain (indptr -> indices -> gathers
// -> store) at 5M rows. Each lane adds its row's edges in CSR order, as the
// full-width one-row kernel does per column block: a column slice of the
// result is bitwise the full-width kernel's columns.
template <int D> struct SlotRounds {   // index rounds (L edges each) per load round
  static constexpr int value = D == 32 ? BBGR_SLOT_ROUNDS32 : D == 16 ? BBGR_SLOT_ROUNDS16 : 2;
};

template <int D, int WMODE, bool MASKED>
__device__ __forceinline__ void gather_slot(const SpmmParams &P, int eb, int ee, int slot,
                                            int sub, float4 &acc) {
  constexpr int L = D / 4;
  constexpr int RR = SlotRounds<D>::value;
  for (int e0 = eb; e0 < ee; e0 += RR * L) {
    int my[RR];
    float mw[RR];
#pragma unroll
    for (int r = 0; r < RR; ++r) {
      const int e = e0 + r * L + sub;
      my[r] = -1;
      mw[r] = 0.f;
      if (e < ee) {
        my[r] = P.indices[e];
        if (MASKED && P.src_mask && !src_live(P, my[r])) my[r] = -1;
        if (my[r] >= 0) {
          if (WMODE == 1) mw[r] = P.edge_val[e];
          if (WMODE == 2) mw[r] = P.col_scale[my[r]] * P.col_scale_s;
        }
      }
    }
    float4 v[RR * L];
    float w[RR * L];
#pragma unroll
    for (int j = 0; j < RR * L; ++j) {
      const int src_lane = slot * L + (j % L);
      const int c = __shfl(my[j / L], src_lane, 16);
      w[j] = WMODE == 0 ? 1.f : __shfl(mw[j / L], src_lane, 16);
      if (e0 + j < ee && (!MASKED || c >= 0)) {
        const float4 *src = reinterpret_cast<const float4 *>(P.x + (long)c * P.ldx) + sub;
        v[j] = c >= P.nt_from ? ld_nt(src) : *src;
      } else {
        v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int j = 0; j < RR * L; ++j)
      acc = WMODE == 0 ? f4_add(acc, v[j]) : f4_fma(w[j], v[j], acc);
  }
}

// A row's gather for any width: the narrow form below 64 columns.
template <int D, int WMODE, bool MASKED, bool BITS = false, int TAG = TAG_NONE>
__device__ __forceinline__ void gather_row(const SpmmParams &P, int eb, int ee, int lane,
                                           float4 (&acc)[RowShape<D>::V]) {
  if constexpr (D < 64) {
    gather_range_narrow<D, WMODE, MASKED>(P, eb, ee, lane, acc[0]);
  } else {
    gather_range<D, WMODE, MASKED, BITS, TAG>(P, eb, ee, lane, acc);
  }
}

// Two short rows per 16-lane group, their batches interleaved: 2*U8 source
// rows in flight per group across two independent rows (U8 per row), so a
// low-degree table (users, avg degree ~10) keeps twice the rows in flight
// for the same registers. Per row the operation sequence is gather_range's
// (edges in CSR order from zero; dead batches skipped), so results match the
// one-row path bitwise (up to the sign of an exact zero).
#ifndef BBGR_PAIR_COMPACT
#define BBGR_PAIR_COMPACT 1
#endif
constexpr bool kPairCompact = BBGR_PAIR_COMPACT != 0;

template <int D, int WMODE, bool MASKED, int TAG = TAG_NONE>
__device__ __forceinline__ void gather_pair(const SpmmParams &P, int ebA, int eeA, int ebB,
                                            int eeB, int lane, float4 (&accA)[D / 64],
                                            float4 (&accB)[D / 64]) {
  constexpr int V = D / 64;
  constexpr int U = MASKED ? Tune<D>::pair_u_masked : Tune<D>::pair_u;   // per row
  const int nA = eeA - ebA, nB = eeB - ebB;
  const int nmax = max(nA, nB);
  for (int o = 0; o < nmax; o += 16) {
    int na = min(16, nA - o), nb = min(16, nB - o);
    int myA = -1, myB = -1;
    float mwA = 0.f, mwB = 0.f;
    // both rows' column indices, then both rows' liveness words, each pair
    // issued before either is waited on: two dependent round trips per batch
    // (the per-row form compiled to index A -> mask A -> index B -> mask B)
    if (lane < na) myA = ld_edge(P.indices + ebA + o + lane);
    if (lane < nb) myB = ld_edge(P.indices + ebB + o + lane);
    if (MASKED && TAG != TAG_READ && P.src_mask) src_live2(P, myA, myB);
    if (WMODE == 1) {
      if (myA >= 0) mwA = ld_edge(P.edge_val + ebA + o + lane);
      if (myB >= 0) mwB = ld_edge(P.edge_val + ebB + o + lane);
    }
    if (WMODE == 2) {
      if (myA >= 0) mwA = P.col_scale[myA] * P.col_scale_s;
      if (myB >= 0) mwB = P.col_scale[myB] * P.col_scale_s;
    }
    int tmA = 0, tmB = 0;
    if constexpr (TAG == TAG_WRITE) {
      tmA = tag_of(P, myA);
      tmB = tag_of(P, myB);
    }
    // compacted masked batches: the live edges' lanes as a bit set per row,
    // walked lowest bit first (CSR order), so a batch takes ceil(live / U)
    // load rounds instead of ceil(n / U) mostly idle ones; unmasked batches
    // walk their first n lanes. No permute in the chain (the set is the
    // ballot's; the pick is one find-first-bit), and the skipped edges would
    // add +0.0 to a sum that is never -0.0: bitwise the uncompacted walk.
    unsigned remA = 0u, remB = 0u;
    if constexpr (MASKED && kPairCompact) {
      remA = na >= 16 ? 0xffffu : na > 0 ? (1u << na) - 1u : 0u;
      remB = nb >= 16 ? 0xffffu : nb > 0 ? (1u << nb) - 1u : 0u;
    }
    if (MASKED && (TAG == TAG_READ || P.src_mask)) {   // a batch with no live source adds nothing
      const unsigned long long la = __ballot(myA >= 0), lb = __ballot(myB >= 0);
      if constexpr (kPairCompact) {
        remA = (unsigned)((la >> (threadIdx.x & 48)) & 0xffffull);
        remB = (unsigned)((lb >> (threadIdx.x & 48)) & 0xffffull);
        na = __popc(remA);
        nb = __popc(remB);
      } else {
        if (((la >> (threadIdx.x & 48)) & 0xffffull) == 0) na = 0;
        if (((lb >> (threadIdx.x & 48)) & 0xffffull) == 0) nb = 0;
      }
    }
    const int nn = max(na, nb);
    for (int j0 = 0; j0 < nn; j0 += U) {
      float4 vA[U][V], vB[U][V];
      int sA[U], sB[U];   // the lanes of this round's edges
#pragma unroll
      for (int j = 0; j < U; ++j) {
        sA[j] = sB[j] = j0 + j;
        if constexpr (MASKED && kPairCompact) {
          sA[j] = __builtin_ctz(remA | 0x10000u);   // (16: past the set, never read)
          sB[j] = __builtin_ctz(remB | 0x10000u);
          remA &= remA - 1u;
          remB &= remB - 1u;
        }
        const int cA = __shfl(myA, sA[j], 16);
        const int cB = __shfl(myB, sB[j], 16);
        if (j0 + j < na && (!MASKED || cA >= 0)) {
          const float4 *src = reinterpret_cast<const float4 *>(P.x + (long)cA * P.ldx) + lane;
          if (cA >= P.nt_from) {
#pragma unroll
            for (int k = 0; k < V; ++k) vA[j][k] = ld_nt(src + 16 * k);
          } else {
#pragma unroll
            for (int k = 0; k < V; ++k) vA[j][k] = src[16 * k];
          }
        } else {
#pragma unroll
          for (int k = 0; k < V; ++k) vA[j][k] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if (j0 + j < nb && (!MASKED || cB >= 0)) {
          const float4 *src = reinterpret_cast<const float4 *>(P.x + (long)cB * P.ldx) + lane;
          if (cB >= P.nt_from) {
#pragma unroll
            for (int k = 0; k < V; ++k) vB[j][k] = ld_nt(src + 16 * k);
          } else {
#pragma unroll
            for (int k = 0; k < V; ++k) vB[j][k] = src[16 * k];
          }
        } else {
#pragma unroll
          for (int k = 0; k < V; ++k) vB[j][k] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int j = 0; j < U; ++j) {
        if (WMODE == 0) {
#pragma unroll
          for (int k = 0; k < V; ++k) {
            accA[k] = f4_add(accA[k], vA[j][k]);
            accB[k] = f4_add(accB[k], vB[j][k]);
          }
        } else {
          const float wA = __shfl(mwA, sA[j], 16);
          const float wB = __shfl(mwB, sB[j], 16);
#pragma unroll
          for (int k = 0; k < V; ++k) {
            accA[k] = f4_fma(wA, vA[j][k], accA[k]);
            accB[k] = f4_fma(wB, vB[j][k], accB[k]);
          }
        }
      }
    }
    if constexpr (TAG == TAG_WRITE) {
      if (lane < na) tag_store(P, (long)ebA + o + lane, myA, tmA);
      if (lane < nb) tag_store(P, (long)ebB + o + lane, myB, tmB);
    }
  }
}

// torch.optim.Adam on one row held by a 16-lane group: the same expression
// order as adam_kernel (train.hip), so fused and separate steps agree bitwise.
// The Adam constants of this launch: the host's, or (captured steps) the step
// t in device memory with the bias corrections of the host-built table.
__device__ __forceinline__ AdamConsts launch_adam_consts(const SpmmParams &P) {
  AdamConsts c = P.adam;
  if (P.adam_state) {
    const long t = clamp_step(P.adam_state);
    c.step = P.adam_lr / P.adam_bc[2 * (t - 1)];
    c.bc2s = P.adam_bc[2 * (t - 1) + 1];
  }
  return c;
}

// `row`: the param row; `mrow`: the moments' row; `crow`: the row of the
// caller-order mirror the updated param row is also stored to (adam_mirror)
template <int D>
__device__ __forceinline__ void adam_row(const SpmmParams &P, long row, long mrow, long crow,
                                         int lane, const float4 (&G)[RowShape<D>::V]) {
  constexpr int V = RowShape<D>::V;
  const AdamConsts ac = launch_adam_consts(P);
  float4 *pp = reinterpret_cast<float4 *>(P.adam_p + (long)row * P.adam_ld) + lane;
  float4 *pm = reinterpret_cast<float4 *>(P.adam_m + (long)mrow * P.adam_ld) + lane;
  float4 *pv = reinterpret_cast<float4 *>(P.adam_v + (long)mrow * P.adam_ld) + lane;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const bool ntm = P.nt_out_from != 0x7fffffff;   // moments: streamed once per step
    float4 p4 = pp[16 * k];
    float4 m4 = ntm ? ld_nt(pm + 16 * k) : pm[16 * k];
    float4 v4 = ntm ? ld_nt(pv + 16 * k) : pv[16 * k];
    adam_elem(p4.x, G[k].x, m4.x, v4.x, ac);
    adam_elem(p4.y, G[k].y, m4.y, v4.y, ac);
    adam_elem(p4.z, G[k].z, m4.z, v4.z, ac);
    adam_elem(p4.w, G[k].w, m4.w, v4.w, ac);
    if (row >= P.nt_out_from) st_nt(pp + 16 * k, p4);
    else pp[16 * k] = p4;
    if (P.adam_mirror)   // write-only random rows: streamed
      st_nt(reinterpret_cast<float4 *>(P.adam_mirror + crow * P.adam_ld) + lane + 16 * k, p4);
    if (ntm) {
      st_nt(pm + 16 * k, m4);
      st_nt(pv + 16 * k, v4);
    } else {
      pm[16 * k] = m4;
      pv[16 * k] = v4;
    }
  }
}

template <int D>
__device__ __forceinline__ void epilogue(const SpmmParams &P, int row, int lane,
                                         const float4 (&T)[RowShape<D>::V]) {
  constexpr int V = RowShape<D>::V;
  if (lane >= RowShape<D>::LANES) return;   // narrow rows: idle lanes
  if (P.y || P.adam_p) {
    const float ys = (P.y_scale ? P.y_scale[row] : 1.f) * P.y_scale_s;
    float4 G[V];
    const long ra = P.add_map ? (long)P.add_map[row] : (long)row;
    if (P.add && (!P.add_mask || P.add_mask[ra])) {
      const float as = (P.add_scale ? P.add_scale[row] : 1.f) * P.add_scale_s;
      const float4 *ad = reinterpret_cast<const float4 *>(P.add + ra * P.ldadd) + lane;
#pragma unroll
      for (int k = 0; k < V; ++k) G[k] = f4_fma(as, ad[16 * k], f4_mul(ys, T[k]));
    } else {
#pragma unroll
      for (int k = 0; k < V; ++k) G[k] = f4_mul(ys, T[k]);
    }
    const long ry = P.y_map ? (long)P.y_map[row] : (long)row;
    if (P.y) {
      float4 *dst = reinterpret_cast<float4 *>(P.y + ry * P.ldy) + lane;
      if (row >= P.nt_out_from) {
#pragma unroll
        for (int k = 0; k < V; ++k) st_nt(dst + 16 * k, G[k]);
      } else {
#pragma unroll
        for (int k = 0; k < V; ++k) dst[16 * k] = G[k];
      }
    }
    const long ra_ = P.adam_map ? (long)P.adam_map[row] : ry;   // the Adam's rows
    const long rm_ = P.adam_mrow ? (long)row : ra_;                // its moments' rows
    const long rp_ = P.adam_mirror ? rm_ : ra_;                    // its param's rows
    if (P.adam_p && P.adam_g) {   // Adam of another table riding on this row write
      const float4 *gr = reinterpret_cast<const float4 *>(P.adam_g + ra_ * P.adam_g_ld) + lane;
      float4 Ga[V];
#pragma unroll
      for (int k = 0; k < V; ++k) {   // gs * g, as adam_kernel forms it
        const float4 g4 = ld_nt(gr + 16 * k);
        Ga[k] = make_float4(P.adam_g_scale * g4.x, P.adam_g_scale * g4.y,
                            P.adam_g_scale * g4.z, P.adam_g_scale * g4.w);
      }
      adam_row<D>(P, rp_, rm_, ra_, lane, Ga);
    } else if (P.adam_p) {
      adam_row<D>(P, rp_, rm_, ra_, lane, G);
    }
  }
  const long rc = P.acc_map ? (long)P.acc_map[row] : (long)row;
  if (P.acc_out && (!P.acc_mask || P.acc_mask[rc])) {
    const float cs = (P.acc_scale ? P.acc_scale[row] : 1.f) * P.acc_scale_s;
    // the layer-mean accumulator is streamed (read once, written once per
    // layer, never gathered): non-temporal, so a dense pass (1.28 GB in and
    // out for the C4 user table) does not evict the gathered rows from the
    // Infinity Cache
    float4 *dst = reinterpret_cast<float4 *>(P.acc_out + rc * P.ldacc_out) + lane;
    if (P.acc_in) {
      const long ri = P.acc_in_map ? (long)P.acc_in_map[row] : rc;
      const float4 *ai =
          reinterpret_cast<const float4 *>(P.acc_in + ri * P.ldacc_in) + lane;
#pragma unroll
      for (int k = 0; k < V; ++k)
        st_nt(dst + 16 * k, f4_mul(P.gamma, f4_fma(cs, T[k], ld_nt(ai + 16 * k))));
    } else {
#pragma unroll
      for (int k = 0; k < V; ++k) st_nt(dst + 16 * k, f4_mul(P.gamma, f4_mul(cs, T[k])));
    }
  }
}

// Fixed-order reduction of the 16 group partials held in LDS; result lands in
// red[0][*]. Called by all 256 threads. It MUST stay a strict left-to-right
// sum from group 0 (no tree): chunk_row_serial reproduces a single-chunk row
// bit for bit by adding the live groups' sums in this order and dropping the
// dead groups' +0.0 terms, which is exact only for a sequential sum.
template <int D>
__device__ __forceinline__ void block_reduce16(float4 *red, int g, int lane,
                                               const float4 (&acc)[RowShape<D>::V]) {
  constexpr int V = RowShape<D>::V;
  constexpr int W = D / 4;  // float4 per row
  if (lane < RowShape<D>::LANES) {
#pragma unroll
    for (int k = 0; k < V; ++k) red[g * W + lane + 16 * k] = acc[k];
  }
  __syncthreads();
  if (threadIdx.x < W) {
    float4 s = red[threadIdx.x];
#pragma unroll
    for (int gg = 1; gg < 16; ++gg) s = f4_add(s, red[gg * W + threadIdx.x]);
    red[threadIdx.x] = s;
  }
  __syncthreads();
}

// Fixed-order sum of a split row's chunk partials (slots base .. base+c-1):
// group g adds slots g, g+16, ... in order, then the 16 group sums are added
// in group order (block_reduce16); g == 0 runs the epilogue.
template <int D>
__device__ __forceinline__ void split_row_finish(const SpmmParams &P, int row, int base, int c,
                                                 float4 *red, int g, int lane) {
  constexpr int V = RowShape<D>::V;
  float4 acc[V];
#pragma unroll
  for (int k = 0; k < V; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int c_lane = lane < RowShape<D>::LANES ? c : 0;   // idle lanes read nothing
#pragma unroll 4
  for (int sl = g; sl < c_lane; sl += 16) {
    const float4 *src =
        reinterpret_cast<const float4 *>(P.partial) + (long)(base + sl) * (D / 4) + lane;
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = f4_add(acc[k], src[16 * k]);
  }
  block_reduce16<D>(red, g, lane, acc);
  if (g == 0) {
    float4 T[V];
#pragma unroll
    for (int k = 0; k < V; ++k) T[k] = red[lane + 16 * k];
    epilogue<D>(P, row, lane, T);
  }
}

// A chunk of a row cut into c > 1 chunks: publish this chunk's partial; the
// last chunk of the row to arrive sums them all (split_row_finish) in this
// launch. Hand-off per cdna_hip_programming.md Guideline 16 (R1 payload,
// counter form): the partial is stored write-through (8-B relaxed agent
// atomic stores = sc1, so no release fence: an agent release here would
// write back the whole XCD L2 once per chunk workgroup) -> every wave drains
// -> barrier -> one relaxed agent ticket fetch_add; the drawer of ticket c-1
// takes one agent-scope acquire before its workgroup reads the slots with
// plain loads. The ticket lives at arrivals[base] (base = the row's first
// chunk) and the reducer re-zeroes it.
template <int D>
__device__ __forceinline__ void split_row_arrive(const SpmmParams &P, int4 ch, float4 *red,
                                                 int g, int lane) {
  constexpr int V = RowShape<D>::V;
  if (g == 0 && lane < RowShape<D>::LANES) {
    unsigned long long *dst = reinterpret_cast<unsigned long long *>(
        reinterpret_cast<float4 *>(P.partial) + (long)ch.w * (D / 4) + lane);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float4 v = red[lane + 16 * k];
      const unsigned long long lo =
          (unsigned long long)__float_as_uint(v.x) | ((unsigned long long)__float_as_uint(v.y) << 32);
      const unsigned long long hi =
          (unsigned long long)__float_as_uint(v.z) | ((unsigned long long)__float_as_uint(v.w) << 32);
      __hip_atomic_store(dst + 32 * k, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(dst + 32 * k + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // chunk j of c (plan_fill_kernel: chunk j starts at eb + floor(len*j/c)),
  // slot = base + j
  const int eb = P.indptr[ch.x];
  const long len = (long)P.indptr[ch.x + 1] - eb;
  const int c = plan_chunks(len, P.long_threshold, P.chunk_edges);
  const int j = (int)(((long)(ch.y - eb) * c + len - 1) / len);
  const int base = ch.w - j;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();   // every wave has read red[] and drained its stores
  int *flag = reinterpret_cast<int *>(red);
  if (threadIdx.x == 0) {
    const int ticket =
        __hip_atomic_fetch_add(P.arrivals + base, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = ticket == c - 1;
    if (last) {
      __hip_atomic_store(P.arrivals + base, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    flag[0] = last;
  }
  __syncthreads();
  const int last = flag[0];
  __syncthreads();   // flag read before split_row_finish reuses red[]
  if (last) split_row_finish<D>(P, ch.x, base, c, red, g, lane);
}

// A single-chunk long row (deg in (long_threshold, chunk_edges]) of a slot-
// bitmap launch, summed by ONE 16-lane group in the order of the chunk
// workgroup that owns such a row elsewhere: lane group g's range
// [eb + g*per, eb + (g+1)*per) from zero (gather_range), then the 16 range
// sums added in group order (block_reduce16). Bitwise the workgroup's value;
// with a few live edges per row the bitmap windows are nearly all dead, and a
// workgroup per row (11k of them at C4) cost more than the scan.
template <int D, int WMODE>
__device__ __forceinline__ void chunk_row_serial(const SpmmParams &P, int eb, int ee, int lane,
                                                 float4 (&s)[RowShape<D>::V]) {
  constexpr int V = RowShape<D>::V;
  const int len = ee - eb;
  const int per = (((len + 15) >> 4) + 15) & ~15;   // the chunk workgroup's split
  // lane g tests range g's bitmap windows (<= 2 of 64 edges), all lanes at
  // once; only live ranges are gathered. A dead range's sum is +0.0 and
  // s + 0.0 == s (s is never -0.0: a sum from +0.0), so skipping it keeps the
  // workgroup's value bit for bit.
  //
  // Lane g also counts range g's live edges and keeps the first one's slot.
  // When no range holds more than one (the common case: ~1 live edge in 600
  // at C4), every live range's sum is its one term (0 + x, or fma(w, x, 0)),
  // so the group loads all their column indices in one round and gathers the
  // rows two at a time, adding the terms in range order: the same operations
  // as the per-range gathers below, without one dependent chain per range.
  int cnt = 0, fe = -1;
  {
    const int gb = eb + lane * per, ge = min(ee, gb + per);
#pragma unroll 1
    for (int e = gb; e < ge; e += 64) {
      unsigned long long w = slot_bits64(P.src_bits, e);
      if (ge - e < 64) w &= (1ull << (ge - e)) - 1ull;
      if (w != 0ull && fe < 0) fe = e + __builtin_ctzll(w);
      cnt += __popcll(w);
    }
  }
  const int base = threadIdx.x & 48;
  unsigned segs = (unsigned)((__ballot(cnt != 0) >> base) & 0xffffull);
  const bool multi = ((__ballot(cnt > 1) >> base) & 0xffffull) != 0ull;
#pragma unroll
  for (int k = 0; k < V; ++k) s[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  bool first = true;
  if (!multi) {
    int my = -1;
    float mw = 0.f;
    if (fe >= 0) {
      my = ld_edge(P.indices + fe);
      if (WMODE == 1) mw = ld_edge(P.edge_val + fe);
      if (WMODE == 2) mw = P.col_scale[my] * P.col_scale_s;
    }
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 1
    while (segs) {
      int gg[2];
      float4 v[2][V];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        gg[j] = segs ? __ffs(segs) - 1 : -1;
        segs &= segs ? segs - 1u : 0u;
        const int c = __shfl(my, gg[j] < 0 ? 0 : gg[j], 16);
        if (gg[j] >= 0) {
          const float4 *src = reinterpret_cast<const float4 *>(P.x + (long)c * P.ldx) + lane;
          if (c >= P.nt_from) {
#pragma unroll
            for (int k = 0; k < V; ++k) v[j][k] = ld_nt(src + 16 * k);
          } else {
#pragma unroll
            for (int k = 0; k < V; ++k) v[j][k] = src[16 * k];
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (gg[j] < 0) continue;
        const float w = __shfl(mw, gg[j], 16);
#pragma unroll
        for (int k = 0; k < V; ++k) {
          const float4 p = WMODE == 0 ? f4_add(z, v[j][k]) : f4_fma(w, v[j][k], z);
          s[k] = first ? p : f4_add(s[k], p);
        }
        first = false;
      }
    }
    return;
  }
#pragma unroll 1
  while (segs) {
    const int g = __ffs(segs) - 1;
    segs &= segs - 1u;
    float4 p[V];
#pragma unroll
    for (int k = 0; k < V; ++k) p[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int gb = eb + g * per;
    gather_row<D, WMODE, true, true>(P, gb, min(ee, gb + per), lane, p);
#pragma unroll
    for (int k = 0; k < V; ++k) s[k] = first ? p[k] : f4_add(s[k], p[k]);
    first = false;
  }
}

// Long rows a slot-bitmap launch sums in its short-row groups (chunk_row_serial)
// instead of chunk workgroups: the rows the plan gives a single chunk (the
// planner's own rule, plan_chunks), i.e. exactly the rows whose chunk
// workgroup sums them as one range split 16 ways (tested at deg = thr, thr+1,
// chunk_edges, chunk_edges+1: test_slot_bitmap_single_chunk_boundary_rows_bitwise).
template <int D, bool BITS>
__device__ __forceinline__ bool serial_long(const SpmmParams &P, int len) {
  if constexpr (BITS && D >= 64) return plan_chunks(len, P.long_threshold, P.chunk_edges) == 1;
  return false;
}

// Short-row workgroup sb of a launch: rows sb*per_block.. of the row range or
// of the row list (whose length is n_list).
template <int D, int WMODE, bool MASKED, bool PAIR, bool BITS, int TAG>
__device__ __forceinline__ void short_rows(const SpmmParams &P, long sb, long n_list, int g,
                                           int lane) {
  constexpr int V = RowShape<D>::V;
  float4 acc[V];
#pragma unroll
  for (int k = 0; k < V; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);

  if constexpr (PAIR && D >= 64) {   // ---- two rows per 16-lane group (rows j, j + 16)
    long rr[2];
    int eb[2], ee[2];
    bool ser[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      long row = (long)P.row_begin + sb * 32 + 16 * h + g;
      if (MASKED && P.row_list) {
        row = row < n_list ? P.row_list[row] : -1;
      } else if (row >= P.row_end) {
        row = -1;
      }
      if (row >= P.n_rows) row = -1;
      eb[h] = ee[h] = 0;
      ser[h] = false;
      if (row >= 0) {
        eb[h] = P.indptr[row];
        ee[h] = P.indptr[row + 1];
        if (MASKED && !P.row_list && P.row_mask && !P.row_mask[row]) {
          row = -1;
        } else if (ee[h] - eb[h] > P.long_threshold) {
          ser[h] = serial_long<D, BITS>(P, ee[h] - eb[h]);
          if (!ser[h]) row = -1;
        }
      }
      if (row < 0) eb[h] = ee[h] = 0;
      rr[h] = row;
    }
    float4 accB[V];
#pragma unroll
    for (int k = 0; k < V; ++k) accB[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    gather_pair<D, WMODE, MASKED, TAG>(P, ser[0] ? 0 : eb[0], ser[0] ? 0 : ee[0],
                                  ser[1] ? 0 : eb[1], ser[1] ? 0 : ee[1], lane, acc, accB);
    if (rr[0] >= 0 && !ser[0]) epilogue<D>(P, (int)rr[0], lane, acc);
    if (rr[1] >= 0 && !ser[1]) epilogue<D>(P, (int)rr[1], lane, accB);
    if (ser[0] || ser[1]) {
#pragma unroll 1
      for (int h = 0; h < 2; ++h) {
        if (!ser[h]) continue;
        chunk_row_serial<D, WMODE>(P, eb[h], ee[h], lane, acc);
        epilogue<D>(P, (int)rr[h], lane, acc);
      }
    }
    return;
  }
  if constexpr (D < 64) {   // ---- narrow short rows: 16/L per group, one per slot
    constexpr int L = D / 4, S = 16 / L;
    const int slot = lane / L, sub = lane - slot * L;
    long row = (long)P.row_begin + sb * (16 * S) + g * S + slot;
    if (MASKED && P.row_list) {
      row = row < n_list ? P.row_list[row] : -1;
    } else if (row >= P.row_end) {
      row = -1;
    }
    if (row >= P.n_rows) row = -1;
    int eb = 0, ee = 0;
    if (row >= 0) {
      eb = P.indptr[row];
      ee = P.indptr[row + 1];
      if (ee - eb > P.long_threshold || (MASKED && !P.row_list && P.row_mask && !P.row_mask[row]))
        row = -1;
    }
    if (row < 0) eb = ee = 0;
    float4 T[1] = {make_float4(0.f, 0.f, 0.f, 0.f)};
    gather_slot<D, WMODE, MASKED>(P, eb, ee, slot, sub, T[0]);
    if (row >= 0) epilogue<D>(P, (int)row, sub, T);
    return;
  }
  // ---- short rows: one 16-lane group per row ------------------------------
  long row = (long)P.row_begin + sb * 16 + g;
  if (MASKED && P.row_list) {
    if (row >= n_list) return;
    row = P.row_list[row];
    if (row < 0) return;
  } else if (row >= P.row_end) {
    return;
  }
  if (row >= P.n_rows) return;
  const int eb = P.indptr[row];
  const int ee = P.indptr[row + 1];
  if (MASKED && !P.row_list && P.row_mask && !P.row_mask[row]) return;
  if (ee - eb > P.long_threshold) {
    if (!serial_long<D, BITS>(P, ee - eb)) return;  // owned by chunk blocks
    chunk_row_serial<D, WMODE>(P, eb, ee, lane, acc);
  } else {
    gather_row<D, WMODE, MASKED, BITS, TAG>(P, eb, ee, lane, acc);
  }
  epilogue<D>(P, (int)row, lane, acc);
}

template <int D, int WMODE, bool MASKED, bool PAIR, bool BITS = false, int TAG = TAG_NONE>
__device__ __forceinline__ void spmm_body(const SpmmParams &P) {
  constexpr int V = RowShape<D>::V;
  __shared__ float4 red[16 * (D / 4)];
  const int g = threadIdx.x >> 4;
  const int lane = threadIdx.x & 15;

  if ((int)blockIdx.x < P.n_chunks) {
    // ---- one chunk of a long row: whole workgroup --------------------------
    const int4 ch = P.chunks[P.chunk_begin + blockIdx.x];  // row, e_begin, e_end, slot
    if (MASKED && P.row_mask && !P.row_mask[ch.x]) return;   // whole workgroup, uniform
    if (MASKED && P.row_list && !P.row_mask) return;         // list mode: short rows only
    if (ch.w < 0 && serial_long<D, BITS>(P, ch.z - ch.y)) return;   // short_rows sums it
    float4 acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int len = ch.z - ch.y;
    const int per = (((len + 15) >> 4) + 15) & ~15;  // multiple of 16
    const int gb = ch.y + g * per;
    const int ge = min(ch.z, gb + per);
    if (gb < ge) gather_row<D, WMODE, MASKED, BITS, TAG>(P, gb, ge, lane, acc);
    block_reduce16<D>(red, g, lane, acc);
    if (ch.w < 0) {   // the row's only chunk
      if (g == 0 && lane < RowShape<D>::LANES) {
        float4 T[V];
#pragma unroll
        for (int k = 0; k < V; ++k) T[k] = red[lane + 16 * k];
        epilogue<D>(P, ch.x, lane, T);
      }
      return;
    }
    split_row_arrive<D>(P, ch, red, g, lane);
    return;
  }
  const long sb = (long)blockIdx.x - P.n_chunks;
  long n = P.n_row_list;
  // list length in device memory (a list built on the stream, e.g. inside a
  // captured step; n_row_list is its capacity): workgroups past it exit
  if (MASKED && P.row_list && P.row_count) n = min(n, *P.row_count);
  short_rows<D, WMODE, MASKED, PAIR, BITS, TAG>(P, sb, n, g, lane);
}

// Full-CSR launches (the roofline kernel) and masked / row-list launches are
// distinct symbols so that profiles separate them. The two-rows-per-group
// (low-degree table) forms are their own symbols too, with their own
// occupancy target.
template <int D, int WMODE>
__global__ __launch_bounds__(256) BBGR_WAVES(WMODE == 0 ? Tune<D>::row_waves0
                                                     : Tune<D>::row_waves) void spmm_kernel(
    SpmmParams P) {
  spmm_body<D, WMODE, false, false>(P);
}

template <int D, int WMODE>
__global__ __launch_bounds__(256) BBGR_WAVES(WMODE == 0 ? Tune<D>::pair_waves0
                                                     : Tune<D>::pair_waves) void spmm_pair_kernel(
    SpmmParams P) {
  spmm_body<D, WMODE, false, true>(P);
}

template <int D, int WMODE>
__global__ __launch_bounds__(256) BBGR_WAVES(WMODE == 0 ? (Tune<D>::row_waves0 ? Tune<D>::row_waves0
                                                                       : Tune<D>::masked_waves)
                                                     : Tune<D>::row_waves) void
spmm_masked_kernel(SpmmParams P) {
  spmm_body<D, WMODE, true, false>(P);
}

template <int D, int WMODE>
__global__ __launch_bounds__(256) BBGR_WAVES(WMODE == 0 ? Tune<D>::pair_waves_masked0
                                                     : Tune<D>::pair_waves_masked) void
spmm_masked_pair_kernel(SpmmParams P) {
  spmm_body<D, WMODE, true, true>(P);
}

// The tagged-index forms (two-row CSRs, d >= 64): the full product that also
// writes the tagged copy of its column indices, and the src-masked product that
// reads liveness from that copy (args.tag_out / src_tagged). Symbols of their
// own: the plain kernels keep their register budgets.
template <int D, int WMODE>
__global__ __launch_bounds__(256) BBGR_WAVES(WMODE == 0 ? Tune<D>::pair_waves0
                                                     : Tune<D>::pair_waves) void spmm_pair_tag_kernel(
    SpmmParams P) {
  spmm_body<D, WMODE, false, true, false, TAG_WRITE>(P);
}

template <int D, int WMODE>
__global__ __launch_bounds__(256) BBGR_WAVES(WMODE == 0 ? Tune<D>::pair_waves_masked0
                                                     : Tune<D>::pair_waves_masked) void
spmm_masked_pair_tagged_kernel(SpmmParams P) {
  spmm_body<D, WMODE, true, true, false, TAG_READ>(P);
}

// Slot-bitmap launches (args.src_bits, d >= 64, one row per group): liveness
// from the bitmap, single-chunk long rows summed by their row's group
// (chunk_row_serial). A symbol of its own so the plain masked kernels keep
// their register budget. Unweighted at d = 64: BBGR_BITS_WAVES0 (the round-3
// 8-wave target spills since round 4's single-live-edge path; compiler's
// choice now).
template <int D, int WMODE>
__global__ __launch_bounds__(256) BBGR_WAVES(WMODE == 0 && D == 64 ? BBGR_BITS_WAVES0 : Tune<D>::masked_waves) void
spmm_bits_kernel(
    SpmmParams P) {
  spmm_body<D, WMODE, true, false, true>(P);
}

// Full-CSR launch whose epilogue applies the fused Adam step (its bytes add the
// parameter / moment streams): a third symbol so rooflines stay per kind.
template <int D, int WMODE>
__global__ __launch_bounds__(256) BBGR_WAVES(WMODE == 0 ? Tune<D>::row_waves0
                                                     : Tune<D>::row_waves) void spmm_adam_kernel(
    SpmmParams P) {
  spmm_body<D, WMODE, false, false>(P);
}

template <int D, int WMODE>
__global__ __launch_bounds__(256) BBGR_WAVES(Tune<D>::pair_waves) void spmm_adam_pair_kernel(
    SpmmParams P) {
  spmm_body<D, WMODE, false, true>(P);
}

template <int D>
__global__ __launch_bounds__(256) void epilogue_kernel(SpmmParams P, const float *t,
                                                       long ldt) {
  constexpr int V = RowShape<D>::V;
  const long j = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int lane = threadIdx.x & 15;
  long row = j;
  if (P.row_list) {   // compact input: row j of t -> output row row_list[j]
    if (j >= P.n_row_list) return;
    row = P.row_list[j];
    if (row < 0) return;
  }
  if (row >= P.n_rows) return;
  if (P.row_mask && !P.row_mask[row]) return;
  if (lane >= RowShape<D>::LANES) return;
  const float4 *src = reinterpret_cast<const float4 *>(t + j * ldt) + lane;
  float4 T[V];
#pragma unroll
  for (int k = 0; k < V; ++k) T[k] = src[16 * k];
  epilogue<D>(P, (int)row, lane, T);
}

template <int D, int WMODE>
static int launch_spmm(const SpmmParams &P, int n_split, hipStream_t st, bool tag_read) {
  const bool masked = P.src_mask || P.row_mask || P.row_list || tag_read;
  const long short_rows = P.row_list ? P.n_row_list : (long)(P.row_end - P.row_begin);
  const bool pair = D >= 64 && P.pair_rows;
  const long per_block = D < 64 ? 16 * (16 / (D / 4)) : (pair ? 32 : 16);
  const long short_blocks = (short_rows + per_block - 1) / per_block;
  const long grid = (long)P.n_chunks + short_blocks;
  if ((P.tag_out || tag_read) && !(D >= 64 && pair)) {
    set_error("bbgr_spmm: tagged indices need a two-row CSR (average degree <= 24) and d >= 64");
    return BBGR_ERR_UNSUPPORTED;
  }
  if (grid > 0) {
    const dim3 gd((unsigned)grid), bd(256);
    if constexpr (D >= 64) {
      if (pair) {
        if (tag_read) hipLaunchKernelGGL((spmm_masked_pair_tagged_kernel<D, WMODE>), gd, bd, 0, st, P);
        else if (P.tag_out) hipLaunchKernelGGL((spmm_pair_tag_kernel<D, WMODE>), gd, bd, 0, st, P);
        else if (masked) hipLaunchKernelGGL((spmm_masked_pair_kernel<D, WMODE>), gd, bd, 0, st, P);
        else if (P.adam_p) hipLaunchKernelGGL((spmm_adam_pair_kernel<D, WMODE>), gd, bd, 0, st, P);
        else hipLaunchKernelGGL((spmm_pair_kernel<D, WMODE>), gd, bd, 0, st, P);
        BBGR_LAUNCHED("spmm_kernel");
        return BBGR_OK;
      }
    }
    if constexpr (D >= 64) {
      if (P.src_bits) {
        hipLaunchKernelGGL((spmm_bits_kernel<D, WMODE>), gd, bd, 0, st, P);
        BBGR_LAUNCHED("spmm_kernel");
        return BBGR_OK;
      }
    }
    if (masked) hipLaunchKernelGGL((spmm_masked_kernel<D, WMODE>), gd, bd, 0, st, P);
    else if (P.adam_p) hipLaunchKernelGGL((spmm_adam_kernel<D, WMODE>), gd, bd, 0, st, P);
    else hipLaunchKernelGGL((spmm_kernel<D, WMODE>), gd, bd, 0, st, P);
    BBGR_LAUNCHED("spmm_kernel");
  }
  (void)n_split;   // split rows are finished in-launch (split_row_arrive)
  return BBGR_OK;
}

template <int D>
static int dispatch_wmode(const SpmmParams &P, int wmode, int n_split,
                          hipStream_t st, bool tag_read) {
  switch (wmode) {
    case 0: return launch_spmm<D, 0>(P, n_split, st, tag_read);
    case 1: return launch_spmm<D, 1>(P, n_split, st, tag_read);
    case 2: return launch_spmm<D, 2>(P, n_split, st, tag_read);
  }
  set_error("bbgr_spmm: weight_mode %d not in {0,1,2}", wmode);
  return BBGR_ERR_INVALID;
}

// Two short rows per group for low-degree tables (average degree <= 24:
// the user side of the bipartite graph); BBGR_SPMM_PAIR=0/1 forces it off/on
// (A/B experiments).
static int pair_rows(const bbgr_csr *csr) {
  const char *env = getenv("BBGR_SPMM_PAIR");
  if (env && *env) return atoi(env) != 0;
  return csr->n_rows > 0 && csr->nnz <= 24L * csr->n_rows;
}

static bool ld_ok(const float *p, long ld, int d) {
  return p == nullptr || (aligned16(p) && ld >= d && (ld & 3) == 0);
}

}  // namespace bbgr

using namespace bbgr;

static void fill_epilogue(SpmmParams &P, const bbgr_spmm_args *a) {
  P.y = a->y;
  P.ldy = a->ldy;
  P.y_scale = a->y_scale;
  P.y_scale_s = a->y_scale_s;
  P.add = a->add;
  P.ldadd = a->ldadd;
  P.add_scale = a->add_scale;
  P.add_scale_s = a->add_scale_s;
  P.acc_in = a->acc_in;
  P.ldacc_in = a->ldacc_in;
  P.acc_out = a->acc_out;
  P.ldacc_out = a->ldacc_out;
  P.acc_scale = a->acc_scale;
  P.acc_scale_s = a->acc_scale_s;
  P.gamma = a->gamma;
  P.acc_mask = a->acc_mask;
  P.add_mask = a->add_mask;
  P.adam_p = a->adam_param;
  P.adam_m = a->adam_exp_avg;
  P.adam_v = a->adam_exp_avg_sq;
  P.adam_ld = a->adam_ld;
  P.adam_lr = a->adam_lr;
  P.adam_bc = a->adam_bc_table;
  P.adam_state = (const long *)a->adam_state;
  // with device step state the bias corrections come from the table (set
  // per launch from state[0]); 1.0 keeps the host-side constants finite
  const bool dev = a->adam_state != nullptr;
  P.adam = adam_consts(a->adam_lr, a->adam_beta1, a->adam_beta2, a->adam_eps,
                       a->adam_weight_decay, dev ? 1.f : a->adam_bias_correction1,
                       dev ? 1.f : a->adam_bias_correction2_sqrt);
  P.y_map = a->y_map;
  P.acc_map = a->acc_map;
  P.add_map = a->add_map;
  P.acc_in_map = a->acc_in_map;
  P.src_bits = a->src_bits;
  P.adam_g = a->adam_grad;
  P.adam_g_ld = a->adam_grad_ld;
  P.adam_g_scale = a->adam_grad_scale;
  P.adam_map = a->adam_map;
  P.adam_mrow = a->adam_moments_unmapped != 0;
  P.adam_mirror = a->adam_mirror;
  P.src_mask_bits = a->src_mask_bits;
}

static bool adam_ok(const bbgr_spmm_args *a, int d) {
  if (!a->adam_param) return !a->adam_mirror;
  if (a->adam_mirror && !(a->adam_moments_unmapped && ld_ok(a->adam_mirror, a->adam_ld, d)))
    return false;
  const bool dev = a->adam_state != nullptr;
  return a->adam_exp_avg && a->adam_exp_avg_sq && ld_ok(a->adam_param, a->adam_ld, d) &&
         ld_ok(a->adam_exp_avg, a->adam_ld, d) && ld_ok(a->adam_exp_avg_sq, a->adam_ld, d) &&
         (!a->adam_grad || ld_ok(a->adam_grad, a->adam_grad_ld, d)) &&
         (dev ? a->adam_bc_table != nullptr
              : (a->adam_bias_correction1 > 0.f && a->adam_bias_correction2_sqrt > 0.f));
}

extern "C" int bbgr_epilogue(int32_t n_rows, const float *t, int64_t ldt,
                             const bbgr_spmm_args *a, bbgr_stream_t stream) {
  BBGR_REQUIRE(a && n_rows >= 0, "bbgr_epilogue: bad args");
  const int d = a->d;
  if (!supported_width(d)) {
    set_error("bbgr_epilogue: embedding dim %d unsupported (8, 16, 32, 64, 128, 256)", d);
    return BBGR_ERR_UNSUPPORTED;
  }
  if (n_rows == 0) return BBGR_OK;
  BBGR_REQUIRE(t && ld_ok(t, ldt, d) && ld_ok(a->y, a->ldy, d) && ld_ok(a->add, a->ldadd, d) &&
                   ld_ok(a->acc_in, a->ldacc_in, d) && ld_ok(a->acc_out, a->ldacc_out, d) &&
                   adam_ok(a, d),
               "bbgr_epilogue: tables must be 16-byte aligned with ld >= d, ld % 4 == 0");
  BBGR_REQUIRE(!a->row_list || a->n_row_list >= 0, "bbgr_epilogue: negative n_row_list");
  SpmmParams P = {};
  P.n_rows = n_rows;
  P.nt_from = P.nt_out_from = 0x7fffffff;
  fill_epilogue(P, a);
  P.row_mask = a->row_mask;
  P.row_list = (const long *)a->row_list;
  P.n_row_list = a->n_row_list;
  const long n_in = a->row_list ? (long)a->n_row_list : (long)n_rows;
  if (n_in == 0) return BBGR_OK;
  const unsigned grid = (unsigned)((n_in + 15) / 16);
  hipStream_t st = as_stream(stream);
  switch (d) {
    case 8: hipLaunchKernelGGL(epilogue_kernel<8>, dim3(grid), dim3(256), 0, st, P, t, (long)ldt); break;
    case 16: hipLaunchKernelGGL(epilogue_kernel<16>, dim3(grid), dim3(256), 0, st, P, t, (long)ldt); break;
    case 32: hipLaunchKernelGGL(epilogue_kernel<32>, dim3(grid), dim3(256), 0, st, P, t, (long)ldt); break;
    case 64: hipLaunchKernelGGL(epilogue_kernel<64>, dim3(grid), dim3(256), 0, st, P, t, (long)ldt); break;
    case 128: hipLaunchKernelGGL(epilogue_kernel<128>, dim3(grid), dim3(256), 0, st, P, t, (long)ldt); break;
    default: hipLaunchKernelGGL(epilogue_kernel<256>, dim3(grid), dim3(256), 0, st, P, t, (long)ldt); break;
  }
  BBGR_LAUNCHED("epilogue_kernel");
  return BBGR_OK;
}

extern "C" int bbgr_spmm(const bbgr_csr *csr, const bbgr_spmm_args *a,
                         bbgr_stream_t stream) {
  BBGR_REQUIRE(csr && a, "bbgr_spmm: null csr/args");
  BBGR_REQUIRE(csr->n_rows >= 0 && csr->n_cols >= 0 && csr->nnz >= 0,
               "bbgr_spmm: negative csr size");
  BBGR_REQUIRE(csr->indptr && (csr->nnz == 0 || csr->indices),
               "bbgr_spmm: null csr arrays");
  const int d = a->d;
  if (!supported_width(d)) {
    set_error("bbgr_spmm: embedding dim %d unsupported (8, 16, 32, 64, 128, 256)", d);
    return BBGR_ERR_UNSUPPORTED;
  }
  BBGR_REQUIRE(a->x || csr->nnz == 0, "bbgr_spmm: null x");
  BBGR_REQUIRE(ld_ok(a->x, a->ldx, d) && ld_ok(a->y, a->ldy, d) &&
                   ld_ok(a->add, a->ldadd, d) && ld_ok(a->acc_in, a->ldacc_in, d) &&
                   ld_ok(a->acc_out, a->ldacc_out, d),
               "bbgr_spmm: tables must be 16-byte aligned with ld >= d, ld % 4 == 0");
  BBGR_REQUIRE(adam_ok(a, d), "bbgr_spmm: fused Adam needs param/exp_avg/exp_avg_sq "
                               "(16-byte aligned, adam_ld >= d) and bias corrections > 0");
  BBGR_REQUIRE(!a->adam_param || !(a->src_mask || a->row_mask || a->row_list || a->use_range),
               "bbgr_spmm: fused Adam needs every row (no masks, row list or range)");
  BBGR_REQUIRE(!a->src_mask_bits || a->src_mask,
               "bbgr_spmm: src_mask_bits packs src_mask (pass both)");
  BBGR_REQUIRE(!a->src_bits || a->src_mask,
               "bbgr_spmm: src_bits needs src_mask (narrow and two-row kernels read the mask)");
  BBGR_REQUIRE(a->weight_mode != 1 || a->edge_val, "bbgr_spmm: weight_mode 1 needs edge_val");
  BBGR_REQUIRE(a->weight_mode != 2 || a->col_scale, "bbgr_spmm: weight_mode 2 needs col_scale");
  BBGR_REQUIRE(csr->n_chunks == 0 || csr->chunks, "bbgr_spmm: plan chunks missing");
  BBGR_REQUIRE(csr->n_split == 0 || (csr->split && a->partial),
               "bbgr_spmm: split rows need plan + partial workspace");
  BBGR_REQUIRE(csr->n_chunks == 0 || csr->long_threshold > 0,
               "bbgr_spmm: plan without long_threshold");

  SpmmParams P = {};
  P.n_rows = csr->n_rows;
  P.long_threshold = csr->n_chunks ? csr->long_threshold : 0x7fffffff;
  P.n_chunks = csr->n_chunks;
  P.indptr = csr->indptr;
  P.indices = csr->indices;
  P.chunks = reinterpret_cast<const int4 *>(csr->chunks);
  P.split = reinterpret_cast<const int4 *>(csr->split);
  P.x = a->x;
  P.ldx = a->ldx;
  P.edge_val = a->edge_val;
  P.col_scale = a->col_scale;
  P.col_scale_s = a->col_scale_s;
  fill_epilogue(P, a);
  P.partial = a->partial;
  P.chunk_edges = csr->chunk_edges > 0 ? csr->chunk_edges : 2048;
  P.arrivals = a->partial ? reinterpret_cast<int *>(a->partial + (long)csr->n_chunks * d)
                          : nullptr;
  P.src_mask = a->src_mask;
  P.row_mask = a->row_mask;
  P.row_list = (const long *)a->row_list;
  P.n_row_list = a->n_row_list;
  P.row_count = (const long *)a->row_count;
  BBGR_REQUIRE(!a->row_count || a->row_list, "bbgr_spmm: row_count needs row_list");
  int n_split = csr->n_split;
  P.row_begin = 0;
  P.row_end = csr->n_rows;
  P.chunk_begin = 0;
  if (a->use_range) {
    const int *r = a->range;
    BBGR_REQUIRE(r[0] >= 0 && r[0] <= r[1] && r[1] <= csr->n_rows && r[2] >= 0 &&
                     r[2] <= r[3] && r[3] <= csr->n_chunks && r[4] >= 0 && r[4] <= r[5] &&
                     r[5] <= csr->n_split,
                 "bbgr_spmm: range out of bounds");
    BBGR_REQUIRE(!a->row_list || a->row_mask,
                 "bbgr_spmm: range with row_list needs row_mask (chunk rows)");
    if (!a->row_list) {   // with a row list the short rows are the list's entries
      P.row_begin = r[0];
      P.row_end = r[1];
    }
    P.chunk_begin = r[2];
    P.n_chunks = r[3] - r[2];
    P.split = reinterpret_cast<const int4 *>(csr->split) + r[4];
    n_split = r[5] - r[4];
  }
  BBGR_REQUIRE(!a->row_list || a->n_row_list >= 0, "bbgr_spmm: negative n_row_list");
  // chunk workgroups of a list launch compute only rows flagged in row_mask:
  // without the mask, long listed rows would be skipped
  BBGR_REQUIRE(!a->row_list || a->row_mask || csr->n_chunks == 0,
               "bbgr_spmm: row_list needs row_mask when the plan has long-row chunks");
  P.pair_rows = d >= 64 && pair_rows(csr);
  // tagged indices: a full launch writes the copy, a masked one reads it
  BBGR_REQUIRE(!a->tag_out || (a->tag_mask && !a->src_tagged && !a->src_mask && !a->row_mask &&
                               !a->row_list && !a->use_range && !a->adam_param),
               "bbgr_spmm: tag_out needs tag_mask and a full launch (no masks, list, range or "
               "fused Adam)");
  BBGR_REQUIRE(!a->src_tagged || (!a->src_mask && !a->src_bits && !a->adam_param),
               "bbgr_spmm: src_tagged replaces src_mask (no src_mask / src_bits / fused Adam)");
  const bool tag_read = a->src_tagged != nullptr;
  P.tag_out = a->tag_out;
  P.tag_mask = a->tag_mask;
  if (tag_read) P.indices = a->src_tagged;
  P.nt_from = a->stream_from > 0 ? a->stream_from : 0x7fffffff;
  P.nt_out_from = a->stream_out_from > 0 ? a->stream_out_from : 0x7fffffff;
  hipStream_t st = as_stream(stream);
  switch (d) {
    case 8: return dispatch_wmode<8>(P, a->weight_mode, n_split, st, tag_read);
    case 16: return dispatch_wmode<16>(P, a->weight_mode, n_split, st, tag_read);
    case 32: return dispatch_wmode<32>(P, a->weight_mode, n_split, st, tag_read);
    case 64: return dispatch_wmode<64>(P, a->weight_mode, n_split, st, tag_read);
    case 128: return dispatch_wmode<128>(P, a->weight_mode, n_split, st, tag_read);
    default: return dispatch_wmode<256>(P, a->weight_mode, n_split, st, tag_read);
  }
}

// ---------------------------------------------------------------------------
// The entry-point names of SURVEY §8(b)'s ABI sketch, kept as thin forms of
// the entry points above (include/bbgr.h, "Blueprint names").
// ---------------------------------------------------------------------------
extern "C" int bbgr_spmm_f32(const bbgr_csr *A, const float *X, int64_t ldx, float *Y,
                             int64_t ldy, int32_t d, const float *row_scale,
                             const float *col_scale, float *acc, float acc_scale,
                             bbgr_stream_t stream) {
  BBGR_REQUIRE(A, "bbgr_spmm_f32: null csr");
  BBGR_REQUIRE(A->n_split == 0,
               "bbgr_spmm_f32: the plan has split rows; use bbgr_spmm with a partial workspace");
  bbgr_spmm_args a;
  std::memset(&a, 0, sizeof a);
  a.d = d;
  a.x = X;
  a.ldx = ldx;
  a.weight_mode = col_scale ? 2 : 0;
  a.col_scale = col_scale;
  a.col_scale_s = 1.f;
  a.y = Y;
  a.ldy = ldy;
  a.y_scale = row_scale;
  a.y_scale_s = 1.f;
  if (acc) {   // acc += acc_scale * Y: the epilogue adds acc_scale * row_scale * T
    a.acc_in = acc;
    a.ldacc_in = ldy;
    a.acc_out = acc;
    a.ldacc_out = ldy;
    a.acc_scale = row_scale;
    a.acc_scale_s = acc_scale;
  }
  a.gamma = 1.f;
  return bbgr_spmm(A, &a, stream);
}

extern "C" int bbgr_bpr_fwd_bwd(const bbgr_bpr_args *args, bbgr_stream_t stream) {
  return bbgr_bpr(args, stream);
}

extern "C" int bbgr_adam_f32(int64_t n, float *param, const float *grad, float *exp_avg,
                             float *exp_avg_sq, float lr, float beta1, float beta2, float eps,
                             float weight_decay, float grad_scale, float bias_correction1,
                             float bias_correction2_sqrt, bbgr_stream_t stream) {
  return bbgr_adam(n, param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay,
                   grad_scale, bias_correction1, bias_correction2_sqrt, stream);
}

extern "C" int bbgr_negsample(int64_t batch, const int64_t *users, const int32_t *indptr,
                              const int32_t *indices, int32_t n_items, const double *cdf,
                              float mix_pop, int32_t max_tries, uint64_t seed, uint64_t counter,
                              int64_t *pos, int64_t *neg, int32_t *fail_count,
                              bbgr_stream_t stream) {
  return bbgr_sample(batch, users, indptr, indices, n_items, cdf, mix_pop, max_tries, seed,
                     counter, pos, neg, fail_count, stream);
}
