// Shared helpers for the bbgr HIP sources: error state, launch checks,
// Philox4x32-10 counter-based RNG. gfx950 (CDNA4, wave64) only.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string>

#include "bbgr.h"

namespace bbgr {

void set_error(const char *fmt, ...);

inline int hip_fail(hipError_t e, const char *what) {
  set_error("%s: %s", what, hipGetErrorString(e));
  return BBGR_ERR_HIP;
}

#define BBGR_HIP(call)                                                        \
  do {                                                                        \
    hipError_t e_ = (call);                                                   \
    if (e_ != hipSuccess) return ::bbgr::hip_fail(e_, #call);                 \
  } while (0)

#define BBGR_LAUNCHED(name)                                                   \
  do {                                                                        \
    hipError_t e_ = hipGetLastError();                                        \
    if (e_ != hipSuccess) return ::bbgr::hip_fail(e_, "launch " name);       \
  } while (0)

#define BBGR_REQUIRE(cond, msg)                                               \
  do {                                                                        \
    if (!(cond)) {                                                            \
      ::bbgr::set_error("%s", msg);                                           \
      return BBGR_ERR_INVALID;                                                \
    }                                                                         \
  } while (0)

inline hipStream_t as_stream(bbgr_stream_t s) {
  return reinterpret_cast<hipStream_t>(s);
}

inline bool aligned16(const void *p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

// Round a workspace carve offset up to 256 bytes.
inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11). Counter (c0..c3), key (k0,k1).
// ---------------------------------------------------------------------------
struct u32x4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0,
                                               uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    const uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// 53-bit uniform double in [0,1) from two 32-bit words.
__device__ __forceinline__ double u01_53(uint32_t a, uint32_t b) {
  const uint64_t v = ((uint64_t)a << 32 | b) >> 11;
  return (double)v * (1.0 / 9007199254740992.0);
}

// ---------------------------------------------------------------------------
// Row shape of a d-wide fp32 table row held by one 16-lane group: d >= 64 ->
// all 16 lanes, V = d/64 float4 each (lane l holds float4 columns l, l+16, ..);
// narrow rows (d = 8, 16, 32: the column slices of a column-sharded table)
// -> the first d/4 lanes, one float4 each; the other lanes idle.
// ---------------------------------------------------------------------------
template <int D> struct RowShape {
  static_assert(D == 8 || D == 16 || D == 32 || D == 64 || D == 128 || D == 256,
                "row width");
  static constexpr int LANES = D >= 64 ? 16 : D / 4;
  static constexpr int V = D >= 64 ? D / 64 : 1;
};

inline bool supported_width(int d) {
  return d == 8 || d == 16 || d == 32 || d == 64 || d == 128 || d == 256;
}

// Streaming (non-temporal) 16-byte loads / stores: data touched once per
// pass that should not displace cached rows.
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_nt(const float4 *p) {
  const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ int ld_nt(const int *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ float ld_nt(const float *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st_nt(float4 *p, float4 v) {
  f4v w;
  w.x = v.x;
  w.y = v.y;
  w.z = v.z;
  w.w = v.w;
  __builtin_nontemporal_store(w, reinterpret_cast<f4v *>(p));
}

// ---------------------------------------------------------------------------
// torch.optim.Adam on one element (amsgrad=False, maximize=False). Shared by
// adam_kernel and the SpMM epilogue's fused step with every rounding spelled
// out (explicit fmaf, no contraction) so the two paths agree bit for bit.
// ---------------------------------------------------------------------------
struct AdamConsts {
  float step;   // lr / bias_correction1
  float w1;     // 1 - beta1
  float b2;     // beta2
  float w2;     // 1 - beta2
  float eps;
  float wd;     // weight_decay
  float bc2s;   // sqrt(bias_correction2)
};

__host__ __device__ inline AdamConsts adam_consts(float lr, float b1, float b2, float eps,
                                                  float wd, float bc1, float bc2s) {
  return AdamConsts{lr / bc1, 1.0f - b1, b2, 1.0f - b2, eps, wd, bc2s};
}

__device__ __forceinline__ void adam_elem(float &p, float g, float &m, float &v,
                                          const AdamConsts &c) {
#pragma clang fp contract(off)
  if (c.wd != 0.f) g = fmaf(c.wd, p, g);
  m = fmaf(c.w1, g - m, m);                    // lerp(m, g, 1 - beta1)
  v = fmaf(c.w2 * g, g, v * c.b2);             // beta2 v + (1 - beta2) g^2
  const float denom = sqrtf(v) / c.bc2s + c.eps;
  p = fmaf(-c.step, m / denom, p);             // p - lr/bc1 * m / denom
}

// Device step state {t, counter, next counter, table length} (bbgr_step_begin):
// the step t clamped into the bias-correction table [1, state[3]]. Exact: in
// fp32 both 1 - beta1^t and sqrt(1 - beta2^t) reach 1.0f long before any table
// length the host builds (2^20 steps), so every t past the end reads the same
// constants its own entry would hold; a replayed graph can never read past it.
__device__ __forceinline__ long clamp_step(const long *state) {
  const long t = state[0], n = state[3];
  return t < 1 ? 1 : (t > n ? n : t);
}

// The load-balance plan's chunk count of a row of `deg` edges (plan_counts_kernel):
// 0 for a short row (deg <= thr), else ceil(deg / chunk). Every reader of the
// plan derives a row's chunking from this one rule (split_row_arrive's chunk
// index, the slot-bitmap kernel's single-chunk rows).
__host__ __device__ __forceinline__ int plan_chunks(long deg, int thr, int chunk) {
  return deg > thr ? (int)((deg + chunk - 1) / chunk) : 0;
}

}  // namespace bbgr
