// Probe: launch shapes of the separate Adam step (28 B per parameter: p, g,
// m, v in; p, m, v out) on the C4 user table (5M x 64) and item table
// (1M x 64), against a plain copy and a 4-read / 3-write stream with no math.
// Every Adam variant runs adam_elem (common.h) on the same elements, so all
// give the same bits; the probe checks that against variant 0.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include \
//     -I <pkg>/csrc tools/adam_variants.hip -o tools/adam_variants
//   ./tools/adam_variants [reps]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "common.h"

using namespace bbgr;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__device__ __forceinline__ void upd4(float4 &pp, float4 gg, float4 &mm, float4 &vv,
                                     const AdamConsts &c) {
  adam_elem(pp.x, gg.x, mm.x, vv.x, c);
  adam_elem(pp.y, gg.y, mm.y, vv.y, c);
  adam_elem(pp.z, gg.z, mm.z, vv.z, c);
  adam_elem(pp.w, gg.w, mm.w, vv.w, c);
}

// 0: the shipped form (grid-stride, one float4 per stream per iteration)
__global__ __launch_bounds__(256) void adam_v0(long n4, float4 *p, const float4 *g, float4 *m,
                                               float4 *v, AdamConsts c) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    float4 pp = p[i], gg = g[i], mm = m[i], vv = v[i];
    upd4(pp, gg, mm, vv, c);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

// 1: U float4 per stream per iteration, all loads issued before the math;
// optional non-temporal loads / stores
template <int U, bool NT>
__global__ __launch_bounds__(256) void adam_vu(long n4, float4 *p, const float4 *g, float4 *m,
                                               float4 *v, AdamConsts c) {
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    float4 pp[U], gg[U], mm[U], vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long k = i + u * stride;
      if (NT) {
        pp[u] = ld_nt(p + k);
        gg[u] = ld_nt(g + k);
        mm[u] = ld_nt(m + k);
        vv[u] = ld_nt(v + k);
      } else {
        pp[u] = p[k];
        gg[u] = g[k];
        mm[u] = m[k];
        vv[u] = v[k];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) upd4(pp[u], gg[u], mm[u], vv[u], c);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long k = i + u * stride;
      if (NT) {
        st_nt(p + k, pp[u]);
        st_nt(m + k, mm[u]);
        st_nt(v + k, vv[u]);
      } else {
        p[k] = pp[u];
        m[k] = mm[u];
        v[k] = vv[u];
      }
    }
  }
  for (; i < n4; i += stride) {
    float4 pp = p[i], gg = g[i], mm = m[i], vv = v[i];
    upd4(pp, gg, mm, vv, c);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

// 2: each workgroup owns a contiguous tile of T float4 per stream (U per
// thread, consecutive threads on consecutive float4): a workgroup's four
// read streams and three write streams stay within a few DRAM pages
template <int U, bool NT>
__global__ __launch_bounds__(256) void adam_tile(long n4, float4 *p, const float4 *g, float4 *m,
                                                 float4 *v, AdamConsts c) {
  const long tile = 256L * U;
  for (long t0 = (long)blockIdx.x * tile; t0 < n4; t0 += (long)gridDim.x * tile) {
    float4 pp[U], gg[U], mm[U], vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long k = t0 + u * 256 + threadIdx.x;
      if (k < n4) {
        if (NT) {
          pp[u] = ld_nt(p + k);
          gg[u] = ld_nt(g + k);
          mm[u] = ld_nt(m + k);
          vv[u] = ld_nt(v + k);
        } else {
          pp[u] = p[k];
          gg[u] = g[k];
          mm[u] = m[k];
          vv[u] = v[k];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long k = t0 + u * 256 + threadIdx.x;
      if (k < n4) {
        upd4(pp[u], gg[u], mm[u], vv[u], c);
        if (NT) {
          st_nt(p + k, pp[u]);
          st_nt(m + k, mm[u]);
          st_nt(v + k, vv[u]);
        } else {
          p[k] = pp[u];
          m[k] = mm[u];
          v[k] = vv[u];
        }
      }
    }
  }
}

// ceilings: a copy (1 read, 1 write) and 4 reads / 3 writes with no math
__global__ __launch_bounds__(256) void copy_k(long n4, const float4 *a, float4 *b) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x)
    b[i] = a[i];
}
__global__ __launch_bounds__(256) void rw43_k(long n4, float4 *p, const float4 *g, float4 *m,
                                              float4 *v) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    float4 pp = p[i], gg = g[i], mm = m[i], vv = v[i];
    p[i] = make_float4(pp.x + gg.x, pp.y + gg.y, pp.z + gg.z, pp.w + gg.w);
    m[i] = mm;
    v[i] = vv;
  }
}

struct Bufs {
  float4 *p, *g, *m, *v;
};

static void fill(const Bufs &b, long n4, const float *h, float4 *pm, float4 *pv) {
  CK(hipMemcpy(b.p, h, n4 * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(b.g, h + 4 * n4, n4 * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(b.m, pm, n4 * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(b.v, pv, n4 * 16, hipMemcpyHostToDevice));
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 30;
  const AdamConsts c = adam_consts(1e-3f, 0.9f, 0.999f, 1e-8f, 0.f, 1.f - 0.9f * 0.9f,
                                   sqrtf(1.f - 0.999f * 0.999f));
  const long rows_list[2] = {5000000, 1000000};
  printf("[");
  bool first = true;
  for (int ri = 0; ri < 2; ++ri) {
    const long n = rows_list[ri] * 64, n4 = n / 4;
    Bufs b;
    CK(hipMalloc(&b.p, n * 4));
    CK(hipMalloc(&b.g, n * 4));
    CK(hipMalloc(&b.m, n * 4));
    CK(hipMalloc(&b.v, n * 4));
    float *h = (float *)malloc(n * 8);
    float *hm = (float *)malloc(n * 4), *hv = (float *)malloc(n * 4);
    unsigned s = 12345u;
    for (long i = 0; i < 2 * n; ++i) {
      s = s * 1664525u + 1013904223u;
      h[i] = ((s >> 8) * (1.0f / 16777216.0f)) - 0.5f;
    }
    for (long i = 0; i < n; ++i) {
      hm[i] = 0.1f * h[i];
      hv[i] = h[i] * h[i] * 0.01f;
    }
    float *ref = (float *)malloc(n * 4), *out = (float *)malloc(n * 4);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct V {
      const char *name;
      int kind;
      long grid;
    };
    const long full = (n4 + 255) / 256;
    V vs[] = {{"v0_cap4096", 0, 4096},      {"v0_full", 0, full},
              {"u2_cap4096", 1, 4096},      {"u4_cap4096", 2, 4096},
              {"u2_cap2048", 1, 2048},      {"u2nt_cap4096", 3, 4096},
              {"u4nt_cap2048", 4, 2048},    {"tile4_cap4096", 5, 4096},
              {"tile8_cap2048", 6, 2048},   {"tile4nt_cap4096", 7, 4096},
              {"tile4_full", 5, (n4 + 1023) / 1024}, {"tile4nt_full", 7, (n4 + 1023) / 1024},
              {"tile4nt_cap8192", 7, 8192}, {"tile4nt_cap2048", 7, 2048},
              {"tile2nt_cap4096", 10, 4096}, {"tile2nt_full", 10, (n4 + 511) / 512},
              {"tile8nt_cap2048", 11, 2048}, {"tile8nt_full", 11, (n4 + 2047) / 2048},
              {"copy", 8, 4096},
              {"rw43", 9, 4096}};
    for (const V &vv : vs) {
      fill(b, n4, h, (float4 *)hm, (float4 *)hv);
      auto launch = [&]() {
        const dim3 gd((unsigned)vv.grid), bd(256);
        switch (vv.kind) {
          case 0: hipLaunchKernelGGL(adam_v0, gd, bd, 0, 0, n4, b.p, b.g, b.m, b.v, c); break;
          case 1: hipLaunchKernelGGL((adam_vu<2, false>), gd, bd, 0, 0, n4, b.p, b.g, b.m, b.v, c); break;
          case 2: hipLaunchKernelGGL((adam_vu<4, false>), gd, bd, 0, 0, n4, b.p, b.g, b.m, b.v, c); break;
          case 3: hipLaunchKernelGGL((adam_vu<2, true>), gd, bd, 0, 0, n4, b.p, b.g, b.m, b.v, c); break;
          case 4: hipLaunchKernelGGL((adam_vu<4, true>), gd, bd, 0, 0, n4, b.p, b.g, b.m, b.v, c); break;
          case 5: hipLaunchKernelGGL((adam_tile<4, false>), gd, bd, 0, 0, n4, b.p, b.g, b.m, b.v, c); break;
          case 6: hipLaunchKernelGGL((adam_tile<8, false>), gd, bd, 0, 0, n4, b.p, b.g, b.m, b.v, c); break;
          case 7: hipLaunchKernelGGL((adam_tile<4, true>), gd, bd, 0, 0, n4, b.p, b.g, b.m, b.v, c); break;
          case 10: hipLaunchKernelGGL((adam_tile<2, true>), gd, bd, 0, 0, n4, b.p, b.g, b.m, b.v, c); break;
          case 11: hipLaunchKernelGGL((adam_tile<8, true>), gd, bd, 0, 0, n4, b.p, b.g, b.m, b.v, c); break;
          case 8: hipLaunchKernelGGL(copy_k, gd, bd, 0, 0, n4, b.g, b.m); break;
          default: hipLaunchKernelGGL(rw43_k, gd, bd, 0, 0, n4, b.p, b.g, b.m, b.v); break;
        }
      };
      // one step from the same state for the bit check
      launch();
      CK(hipDeviceSynchronize());
      bool same = true;
      if (vv.kind <= 7 || vv.kind >= 10) {
        CK(hipMemcpy(out, b.p, n * 4, hipMemcpyDeviceToHost));
        if (vv.kind == 0 && vv.grid == 4096) memcpy(ref, out, n * 4);
        else same = memcmp(ref, out, n * 4) == 0;
      }
      for (int w = 0; w < 3; ++w) launch();
      CK(hipEventRecord(e0, 0));
      for (int r = 0; r < reps; ++r) launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      const double bytes = vv.kind == 8 ? 8.0 * n : 28.0 * n;  // copy: 1 read + 1 write
      printf("%s{\"rows\": %ld, \"variant\": \"%s\", \"grid\": %ld, \"ms\": %.4f, \"TBps\": %.3f, "
             "\"bitwise_v0\": %s}\n",
             first ? "" : ",", rows_list[ri], vv.name, vv.grid, ms, bytes / (ms * 1e-3) / 1e12,
             same ? "true" : "false");
      first = false;
      fflush(stdout);
    }
    CK(hipFree(b.p));
    CK(hipFree(b.g));
    CK(hipFree(b.m));
    CK(hipFree(b.v));
    free(h);
    free(hm);
    free(hv);
    free(ref);
    free(out);
  }
  printf("]\n");
  return 0;
}
