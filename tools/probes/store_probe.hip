// Store-pattern probe (round 5): why the two-rows-per-group SpMM kernels
// issue more L2 write requests than the one-row kernels for the same dense
// output table (profiles/round5/r5c_*: TCC_WRITE 32.5M vs 20.0M per 1.28 GB).
// Writes a 5M x 64 fp32 table with the store shapes of spmm.hip's epilogues:
//   mode 0  one row per 16-lane group, 16 rows per 256-thread block
//   mode 1  two rows per group (rows j, j+16), 32 rows per block, stored A then B
//   mode 2  mode 1 with a per-group data-dependent delay before each store
//   mode 3  mode 0 with the same delay
//   mode 4  mode 1, rows (2g, 2g+1) per group instead of (g, g+16)
// nt = 1: non-temporal stores. Run under rocprofv3 --pmc TCC_WRITE_sum ...
//   hipcc --offload-arch=gfx950 -O3 -o store_probe store_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st(float4 *p, float4 v, int nt) {
  if (nt) {
    f4v w;
    w.x = v.x;
    w.y = v.y;
    w.z = v.z;
    w.w = v.w;
    __builtin_nontemporal_store(w, reinterpret_cast<f4v *>(p));
  } else {
    *p = v;
  }
}

__device__ __forceinline__ float4 spin(int row, float4 v, int delay) {
  // a data-dependent amount of work per group (0..delay iterations)
  const int n = delay ? (int)((row * 2654435761u) >> 27) % delay : 0;
  for (int i = 0; i < n; ++i) v.x = v.x * 1.0000001f + 1e-7f;
  return v;
}

__global__ __launch_bounds__(256) void probe(float *y, int n_rows, int mode, int nt, int delay) {
  const int g = threadIdx.x >> 4, lane = threadIdx.x & 15;
  if (mode == 0 || mode == 3) {
    const int row = blockIdx.x * 16 + g;
    if (row >= n_rows) return;
    float4 v = make_float4(row, lane, 1.f, 2.f);
    if (mode == 3) v = spin(row, v, delay);
    st(reinterpret_cast<float4 *>(y + (long)row * 64) + lane, v, nt);
    return;
  }
  int ra, rb;
  if (mode == 4) {
    ra = blockIdx.x * 32 + 2 * g;
    rb = ra + 1;
  } else {
    ra = blockIdx.x * 32 + g;
    rb = ra + 16;
  }
  float4 va = make_float4(ra, lane, 1.f, 2.f), vb = make_float4(rb, lane, 1.f, 2.f);
  if (mode == 2) {
    va = spin(ra, va, delay);
    vb = spin(rb, vb, delay);
  }
  if (ra < n_rows) st(reinterpret_cast<float4 *>(y + (long)ra * 64) + lane, va, nt);
  if (rb < n_rows) st(reinterpret_cast<float4 *>(y + (long)rb * 64) + lane, vb, nt);
}

int main(int argc, char **argv) {
  const int n_rows = 5000000;
  const int delay = argc > 1 ? atoi(argv[1]) : 64;
  float *y;
  if (hipMalloc(&y, (size_t)n_rows * 64 * 4) != hipSuccess) return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep) {
    for (int mode = 0; mode < 5; ++mode) {
      for (int nt = 0; nt < 2; ++nt) {
        const int per = (mode == 0 || mode == 3) ? 16 : 32;
        const int grid = (n_rows + per - 1) / per;
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(probe, dim3(grid), dim3(256), 0, 0, y, n_rows, mode, nt, delay);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, a, b);
        if (rep == 2) printf("mode %d nt %d: %.3f ms (%.2f TB/s)\n", mode, nt, ms,
                             n_rows * 256.0 / (ms * 1e9));
      }
    }
  }
  (void)hipFree(y);
  return 0;
}
