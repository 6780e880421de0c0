// XCD-local column slices for small-graph SpMM gathers:
// does gathering 32-B row slices from a table slice that fits one XCD's 4 MB
// L2 beat gathering whole 256-B rows from the Infinity Cache?
//
//   hipcc --offload-arch=gfx950 -O3 -o xcd_slice_probe xcd_slice_probe.hip
//   ./xcd_slice_probe [rows_out] [rows_src] [deg]     (C2 item<-user: 50000 100000 20)
//
// Three kernels compute out[r] = sum over its deg edges of src[idx[e]] (d = 64
// fp32), the edge lists random, the same sums:
//   whole   one 16-lane group per output row, each lane a float4 of the
//           256-B source row (the product kernels' shape)
//   xcd     the tables in 8 column slices [8][rows][8]; workgroup b serves
//           slice b % 8, so with round-robin workgroup dispatch each XCD
//           gathers from one 1.6-3.2 MB slice only; 2 lanes (2 float4) per
//           row slice, 8 rows per 16 lanes
//   blocked the same slices with slice b / (blocks / 8): every XCD sees
//           every slice (the control for the XCD placement)
// Prints ms per launch and the gather rate (edges * 256 B / t).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

__global__ __launch_bounds__(256) void whole_kernel(int n_out, int deg, const int *idx,
                                                    const float4 *src, float4 *out) {
  const int r = blockIdx.x * 16 + (threadIdx.x >> 4);
  const int lane = threadIdx.x & 15;
  if (r >= n_out) return;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int *e = idx + (long)r * deg;
  for (int k = 0; k < deg; ++k) {
    const float4 v = src[(long)e[k] * 16 + lane];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  out[(long)r * 16 + lane] = acc;
}

// slices: src_s[s][row][2 float4], out_s[s][row][2 float4]
template <bool XCD>
__global__ __launch_bounds__(256) void slice_kernel(int n_out, int n_src, int deg,
                                                    int blocks_per_slice, const int *idx,
                                                    const float4 *src_s, float4 *out_s) {
  const int s = XCD ? (int)(blockIdx.x % 8) : (int)(blockIdx.x / blocks_per_slice);
  const int b = XCD ? (int)(blockIdx.x / 8) : (int)(blockIdx.x % blocks_per_slice);
  const int r = b * 128 + (threadIdx.x >> 1);   // 128 rows per 256 threads
  const int h = threadIdx.x & 1;
  if (r >= n_out) return;
  const float4 *S = src_s + (long)s * n_src * 2;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int *e = idx + (long)r * deg;
  for (int k = 0; k < deg; ++k) {
    const float4 v = S[(long)e[k] * 2 + h];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  out_s[((long)s * n_out + r) * 2 + h] = acc;
}

int main(int argc, char **argv) {
  const int n_out = argc > 1 ? std::atoi(argv[1]) : 50000;
  const int n_src = argc > 2 ? std::atoi(argv[2]) : 100000;
  const int deg = argc > 3 ? std::atoi(argv[3]) : 20;
  const long E = (long)n_out * deg;
  std::mt19937 g(7);
  std::uniform_int_distribution<int> U(0, n_src - 1);
  std::vector<int> h_idx(E);
  for (auto &x : h_idx) x = U(g);
  std::vector<float> h_src((size_t)n_src * 64);
  for (size_t i = 0; i < h_src.size(); ++i) h_src[i] = (float)((i * 2654435761u) % 1000) / 997.f;
  std::vector<float> h_src_s(h_src.size());   // [8][rows][8]
  for (int r = 0; r < n_src; ++r)
    for (int c = 0; c < 64; ++c) h_src_s[((size_t)(c / 8) * n_src + r) * 8 + c % 8] = h_src[(size_t)r * 64 + c];
  int *d_idx;
  float4 *d_src, *d_src_s, *d_out, *d_out_s;
  CK(hipMalloc(&d_idx, E * 4));
  CK(hipMalloc(&d_src, h_src.size() * 4));
  CK(hipMalloc(&d_src_s, h_src.size() * 4));
  CK(hipMalloc(&d_out, (size_t)n_out * 256));
  CK(hipMalloc(&d_out_s, (size_t)n_out * 256));
  CK(hipMemcpy(d_idx, h_idx.data(), E * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_src, h_src.data(), h_src.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_src_s, h_src_s.data(), h_src.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int bps = (n_out + 127) / 128;
  auto run = [&](int which) {
    if (which == 0)
      hipLaunchKernelGGL(whole_kernel, dim3((n_out + 15) / 16), dim3(256), 0, 0, n_out, deg, d_idx,
                         d_src, d_out);
    else if (which == 1)
      hipLaunchKernelGGL(slice_kernel<true>, dim3(8 * bps), dim3(256), 0, 0, n_out, n_src, deg, bps,
                         d_idx, d_src_s, d_out_s);
    else
      hipLaunchKernelGGL(slice_kernel<false>, dim3(8 * bps), dim3(256), 0, 0, n_out, n_src, deg,
                         bps, d_idx, d_src_s, d_out_s);
  };
  const char *names[3] = {"whole", "xcd", "blocked"};
  for (int rep = 0; rep < 2; ++rep)
    for (int w = 0; w < 3; ++w) {
      for (int i = 0; i < 5; ++i) run(w);
      CK(hipDeviceSynchronize());
      const int iters = 50;
      CK(hipEventRecord(a, 0));
      for (int i = 0; i < iters; ++i) run(w);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, a, b));
      ms /= iters;
      std::printf("%-8s rows_out %d rows_src %d deg %d: %.4f ms  gather %.2f TB/s\n", names[w],
                  n_out, n_src, deg, ms, (double)E * 256 / (ms * 1e-3) / 1e12);
    }
  // the three agree (same sums, same order)
  std::vector<float> o((size_t)n_out * 64), os((size_t)n_out * 64);
  run(0);
  run(1);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(o.data(), d_out, o.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(os.data(), d_out_s, os.size() * 4, hipMemcpyDeviceToHost));
  long bad = 0;
  for (int r = 0; r < n_out; ++r)
    for (int c = 0; c < 64; ++c)
      bad += o[(size_t)r * 64 + c] != os[((size_t)(c / 8) * n_out + r) * 8 + c % 8];
  std::printf("mismatches %ld\n", bad);
  return bad != 0;
}
