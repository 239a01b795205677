// Do float64 MFMA (v_mfma_f64_16x16x4_f64) and float64 VALU FMAs (v_fma_f64) share the SIMD's DP
// hardware on gfx950?  One wave per SIMD (1 024 one-wave blocks), three loops of the same length:
//   M: 8 independent float64 MFMA accumulators per iteration
//   V: 64 float64 FMAs per lane per iteration (16 independent chains)
//   X: both in one iteration (the wave issues the MFMAs and the FMAs interleaved, in order)
// Separate pipes: X ~ max(M, V).  Shared: X ~ M + V.
//     hipcc -O3 --offload-arch=gfx950 tools/calib/dp_pipes.hip -o tools/calib/dp_pipes && ./tools/calib/dp_pipes
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int kBlocks = 1024, kThreads = 64, kMaxBlocks = 4096;

template <bool DO_M, bool DO_V>
__global__ __launch_bounds__(kThreads) void k_loop(int n, double* out) {
  d4 acc[8];
  double x[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = 1.0 + (threadIdx.x + i) * 1e-9;
  const double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9, m = 0.999999999, c = 1e-12;
  for (int it = 0; it < n; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (DO_M) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
      if (DO_V) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[(k & 1) * 8 + i] = fma(x[(k & 1) * 8 + i], m, c);
      }
    }
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
#pragma unroll
  for (int i = 0; i < 16; ++i) s += x[i];
  out[blockIdx.x * kThreads + threadIdx.x] = s;  // out holds kMaxBlocks * kThreads doubles (grids <= kMaxBlocks)
}

int main() {
  double* out = nullptr;
  if (hipMalloc(&out, sizeof(double) * kMaxBlocks * kThreads) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int n = 4000;
  float t[3] = {0, 0, 0};
  for (int rep = 0; rep < 2; ++rep) {
    for (int k = 0; k < 3; ++k) {
      (void)hipEventRecord(e0);
      if (k == 0) hipLaunchKernelGGL((k_loop<true, false>), dim3(kBlocks), dim3(kThreads), 0, 0, n, out);
      if (k == 1) hipLaunchKernelGGL((k_loop<false, true>), dim3(kBlocks), dim3(kThreads), 0, 0, n, out);
      if (k == 2) hipLaunchKernelGGL((k_loop<true, true>), dim3(kBlocks), dim3(kThreads), 0, 0, n, out);
      const hipError_t le = hipGetLastError();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&t[k], e0, e1);
      if (le != hipSuccess) { printf("launch %d: %s\n", k, hipGetErrorString(le)); return 1; }
    }
  }
  const double mfma = (double)kBlocks * n * 8, fma_lane = (double)kBlocks * kThreads * n * 64;
  printf("M %.3f ms: %.1f TF f64 MFMA (%.0f cycles per MFMA per SIMD at 2.4 GHz)\n", t[0], 2 * mfma * 1024 / t[0] / 1e9,
         t[0] * 1e-3 * 2.4e9 / (n * 8.0));
  printf("V %.3f ms: %.1f TF f64 VALU (one wave per SIMD)\n", t[1], 2 * fma_lane / t[1] / 1e9);
  printf("X %.3f ms: both in one wave; separate pipes ~max(M, V) = %.3f, shared ~M + V = %.3f\n", t[2],
         t[0] > t[1] ? t[0] : t[1], t[0] + t[1]);
  // the MFMA loop at 2 and 4 waves per SIMD (2 048 / 4 096 blocks): is one wave per SIMD latency-limited?
  for (int w = 2; w <= 4; w *= 2) {
    float tm = 0;
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL((k_loop<true, false>), dim3(kBlocks * w), dim3(kThreads), 0, 0, n, out);
      const hipError_t le = hipGetLastError();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&tm, e0, e1);
      if (le != hipSuccess) { printf("launch: %s\n", hipGetErrorString(le)); return 1; }
    }
    printf("M x%d waves per SIMD %.3f ms: %.1f TF f64 MFMA\n", w, tm, 2 * mfma * w * 1024 / tm / 1e9);
  }
  (void)hipFree(out);
  return 0;
}
