// Issue-rate probe: scalar v_fma_f32 / v_add_f32 vs packed v_pk_fma_f32 / v_pk_add_f32 (gfx950).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float pk2 __attribute__((ext_vector_type(2)));
template <int MODE>
__global__ void k(float* out, int iters) {
  float a[8]; pk2 p[8];
  for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * 0.001f + i; p[i] = pk2{a[i], a[i] + 1.f}; }
  const float b = 1.0001f, c = 0.5f; const pk2 pb = {b, b}, pc = {c, c};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (MODE == 0) {  // 2 scalar fma per "pair"
        float x = a[i], y = a[i] + 0.f;
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(p[i].x) : "v"(b), "v"(c));
        (void)x; (void)y;
      } else if (MODE == 1) {
        asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[i]) : "v"(pb), "v"(pc));
      } else if (MODE == 2) {
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(p[i].x) : "v"(c));
      } else if (MODE == 3) {
        asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[i]) : "v"(pc));
      } else if (MODE == 4) {  // pk_mul with op_sel swizzle (complex-multiply style)
        asm volatile("v_pk_mul_f32 %0, %0, %1 op_sel_hi:[0,1]" : "+v"(p[i]) : "v"(pb));
      }
    }
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += a[i] + p[i].x + p[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int MODE>
float run(float* out, int blocks, int iters) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  k<MODE><<<blocks, 256>>>(out, iters);
  hipEventRecord(e0);
  k<MODE><<<blocks, 256>>>(out, iters);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); return ms;
}
int main() {
  float* out; const int blocks = 256 * 8, iters = 4096;
  if (hipMalloc(&out, blocks * 256 * 4) != hipSuccess) return 1;
  const double waves = blocks * 4.0, instr_pairs = waves * iters * 8;  // per mode: 8 "pairs" per iter
  const char* names[] = {"2x v_fma_f32", "1x v_pk_fma_f32", "2x v_add_f32", "1x v_pk_add_f32", "1x v_pk_mul_f32 opsel"};
  float t[5] = {run<0>(out, blocks, iters), run<1>(out, blocks, iters), run<2>(out, blocks, iters), run<3>(out, blocks, iters), run<4>(out, blocks, iters)};
  for (int m = 0; m < 5; ++m) {
    // cycles per pair per SIMD at 2.4 GHz: time * f * 1024 SIMDs / (pairs)
    printf("%-24s %.3f ms  %.2f cyc/pair/SIMD\n", names[m], t[m], t[m] * 1e-3 * 2.4e9 * 1024 / instr_pairs);
  }
  return 0;
}
