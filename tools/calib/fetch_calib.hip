// FETCH_SIZE / WRITE_SIZE calibration for the access widths of the VSG kernels (gfx950).
// Streams a buffer far larger than the Infinity Cache once with (a) 4-byte-per-lane coalesced
// loads (the stack kernel's sub-window loads), (b) 16-byte-per-lane loads (the guide's calibrated
// case), and (c) 4-byte float atomic adds, so that rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE per
// dispatch can be divided by the known byte counts.   hipcc --offload-arch=gfx950 -O3 -o fetch_calib
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void read4(const float* __restrict__ x, size_t n, float* __restrict__ out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += x[i];
  if (s == 12345.f) out[0] = s;  // keeps the loads
}

__global__ void read16(const float4* __restrict__ x, size_t n4, float* __restrict__ out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = x[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) out[0] = s;
}

__global__ void atomic4(float* __restrict__ y, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    atomicAdd(y + i, 1.0f);
}

int main() {
  const size_t bytes = (size_t)1 << 30;  // 1 GiB, 4x the Infinity Cache
  const size_t n = bytes / 4;
  float *x, *y, *out;
  if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&y, 256u << 20) != hipSuccess || hipMalloc(&out, 4) != hipSuccess)
    return 1;
  hipMemset(x, 0, bytes);
  hipMemset(y, 0, 256u << 20);
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL(read4, dim3(4096), dim3(256), 0, 0, x, n, out);
    hipLaunchKernelGGL(read16, dim3(4096), dim3(256), 0, 0, (const float4*)x, n / 4, out);
    hipLaunchKernelGGL(atomic4, dim3(4096), dim3(256), 0, 0, y, (size_t)(64u << 20));
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("read4 bytes %zu read16 bytes %zu atomic bytes %zu\n", bytes, bytes, (size_t)(256u << 20));
  hipFree(x);
  hipFree(y);
  hipFree(out);
  return 0;
}
