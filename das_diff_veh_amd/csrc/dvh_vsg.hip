// Virtual-shot-gather cross-correlation + class stacking on MI355X (gfx950).
//
// Replaces, for a whole batch of vehicle passes at once:
//   XCORR_vshot                      modules/utils.py:289-314
//   XCORR_two_traces / repeat1d      modules/utils.py:250-270
//   xcorr_two_traces_based_on_traj   apis/virtual_shot_gather.py:14-43
//   post_processing_XCF              apis/virtual_shot_gather.py:129-142
//   construct_shot_gather[_other_side] + the two-sided average   apis/virtual_shot_gather.py:145-192
//   sum(images) / len(images)        apis/imaging_classes.py:106-107 (VirtualShotGather.__add__/__truediv__)
//
// Work unit: one (pass, gather row).  One wave64 computes BOTH sides of the row:
//   for each side, for each of the nwin sub-windows of its time slice, z = pivot + i*receiver is
//   transformed by one complex FFT (LDS Stockham), the cross spectrum P*conj(R) is extracted from
//   Z[f], conj(Z[-f]) and accumulated in registers; then ONE inverse FFT of Cf + i*Co yields both
//   sides' correlations (real and imaginary parts).  The epilogue applies each row type's lag
//   permutation (roll(w//2), time flip on the forward side), the per-pass amplitude normalisation
//   (1 / max of the pivot autocorrelation, from vsg_scales_kernel), the optional row L2 norm, and
//   the two-sided average rule (rows whose other side is finite and non-zero).
// Lag conventions, with c[k] = sum_n p[(n+k) % w] r[n] and h = w // 2:
//   forward, channel <= pivot (shared pivot window):   F[j] = c[(w-1-j-h) mod w]
//   forward, channel >  pivot (trajectory window):     F[j] = c[(j+h+1) mod w]
//   other,   channel >= pivot (shared, reverse=True):  O[j] = c[(h-1-j) mod w]
//   other,   channel <  pivot (trajectory window):     O[j] = c[(j-h) mod w]
//
// Windows are fp32, channel-major: sample (pass p, channel c, time t) at
//   win[p * pass_stride + c * ch_stride + t].
// seg_tab[((p * R + i) * 2 + side) * 2 + {0,1}] = {slice start, slice length} for gather row i
// (channel row0[p] + i) on side 0 = forward, 1 = other; pass_tab[p * 2 + {0,1}] = {row0, pivot}.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "fft_wave.h"
#include "dvh_common.h"
#include "dvh.h"

namespace dvh {

constexpr int kWaves = 4;
constexpr int kBlock = 64 * kWaves;

enum : int32_t {
  kFlagOtherSide = 1,
  kFlagNorm = 2,
  kFlagNormAmp = 4,
};

struct VsgArgs {
  const float* win;
  int64_t pass_stride;
  int64_t ch_stride;
  const int32_t* pass_tab;
  const int32_t* seg_tab;
  int32_t n_pass;
  int32_t R;
  int32_t w;
  int32_t hop;
  int32_t flags;
};

__device__ __forceinline__ int pmod(int a, int m) {
  const int r = a % m;
  return r < 0 ? r + m : r;
}

__device__ __forceinline__ int n_subwin(int L, int w, int hop) { return (L >= w) ? (L - w) / hop + 1 : 0; }

// Wave-uniform value (keeps table indices and table entries in SGPRs -> scalar loads).
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Global -> register staging of one sub-window z = pivot + i * receiver (lane owns n = lane + 64 j).
template <int N>
__device__ __forceinline__ void load_subwin(const float* __restrict__ piv, const float* __restrict__ rcv, int a,
                                            int w, int lane, float2 (&z)[(N + 63) / 64]) {
  constexpr int NJ = (N + 63) / 64;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = lane + 64 * j;
    z[j] = (n < w) ? make_float2(piv[a + n], rcv[a + n]) : make_float2(0.f, 0.f);
  }
}

// Both sides of one gather row -> raw correlations in LDS: Y[k].x = N * sum_s c_f, -Y[k].y = N * sum_s c_o.
// The sub-windows of both sides form one sequence q = 0 .. nwf + nwo - 1; the global loads of
// sub-window q + 1 are issued before the FFT of sub-window q so their latency hides under it.
template <int N>
__device__ __forceinline__ const float2* row_correlations(const VsgArgs& A, int p, int i, bool other,
                                                          float2* bufA, float2* bufB, const float2* tw,
                                                          int lane, int& nwin_f, int& nwin_o, int& ch,
                                                          int& pivot) {
  constexpr int NJ = (N + 63) / 64;
  p = uni(p);
  i = uni(i);
  const int row0 = uni(A.pass_tab[2 * p]);
  pivot = uni(A.pass_tab[2 * p + 1]);
  ch = row0 + i;
  const float* base = A.win + (int64_t)p * A.pass_stride;
  const float* piv = base + (int64_t)pivot * A.ch_stride;
  const float* rcv = base + (int64_t)ch * A.ch_stride;
  const int32_t* seg = A.seg_tab + ((int64_t)p * A.R + i) * 4;
  const int w = A.w, hop = A.hop;
  const int a_f = uni(seg[0]), a_o = uni(seg[2]);
  nwin_f = n_subwin(uni(seg[1]), w, hop);
  nwin_o = other ? n_subwin(uni(seg[3]), w, hop) : 0;
  const int nq = nwin_f + nwin_o;
  float2 Cf[NJ], Co[NJ], z[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    Cf[j] = make_float2(0.f, 0.f);
    Co[j] = make_float2(0.f, 0.f);
  }
  if (nq > 0) load_subwin<N>(piv, rcv, nwin_f > 0 ? a_f : a_o, w, lane, z);
  for (int q = 0; q < nq; ++q) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = lane + 64 * j;
      if (n < N) bufA[n] = z[j];
    }
    if (q + 1 < nq) {
      const int qn = q + 1;
      const int an = qn < nwin_f ? a_f + qn * hop : a_o + (qn - nwin_f) * hop;
      load_subwin<N>(piv, rcv, an, w, lane, z);
    }
    wave_sync();
    const float2* X = FftPlan<N>::T::run(bufA, bufB, tw, lane);
    const bool fwd = q < nwin_f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int f = lane + 64 * j;
      if (f < N) {
        const float2 Az = X[f];
        const float2 Bc = X[f == 0 ? 0 : N - f];  // B = conj(Bc)
        const float bx = Bc.x, by = -Bc.y;
        // P = (A + B) / 2, R = (A - B) / 2i  ->  P conj(R) = (i / 4) (A + B) conj(A - B)
        const float cx = 0.5f * (bx * Az.y - by * Az.x);
        const float cy = 0.25f * ((Az.x * Az.x + Az.y * Az.y) - (bx * bx + by * by));
        if (fwd) {
          Cf[j].x += cx;
          Cf[j].y += cy;
        } else {
          Co[j].x += cx;
          Co[j].y += cy;
        }
      }
    }
    wave_sync();
  }
  // inverse FFT of W = Cf + i Co via conj(FFT(conj(W)))
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int f = lane + 64 * j;
    if (f < N) bufA[f] = make_float2(Cf[j].x - Co[j].y, -(Cf[j].y + Co[j].x));
  }
  wave_sync();
  return FftPlan<N>::T::run(bufA, bufB, tw, lane);
}

// c[k] (scaled by N * nwin) for the side held in component `comp` (0 -> fwd (+x), 1 -> other (-y)).
template <int N, bool PAD>
__device__ __forceinline__ float2 read_c(const float2* Y, int k, int w) {
  float2 v = Y[k];
  if (PAD && k > 0) {
    const float2 u = Y[N - w + k];
    v.x += u.x;
    v.y += u.y;
  }
  return make_float2(v.x, -v.y);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// Per-pass scale of each side: 1 / max(pivot autocorrelation row) after the optional row norm
// (post_processing_XCF with norm_amp=True); 1 / ||window||_F^2 when neither norm is requested.
template <int N, bool PAD>
__global__ __launch_bounds__(kBlock) void vsg_scales_kernel(VsgArgs A, const double* __restrict__ sumsq,
                                                             float* __restrict__ scales) {
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  float2* tw = smem;
  init_twiddles<N>(tw);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  float2* bufA = smem + N + wave * 2 * N;
  float2* bufB = bufA + N;
  const bool other = (A.flags & kFlagOtherSide) != 0;
  const bool norm = (A.flags & kFlagNorm) != 0;
  const bool norm_amp = (A.flags & kFlagNormAmp) != 0;
  constexpr int NJ = (N + 63) / 64;
  for (int p = blockIdx.x * kWaves + wave; p < A.n_pass; p += gridDim.x * kWaves) {
    if (!norm_amp) {
      if (lane == 0) {
        const float s = norm ? 1.0f : (float)(1.0 / sumsq[p]);
        scales[2 * p] = s;
        scales[2 * p + 1] = s;
      }
      continue;
    }
    const int i = A.pass_tab[2 * p + 1] - A.pass_tab[2 * p];  // pivot row of the gather
    int nwf, nwo, ch, pivot;
    const float2* Y = row_correlations<N>(A, p, i, other, bufA, bufB, tw, lane, nwf, nwo, ch, pivot);
    float mf = -INFINITY, mo = -INFINITY, sf = 0.f, so = 0.f;
    bool nanf = false, nano = false;
    // a side with no sub-window is exactly zero in the reference (the packed inverse FFT would
    // otherwise leak the other side's rounding into it)
    const float2 live = make_float2(nwf > 0 ? 1.f : 0.f, nwo > 0 ? 1.f : 0.f);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int k = lane + 64 * j;
      if (k < A.w) {
        float2 c = read_c<N, PAD>(Y, k, A.w);
        c.x *= live.x;
        c.y *= live.y;
        nanf |= isnan(c.x);
        nano |= isnan(c.y);
        mf = fmaxf(mf, c.x);
        mo = fmaxf(mo, c.y);
        sf += c.x * c.x;
        so += c.y * c.y;
      }
    }
    wave_sync();
    mf = wave_max(mf);
    mo = wave_max(mo);
    const bool anynanf = __ballot(nanf) != 0, anynano = __ballot(nano) != 0;
    float amax_f, amax_o;
    if (norm) {
      sf = wave_sum(sf);
      so = wave_sum(so);
      amax_f = mf / sqrtf(sf);
      amax_o = mo / sqrtf(so);
    } else {
      amax_f = nwf > 0 ? mf / ((float)N * (float)nwf) : 0.f;
      amax_o = nwo > 0 ? mo / ((float)N * (float)nwo) : 0.f;
    }
    if (anynanf) amax_f = NAN;
    if (anynano) amax_o = NAN;
    if (lane == 0) {
      scales[2 * p] = 1.0f / amax_f;
      scales[2 * p + 1] = other ? 1.0f / amax_o : 0.f;
    }
  }
}

// Final gather row for (pass p, row i): G[m] for j = lane + 64 m.
template <int N, bool PAD>
__device__ __forceinline__ void gather_row(const VsgArgs& A, const float* __restrict__ scales, int p, int i,
                                           float2* bufA, float2* bufB, const float2* tw, int lane,
                                           float (&G)[(N + 63) / 64]) {
  constexpr int NJ = (N + 63) / 64;
  const bool other = (A.flags & kFlagOtherSide) != 0;
  const bool norm = (A.flags & kFlagNorm) != 0;
  int nwf, nwo, ch, pivot;
  const float2* Y = row_correlations<N>(A, p, i, other, bufA, bufB, tw, lane, nwf, nwo, ch, pivot);
  const int w = A.w, h = w / 2;
  // a side with no sub-window is exactly zero in the reference (see vsg_scales_kernel)
  const float2 live = make_float2(nwf > 0 ? 1.f : 0.f, nwo > 0 ? 1.f : 0.f);
  float ff, fo;
  if (norm) {
    float sf = 0.f, so = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int k = lane + 64 * j;
      if (k < w) {
        float2 c = read_c<N, PAD>(Y, k, w);
        c.x *= live.x;
        c.y *= live.y;
        sf += c.x * c.x;
        so += c.y * c.y;
      }
    }
    ff = 1.0f / sqrtf(wave_sum(sf));
    fo = 1.0f / sqrtf(wave_sum(so));
  } else {
    ff = nwf > 0 ? 1.0f / ((float)N * (float)nwf) : 0.f;
    fo = nwo > 0 ? 1.0f / ((float)N * (float)nwo) : 0.f;
  }
  ff *= __builtin_bit_cast(float, uni(__builtin_bit_cast(int, scales[2 * p])));
  fo *= __builtin_bit_cast(float, uni(__builtin_bit_cast(int, scales[2 * p + 1])));
  const bool fwd_shared = ch <= pivot;
  const bool oth_shared = ch >= pivot;
  float O[NJ];
  bool nan_o = false, nz_o = false;
#pragma unroll
  for (int m = 0; m < NJ; ++m) {
    const int j = lane + 64 * m;
    G[m] = 0.f;
    O[m] = 0.f;
    if (j < w) {
      const int kf = fwd_shared ? pmod(w - 1 - j - h, w) : pmod(j + h + 1, w);
      G[m] = (read_c<N, PAD>(Y, kf, w).x * live.x) * ff;
      if (other) {
        const int ko = oth_shared ? pmod(h - 1 - j, w) : pmod(j - h, w);
        O[m] = (read_c<N, PAD>(Y, ko, w).y * live.y) * fo;
        nan_o |= isnan(O[m]);
        nz_o |= (O[m] != 0.f);
      }
    }
  }
  wave_sync();
  if (other) {
    // ||other row|| > 0 in the reference: finite-or-inf, not NaN, and not identically zero
    const bool ok = (__ballot(nan_o) == 0) && (__ballot(nz_o) != 0);
    if (ok) {
#pragma unroll
      for (int m = 0; m < NJ; ++m) G[m] = (G[m] + O[m]) * 0.5f;
    }
  }
}

template <int N, bool PAD>
__global__ __launch_bounds__(kBlock) void vsg_gather_kernel(VsgArgs A, const float* __restrict__ scales,
                                                             float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  float2* tw = smem;
  init_twiddles<N>(tw);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  float2* bufA = smem + N + wave * 2 * N;
  float2* bufB = bufA + N;
  constexpr int NJ = (N + 63) / 64;
  const int64_t n_task = (int64_t)A.n_pass * A.R;
  for (int64_t t = (int64_t)blockIdx.x * kWaves + wave; t < n_task; t += (int64_t)gridDim.x * kWaves) {
    const int p = (int)(t / A.R), i = (int)(t % A.R);
    float G[NJ];
    gather_row<N, PAD>(A, scales, p, i, bufA, bufB, tw, lane, G);
    float* o = out + t * A.w;
#pragma unroll
    for (int m = 0; m < NJ; ++m) {
      const int j = lane + 64 * m;
      if (j < A.w) o[j] = G[m];
    }
  }
}

// Stack mode: task = (chunk c, row i); the wave walks the chunk's passes (all of one class slot),
// sums weight[p] * G_p in registers and adds the row into stack[slot] once.
template <int N, bool PAD>
__global__ __launch_bounds__(kBlock) void vsg_stack_kernel(VsgArgs A, const float* __restrict__ scales,
                                                            const int32_t* __restrict__ order,
                                                            const int32_t* __restrict__ chunk_tab, int32_t n_chunk,
                                                            const float* __restrict__ weight,
                                                            float* __restrict__ stack) {
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  float2* tw = smem;
  init_twiddles<N>(tw);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  float2* bufA = smem + N + wave * 2 * N;
  float2* bufB = bufA + N;
  constexpr int NJ = (N + 63) / 64;
  const int64_t n_task = (int64_t)n_chunk * A.R;
  for (int64_t t = (int64_t)blockIdx.x * kWaves + wave; t < n_task; t += (int64_t)gridDim.x * kWaves) {
    const int c = uni((int)(t / A.R)), i = uni((int)(t % A.R));
    const int b = uni(chunk_tab[3 * c]), e = uni(chunk_tab[3 * c + 1]), slot = uni(chunk_tab[3 * c + 2]);
    float acc[NJ];
#pragma unroll
    for (int m = 0; m < NJ; ++m) acc[m] = 0.f;
    for (int q = b; q < e; ++q) {
      const int p = uni(order[q]);
      float G[NJ];
      gather_row<N, PAD>(A, scales, p, i, bufA, bufB, tw, lane, G);
      const float wp = __builtin_bit_cast(float, uni(__builtin_bit_cast(int, weight[p])));
#pragma unroll
      for (int m = 0; m < NJ; ++m) acc[m] += G[m] * wp;
    }
    float* o = stack + ((int64_t)slot * A.R + i) * A.w;
#pragma unroll
    for (int m = 0; m < NJ; ++m) {
      const int j = lane + 64 * m;
      if (j < A.w) atomicAdd(o + j, acc[m]);
    }
  }
}

// Sum of squares of each pass window (np.linalg.norm(window.data) ** 2), for norm=norm_amp=False.
__global__ __launch_bounds__(kBlock) void window_sumsq_kernel(const float* __restrict__ win, int64_t pass_stride,
                                                               int64_t ch_stride, int32_t n_ch, int32_t n_t,
                                                               double* __restrict__ out) {
  __shared__ double part[kWaves];
  const int p = blockIdx.x;
  const float* base = win + (int64_t)p * pass_stride;
  double s = 0.0;
  for (int c = 0; c < n_ch; ++c) {
    const float* row = base + (int64_t)c * ch_stride;
    for (int t = threadIdx.x; t < n_t; t += blockDim.x) {
      const double v = row[t];
      s += v * v;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < kWaves; ++k) t += part[k];
    out[p] = t;
  }
}

template <int N>
constexpr size_t vsg_lds_bytes() {
  return sizeof(float2) * (size_t)N * (1 + 2 * kWaves);
}

struct VsgKernels {
  const void* scales;
  const void* gather;
  const void* stack;
  size_t lds;
};

template <int N, bool PAD>
VsgKernels vsg_kernels() {
  return VsgKernels{(const void*)vsg_scales_kernel<N, PAD>, (const void*)vsg_gather_kernel<N, PAD>,
                    (const void*)vsg_stack_kernel<N, PAD>, vsg_lds_bytes<N>()};
}

// Transform length for a window length w: exact mixed-radix when available, else a zero-padded
// power of two >= 2w - 1 (linear correlation folded back to circular).  Returns 0 if unsupported.
static int choose_fft(int w, bool* pad) {
  *pad = false;
  if (w == 250 || w == 500 || w == 1000) return w;
  *pad = true;
  if (2 * w - 1 <= 512) return 512;
  if (2 * w - 1 <= 1024) return 1024;
  if (2 * w - 1 <= 2048) return 2048;
  return 0;
}

static bool get_kernels(int w, VsgKernels* k, int* n_out) {
  bool pad;
  const int n = choose_fft(w, &pad);
  *n_out = n;
  switch (n) {
    case 250: *k = vsg_kernels<250, false>(); return true;
    case 500: *k = vsg_kernels<500, false>(); return true;
    case 1000: *k = vsg_kernels<1000, false>(); return true;
    case 512: *k = vsg_kernels<512, true>(); return true;
    case 1024: *k = vsg_kernels<1024, true>(); return true;
    case 2048: *k = vsg_kernels<2048, true>(); return true;
    default: return false;
  }
}

static int check_common(const VsgArgs& A) {
  if (!A.win || !A.pass_tab || !A.seg_tab) return set_error(-2, "null pointer argument");
  if (A.n_pass < 0 || A.R <= 0 || A.w < 2 || A.hop < 1) return set_error(-2, "invalid geometry (R, w, hop)");
  return 0;
}

static int launch(const void* fn, int grid, size_t lds, void** args, hipStream_t s) {
  if (grid <= 0) return 0;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return set_error(-3, hipGetErrorString(e));
  e = hipLaunchKernel(fn, dim3(grid), dim3(kBlock), args, lds, s);
  if (e != hipSuccess) return set_error(-3, hipGetErrorString(e));
  return 0;
}

}  // namespace dvh

using namespace dvh;

DVH_API int dvh_vsg_fft_length(int32_t w) {
  bool pad;
  return choose_fft(w, &pad);
}

DVH_API int dvh_window_sumsq(const float* win, int64_t pass_stride, int64_t ch_stride, int32_t n_pass, int32_t n_ch,
                             int32_t n_t, double* out, void* stream) {
  if (!win || !out) return set_error(-2, "null pointer argument");
  if (n_pass <= 0) return 0;
  hipLaunchKernelGGL(window_sumsq_kernel, dim3(n_pass), dim3(kBlock), 0, (hipStream_t)stream, win, pass_stride,
                     ch_stride, n_ch, n_t, out);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_error(-3, hipGetErrorString(e));
}

DVH_API int dvh_vsg_scales(const float* win, int64_t pass_stride, int64_t ch_stride, int32_t n_pass,
                           const int32_t* pass_tab, const int32_t* seg_tab, int32_t R, int32_t w, int32_t hop,
                           int32_t flags, const double* win_sumsq, float* scales, void* stream) {
  VsgArgs A{win, pass_stride, ch_stride, pass_tab, seg_tab, n_pass, R, w, hop, flags};
  if (int rc = check_common(A)) return rc;
  if (!scales) return set_error(-2, "null scales");
  if (!(flags & kFlagNormAmp) && !(flags & kFlagNorm) && !win_sumsq)
    return set_error(-2, "win_sumsq required when norm and norm_amp are both off");
  VsgKernels k;
  int n;
  if (!get_kernels(w, &k, &n)) return set_error(-4, "unsupported correlation window length");
  void* args[] = {&A, &win_sumsq, &scales};
  return launch(k.scales, (n_pass + kWaves - 1) / kWaves, k.lds, args, (hipStream_t)stream);
}

DVH_API int dvh_vsg_gathers(const float* win, int64_t pass_stride, int64_t ch_stride, int32_t n_pass,
                            const int32_t* pass_tab, const int32_t* seg_tab, int32_t R, int32_t w, int32_t hop,
                            int32_t flags, const float* scales, float* out, void* stream) {
  VsgArgs A{win, pass_stride, ch_stride, pass_tab, seg_tab, n_pass, R, w, hop, flags};
  if (int rc = check_common(A)) return rc;
  if (!scales || !out) return set_error(-2, "null pointer argument");
  VsgKernels k;
  int n;
  if (!get_kernels(w, &k, &n)) return set_error(-4, "unsupported correlation window length");
  const int64_t tasks = (int64_t)n_pass * R;
  const int64_t grid = (tasks + kWaves - 1) / kWaves;
  void* args[] = {&A, &scales, &out};
  return launch(k.gather, (int)(grid > (1 << 30) ? (1 << 30) : grid), k.lds, args, (hipStream_t)stream);
}

DVH_API int dvh_vsg_stack(const float* win, int64_t pass_stride, int64_t ch_stride, int32_t n_pass,
                          const int32_t* pass_tab, const int32_t* seg_tab, int32_t R, int32_t w, int32_t hop,
                          int32_t flags, const float* scales, const int32_t* order, const int32_t* chunk_tab,
                          int32_t n_chunk, const float* weight, float* stack, void* stream) {
  VsgArgs A{win, pass_stride, ch_stride, pass_tab, seg_tab, n_pass, R, w, hop, flags};
  if (int rc = check_common(A)) return rc;
  if (!scales || !order || !chunk_tab || !weight || !stack) return set_error(-2, "null pointer argument");
  VsgKernels k;
  int n;
  if (!get_kernels(w, &k, &n)) return set_error(-4, "unsupported correlation window length");
  const int64_t tasks = (int64_t)n_chunk * R;
  const int64_t grid = (tasks + kWaves - 1) / kWaves;
  void* args[] = {&A, &scales, &order, &chunk_tab, &n_chunk, &weight, &stack};
  return launch(k.stack, (int)(grid > (1 << 30) ? (1 << 30) : grid), k.lds, args, (hipStream_t)stream);
}
