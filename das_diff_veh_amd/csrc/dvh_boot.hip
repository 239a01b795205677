// Bootstrap / convergence resampling on MI355X (gfx950): SURVEY §8(f) row 1.
//
// Replaces, for all resamples of a bootstrap run at once:
//   bootstrap_disp                 apis/imaging_classes.py:8-48 (per resample: VSG stack of
//                                  random.sample(range(1, n), bt_size) windows, compute_disp_image,
//                                  extract_ridge_ref_idx per mode)
//   extract_ridge_ref_idx          modules/utils.py:621-678
// The per-pass gathers are computed once (dvh_vsg_gathers); a resample's stack is the mean of its
// selected gathers (select_mean_kernel); the f-v images of all resamples run through the batched
// dispersion kernels (dvh_disp_*); ridge_kernel walks every (resample, mode) ridge in one wave.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "dvh_common.h"
#include "dvh.h"

namespace dvh {

// out[b][k] = (sum_{j < m} G[sel[b][j]][k]) / m over the contiguous K-element block of each pass,
// summed in selection order (the reference's sum(images) / len(images)).  float4 per lane; the loads of 8
// selections are issued before their adds (in order), so a lane keeps 8 gathers' reads in flight.
__device__ __forceinline__ void select_mean_one(const float* __restrict__ G, int64_t pass_stride, int64_t K,
                                                const int32_t* __restrict__ s, int32_t m, float* __restrict__ o,
                                                bool vec) {
  if (vec) {
    const int64_t k4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (4 * k4 >= K) return;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int j = 0;
    for (; j + 8 <= m; j += 8) {
      float4 g[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) g[u] = reinterpret_cast<const float4*>(G + (int64_t)s[j + u] * pass_stride)[k4];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        acc.x += g[u].x;
        acc.y += g[u].y;
        acc.z += g[u].z;
        acc.w += g[u].w;
      }
    }
    for (; j < m; ++j) {
      const float4 g = reinterpret_cast<const float4*>(G + (int64_t)s[j] * pass_stride)[k4];
      acc.x += g.x;
      acc.y += g.y;
      acc.z += g.z;
      acc.w += g.w;
    }
    // divide (not multiply by 1/m): sum / len as the reference evaluates it
    reinterpret_cast<float4*>(o)[k4] = make_float4(acc.x / (float)m, acc.y / (float)m, acc.z / (float)m, acc.w / (float)m);
  } else {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < K; k += (int64_t)gridDim.x * blockDim.x) {
      float acc = 0.f;
      for (int j = 0; j < m; ++j) acc += G[(int64_t)s[j] * pass_stride + k];
      o[k] = acc / (float)m;
    }
  }
}

__device__ __forceinline__ bool select_vec(const float* G, int64_t pass_stride, int64_t K, const float* out,
                                           int64_t out_stride) {
  return (K % 4 == 0) && (pass_stride % 4 == 0) && (out_stride % 4 == 0) &&
         ((reinterpret_cast<uintptr_t>(G) | reinterpret_cast<uintptr_t>(out)) % 16 == 0);
}

__global__ __launch_bounds__(256) void select_mean_kernel(const float* __restrict__ G, int64_t pass_stride, int64_t K,
                                                          const int32_t* __restrict__ sel, int32_t m,
                                                          float* __restrict__ out, int64_t out_stride) {
  const int b = blockIdx.y;
  select_mean_one(G, pass_stride, K, sel + (int64_t)b * m, m, out + (int64_t)b * out_stride, select_vec(G, pass_stride,
                  K, out, out_stride));
}

// The same for resamples of different sizes in one launch: resample b takes cnt[b] selections from sel + off[b]
// (convergence_test's bt_size = 1 .. 60 x 30 draws: one launch of 1 800 resamples instead of 60 of 30).
__global__ __launch_bounds__(256) void select_mean_var_kernel(const float* __restrict__ G, int64_t pass_stride,
                                                              int64_t K, const int32_t* __restrict__ sel,
                                                              const int32_t* __restrict__ off,
                                                              const int32_t* __restrict__ cnt, float* __restrict__ out,
                                                              int64_t out_stride) {
  const int b = blockIdx.y;
  select_mean_one(G, pass_stride, K, sel + off[b], cnt[b], out + (int64_t)b * out_stride,
                  select_vec(G, pass_stride, K, out, out_stride));
}

// np.argmax order over (value, row): a NaN beats any number, the first row wins ties
__device__ __forceinline__ bool better(float a, int ra, float b, int rb) {
  const bool na = isnan(a), nb = isnan(b);
  if (na != nb) return na;
  if (na || a == b) return ra < rb;
  return a > b;
}

__device__ __forceinline__ void wave_argmax(float& v, int& r) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(v, o);
    const int r2 = __shfl_xor(r, o);
    if (r2 >= 0 && (r < 0 || better(v2, r2, v, r))) {
      v = v2;
      r = r2;
    }
  }
}

// first row r (of nV, velocities descending) with vel[r] < x: rows [0, r) have vel >= x
__device__ __forceinline__ int first_below(const double* __restrict__ vel, int nV, double x) {
  int lo = 0, hi = nV;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (vel[mid] < x) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// first row r with vel[r] <= x
__device__ __forceinline__ int first_at_or_below(const double* __restrict__ vel, int nV, double x) {
  int lo = 0, hi = nV;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (vel[mid] <= x) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// The velocity axis of a walk held in the wave's registers (nV <= 1024: lane l holds rows l S .. l S + S - 1,
// S = ceil(nV / 64)), so that each step's two window bounds and its pick's velocity cost no memory round trip (the
// binary searches over vel[] were 2 x 10 dependent loads per step, the walk's critical path).  Same results as
// first_below / first_at_or_below / vel[r] on a descending axis; larger axes use those.
struct VelAxis {
  static constexpr int kMaxS = 16;
  const double* vel;
  int nV, S, lane;
  bool regs;
  double v[kMaxS];
  __device__ VelAxis(const double* vel_, int nV_, int lane_) : vel(vel_), nV(nV_), S((nV_ + 63) / 64), lane(lane_) {
    regs = nV <= 64 * kMaxS;
#pragma unroll
    for (int k = 0; k < kMaxS; ++k) {
      const int r = lane * S + k;
      v[k] = (regs && k < S && r < nV) ? vel[r] : 0.0;
    }
  }
  // first row whose velocity satisfies the monotone predicate (rows past nV count as satisfying it), nV if none
  template <class P>
  __device__ __forceinline__ int first(P pred) const {
    int f = S;
#pragma unroll
    for (int k = 0; k < kMaxS; ++k) {
      const int r = lane * S + k;
      if (k < S && f == S && (r >= nV || pred(v[k]))) f = k;
    }
    const uint64_t m = __ballot(f < S);
    if (m == 0) return nV;
    const int L = __ffsll((unsigned long long)m) - 1;
    return min(L * S + __shfl(f, L), nV);
  }
  __device__ __forceinline__ int below(double x) const {  // first_below
    return regs ? first([x](double u) { return u < x; }) : first_below(vel, nV, x);
  }
  __device__ __forceinline__ int at_or_below(double x) const {  // first_at_or_below
    return regs ? first([x](double u) { return u <= x; }) : first_at_or_below(vel, nV, x);
  }
  __device__ __forceinline__ double at(int r) const {  // vel[r] for a wave-uniform row r
    if (!regs) return vel[r];
    const int k = r % S;
    double u = 0.0;
#pragma unroll
    for (int j = 0; j < kMaxS; ++j) u = j == k ? v[j] : u;
    return __shfl(u, r / S);
  }
};

// argmax of column c over rows [r0, r1) (first max wins); -1 when the range is empty
__device__ __forceinline__ int column_argmax(const float* __restrict__ F, int nF, int c, int r0, int r1, int lane) {
  float best = 0.f;
  int row = -1;
  for (int r = r0 + lane; r < r1; r += 64) {
    const float v = F[(int64_t)r * nF + c];
    if (row < 0 || better(v, r, best, row)) {
      best = v;
      row = r;
    }
  }
  wave_argmax(best, row);
  return row;
}

constexpr int kMaxBand = 1024;

// One wave per (image b, ridge):  extract_ridge_ref_idx (modules/utils.py:621-678) on the band of
// columns [c0, c0 + nb) of fv[b] ([nV][nF], rows = velocities in descending order vel[r]).
//   ref == INT32_MIN:  vel_max mode (ref_freq_idx=None), raw picks over rows at/after
//             argmin |vel_max - vel| (no smoothing)
//   vref:     per-column reference velocities (ref_vel(freq)), window (vref - sigma, vref + sigma)
//   else:     pick at column ref over all rows, then walk backward / forward with the window
//             (v_prev - sigma, v_prev + sigma); -nb <= ref < 0 is a Python index with the reference's
//             loop order (below); savgol(sgl, 2, mode='interp') of the picks.
// status[b] = 0, or 1 when a window holds no velocity (np.argmax of an empty slice raises).
__global__ __launch_bounds__(64) void ridge_kernel(const float* __restrict__ fv, int64_t b_stride, int32_t nV,
                                                   int32_t nF, int32_t c0, int32_t nb, const double* __restrict__ vel,
                                                   int32_t ref, double sigma, double vel_max,
                                                   const double* __restrict__ vref, const double* __restrict__ sg,
                                                   int32_t sgl, double* __restrict__ out, int32_t* __restrict__ status,
                                                   double* __restrict__ picks) {
  __shared__ double pick[kMaxBand];
  const int b = blockIdx.x, lane = threadIdx.x;
  const float* F = fv + (int64_t)b * b_stride;
  double* o = out + (int64_t)b * nb;
  int err = 0;
  if (ref == INT32_MIN) {
    // max_idx = argmin |vel_max - vel| (first of equal distances)
    double bd = INFINITY;
    int bi = nV;
    for (int r = lane; r < nV; r += 64) {
      const double d = fabs(vel_max - vel[r]);
      if (d < bd || (d == bd && r < bi)) {
        bd = d;
        bi = r;
      }
    }
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) {
      const double d2 = __shfl_xor(bd, s);
      const int i2 = __shfl_xor(bi, s);
      if (d2 < bd || (d2 == bd && i2 < bi)) {
        bd = d2;
        bi = i2;
      }
    }
    for (int i = 0; i < nb; ++i) {
      const int r = column_argmax(F, nF, c0 + i, bi, nV, lane);
      if (lane == 0) o[i] = r >= 0 ? vel[r] : NAN;
      err |= r < 0;
    }
    if (lane == 0) status[b] = err;
    return;
  }
  const VelAxis ax(vel, nV, lane);
  // the walk over columns i_begin, i_begin + dir, ... (i_end excluded) from the pick velocity v; returns the last pick
  auto walk = [&](int i_begin, int i_end, int dir, double v) {
    for (int i = i_begin; i != i_end; i += dir) {
      const int r0 = ax.below(v + sigma), r1 = ax.at_or_below(v - sigma);
      const int r = column_argmax(F, nF, c0 + i, r0, r1, lane);
      err |= r < 0;
      v = r >= 0 ? ax.at(r) : NAN;  // (r is wave-uniform: every lane takes part in the shuffle)
      if (lane == 0) pick[i] = v;
    }
    return v;
  };
  if (vref) {
    for (int i = 0; i < nb; ++i) {
      const int r0 = ax.below(vref[i] + sigma), r1 = ax.at_or_below(vref[i] - sigma);
      const int r = column_argmax(F, nF, c0 + i, r0, r1, lane);
      err |= r < 0;
      const double pv = r >= 0 ? ax.at(r) : NAN;
      if (lane == 0) pick[i] = pv;
    }
  } else if (ref < 0) {
    // a negative reference index is a Python index: out[ref] is column nb + ref, the backward loop
    // range(ref - 1, -1, -1) is empty, and range(ref + 1, len(freq)) walks columns nb + ref + 1 ..
    // nb - 1 and then 0 .. nb - 1 again, seeded by out[-1] (modules/utils.py:662-671)
    const int k0 = nb + ref;
    const int rr = column_argmax(F, nF, c0 + k0, 0, nV, lane);
    const double v = rr >= 0 ? ax.at(rr) : NAN;
    if (lane == 0) pick[k0] = v;
    walk(0, nb, 1, walk(k0 + 1, nb, 1, v));
  } else {
    const int rr = column_argmax(F, nF, c0 + ref, 0, nV, lane);
    const double vr = rr >= 0 ? ax.at(rr) : NAN;  // wave-uniform (every lane holds the reduced row)
    if (lane == 0) pick[ref] = vr;
    walk(ref - 1, -1, -1, vr);  // backward
    walk(ref + 1, nb, 1, vr);   // forward
  }
  __syncthreads();
  if (picks)  // the raw picks before smoothing (parity checks of each pick)
    for (int i = lane; i < nb; i += 64) picks[(int64_t)b * nb + i] = pick[i];
  // savgol_filter(picks, sgl, 2) with mode='interp': interior taps h, edge fits el / er
  const int half = sgl / 2;
  const double* h = sg;
  const double* el = sg + sgl;
  const double* er = el + half * sgl;
  for (int i = lane; i < nb; i += 64) {
    double acc = 0.0;
    if (i < half) {
      for (int t = 0; t < sgl; ++t) acc += el[i * sgl + t] * pick[t];
    } else if (i >= nb - half) {
      for (int t = 0; t < sgl; ++t) acc += er[(i - (nb - half)) * sgl + t] * pick[nb - sgl + t];
    } else {
      for (int t = 0; t < sgl; ++t) acc += h[t] * pick[i - half + t];
    }
    o[i] = acc;
  }
  if (lane == 0) status[b] = err;
}

static int last_launch() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_error(-3, hipGetErrorString(e));
}

}  // namespace dvh

using namespace dvh;

DVH_API int dvh_select_mean(const float* G, int64_t pass_stride, int64_t K, const int32_t* sel, int32_t B, int32_t m,
                            float* out, int64_t out_stride, void* stream) {
  if (!G || !sel || !out) return set_error(-2, "null pointer argument");
  if (m <= 0 || K < 0 || B < 0) return set_error(-2, "invalid sizes");
  if (B == 0 || K == 0) return 0;
  if (B > 65535) return set_error(-4, "too many resamples for one launch");
  const int64_t blocks = (K / 4 + 255) / 256 + 1;
  hipLaunchKernelGGL(select_mean_kernel, dim3((unsigned)blocks, B), dim3(256), 0, (hipStream_t)stream, G, pass_stride,
                     K, sel, m, out, out_stride);
  return last_launch();
}

DVH_API int dvh_select_mean_var(const float* G, int64_t pass_stride, int64_t K, const int32_t* sel, const int32_t* off,
                                const int32_t* cnt, int32_t B, float* out, int64_t out_stride, void* stream) {
  if (!G || !sel || !off || !cnt || !out) return set_error(-2, "null pointer argument");
  if (K < 0 || B < 0) return set_error(-2, "invalid sizes");
  if (B == 0 || K == 0) return 0;
  if (B > 65535) return set_error(-4, "too many resamples for one launch");
  const int64_t blocks = (K / 4 + 255) / 256 + 1;
  hipLaunchKernelGGL(select_mean_var_kernel, dim3((unsigned)blocks, B), dim3(256), 0, (hipStream_t)stream, G,
                     pass_stride, K, sel, off, cnt, out, out_stride);
  return last_launch();
}

DVH_API int dvh_ridge(const float* fv, int64_t b_stride, int32_t B, int32_t nV, int32_t nF, int32_t c0, int32_t nb,
                      const double* vel, int32_t ref, double sigma, double vel_max, const double* vref,
                      const double* sg, int32_t sgl, double* out, int32_t* status, double* picks, void* stream) {
  if (!fv || !vel || !out || !status) return set_error(-2, "null pointer argument");
  if (nb <= 0 || c0 < 0 || c0 + nb > nF || nV <= 0) return set_error(-2, "invalid band");
  if (nb > kMaxBand) return set_error(-4, "band longer than 1024 frequencies");
  if (ref != INT32_MIN || vref) {
    if (!sg || sgl % 2 == 0 || sgl > nb) return set_error(-4, "savgol window must be odd and <= the band length");
    if (ref >= nb || ref < -nb) return set_error(-2, "reference index outside the band");
  }
  if (B <= 0) return 0;
  hipLaunchKernelGGL(ridge_kernel, dim3(B), dim3(64), 0, (hipStream_t)stream, fv, b_stride, nV, nF, c0, nb, vel,
                     ref, sigma, vel_max, vref, sg, sgl, out, status, picks);
  return last_launch();
}
