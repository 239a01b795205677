// Per-pass windowing, taper and bandpass on MI355X (gfx950).
//
//   dvh_sosfiltfilt  bandpass_data (modules/utils.py:179-189): scipy.signal.sosfiltfilt(sos, x, axis=1)
//                    = odd extension by padlen, sosfilt with zi * x_ext[0], reverse, sosfilt with
//                    zi * y[-1], reverse, trim.  One lane per trace, float64 recursion (the order-10
//                    band edge at 1.2 Hz / 125 Hz puts poles within 1e-2 of the unit circle).
//   dvh_mute_traj    SurfaceWaveWindow.mute_along_traj (apis/data_classes.py:49-72): column t is
//                    multiplied by a tukey taper placed along the vehicle trajectory (host tables).
//   dvh_mute_time    SurfaceWaveWindow.mute_along_time (apis/data_classes.py:100-104).
//   dvh_trace_cleanup  the rest of TimeLapseImaging._preprocessing_for_surface_waves
//                    (apis/timeLapseImaging.py:51-71) after the bandpass: find_noise_idx /
//                    impute_noisy_trace (modules/utils.py:316-329) for empty traces (L2 norm below
//                    the threshold) then noisy traces (max above it), then the per-trace L2 norm.
// Data may be float32 (dtype 0) or float64 (dtype 1), modified in place.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dvh_common.h"
#include "dvh.h"

namespace dvh {

constexpr int kMaxSec = 16;

template <typename T>
__global__ __launch_bounds__(64) void sosfiltfilt_kernel(T* __restrict__ x, int64_t n_rows, int64_t row_stride,
                                                          int32_t n_t, const double* __restrict__ sos,
                                                          int32_t n_sec, int32_t padlen,
                                                          const double* __restrict__ zi,
                                                          double* __restrict__ work) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  T* row = x + r * row_stride;
  const int64_t n_ext = (int64_t)n_t + 2 * padlen;
  double* y = work + r * n_ext;
  double b0[kMaxSec], b1[kMaxSec], b2[kMaxSec], a1[kMaxSec], a2[kMaxSec], z0[kMaxSec], z1[kMaxSec];
  for (int s = 0; s < n_sec; ++s) {
    b0[s] = sos[6 * s];
    b1[s] = sos[6 * s + 1];
    b2[s] = sos[6 * s + 2];
    a1[s] = sos[6 * s + 4];
    a2[s] = sos[6 * s + 5];
  }
  const double x0 = (double)row[0], xn = (double)row[n_t - 1];
  // ext[i]: i < padlen -> 2 x0 - x[padlen - i]; i >= padlen + n_t -> 2 xn - x[n_t - 2 - (i - padlen - n_t)]
  auto ext = [&](int64_t i) -> double {
    if (i < padlen) return 2.0 * x0 - (double)row[padlen - i];
    const int64_t j = i - padlen;
    if (j < n_t) return (double)row[j];
    return 2.0 * xn - (double)row[n_t - 2 - (j - n_t)];
  };
  const double e0 = ext(0);
  for (int s = 0; s < n_sec; ++s) {
    z0[s] = zi[2 * s] * e0;
    z1[s] = zi[2 * s + 1] * e0;
  }
  for (int64_t i = 0; i < n_ext; ++i) {
    double v = ext(i);
    for (int s = 0; s < n_sec; ++s) {
      const double o = b0[s] * v + z0[s];
      z0[s] = b1[s] * v - a1[s] * o + z1[s];
      z1[s] = b2[s] * v - a2[s] * o;
      v = o;
    }
    y[i] = v;
  }
  const double yl = y[n_ext - 1];
  for (int s = 0; s < n_sec; ++s) {
    z0[s] = zi[2 * s] * yl;
    z1[s] = zi[2 * s + 1] * yl;
  }
  for (int64_t i = n_ext - 1; i >= 0; --i) {
    double v = y[i];
    for (int s = 0; s < n_sec; ++s) {
      const double o = b0[s] * v + z0[s];
      z0[s] = b1[s] * v - a1[s] * o + z1[s];
      z1[s] = b2[s] * v - a2[s] * o;
      v = o;
    }
    y[i] = v;
  }
  for (int32_t t = 0; t < n_t; ++t) row[t] = (T)y[padlen + t];
}

// tab[(p * n_t + t) * 3 + {0,1,2}] = {start, end, taper_start}; element (x, t) of pass p is scaled by
// taper[taper_start + x - start] for start <= x < end and zeroed elsewhere.
template <typename T>
__global__ __launch_bounds__(256) void mute_traj_kernel(T* __restrict__ data, int64_t pass_stride, int32_t n_ch,
                                                         int32_t n_t, const int32_t* __restrict__ tab,
                                                         const double* __restrict__ taper) {
  const int p = blockIdx.z;
  const int x = blockIdx.y;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_t) return;
  const int32_t* e = tab + ((int64_t)p * n_t + t) * 3;
  T* v = data + (int64_t)p * pass_stride + (int64_t)x * n_t + t;
  const int s = e[0], end = e[1];
  if (x >= s && x < end) {
    *v = (T)((double)*v * taper[e[2] + x - s]);
  } else {
    *v = (T)((double)*v * 0.0);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void mute_time_kernel(T* __restrict__ data, int64_t n_rows, int32_t n_t,
                                                         const double* __restrict__ taper) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_rows * n_t) return;
  data[i] = (T)((double)data[i] * taper[i % n_t]);
}

static int last_launch() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_error(-3, hipGetErrorString(e));
}

// ---------------------------------------------------------------------------------------------
// Trace clean-up of the continuous record (bandpassed, [n_rows][n_t] with row_stride).

constexpr int kStatBlock = 256;

// NaN-propagating max (np.max returns NaN for a row holding one)
__device__ __forceinline__ double nan_max(double a, double b) { return (isnan(a) || a > b) ? a : b; }

template <typename T>
__device__ __forceinline__ void block_row_stats(const T* __restrict__ row, int32_t n_t, double* __restrict__ out2) {
  __shared__ double ss[kStatBlock / 64], mx[kStatBlock / 64];
  double s = 0.0, m = -INFINITY;
  for (int t = threadIdx.x; t < n_t; t += blockDim.x) {
    const double v = (double)row[t];
    s += v * v;
    m = nan_max(m, v);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    m = nan_max(m, __shfl_xor(m, o));
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    ss[w] = s;
    mx[w] = m;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = -INFINITY;
    for (int k = 0; k < kStatBlock / 64; ++k) {
      a += ss[k];
      b = nan_max(b, mx[k]);
    }
    out2[0] = a;  // sum of squares
    out2[1] = b;  // max
  }
  __syncthreads();
}

// stats[r] = {sum x^2, max x} per trace
template <typename T>
__global__ __launch_bounds__(kStatBlock) void row_stats_kernel(const T* __restrict__ x, int64_t row_stride,
                                                                int32_t n_t, double* __restrict__ stats) {
  block_row_stats(x + (int64_t)blockIdx.x * row_stride, n_t, stats + 2 * (int64_t)blockIdx.x);
}

// One find_noise_idx + impute_noisy_trace round (one block): idx = np.argmax(cond) over traces
// (first true, 0 if none) with cond = ||x_r|| < thr (empty) or max(x_r) > thr (noisy); then
// x[idx] = x[idx-1] (last), x[1] (first) or x[idx-1] + x[idx+1] (a sum, as the reference does);
// the trace's stats are refreshed for the next round.
template <typename T>
__global__ __launch_bounds__(kStatBlock) void impute_kernel(T* __restrict__ x, int64_t n_rows, int64_t row_stride,
                                                             int32_t n_t, int32_t empty, double thr,
                                                             double* __restrict__ stats, int32_t* __restrict__ idx_out) {
  __shared__ int first;
  if (threadIdx.x == 0) first = INT32_MAX;
  __syncthreads();
  for (int64_t r = threadIdx.x; r < n_rows; r += blockDim.x) {
    const bool c = empty ? (sqrt(stats[2 * r]) < thr) : (stats[2 * r + 1] > thr);
    if (c) atomicMin(&first, (int)r);
  }
  __syncthreads();
  const int64_t idx = first == INT32_MAX ? 0 : first;
  if (threadIdx.x == 0 && idx_out) *idx_out = (int32_t)idx;
  if (n_rows < 2) return;  // x[0] = x[-1] is x[0] itself
  T* dst = x + idx * row_stride;
  const T* a = x + (idx + 1 == n_rows ? idx - 1 : (idx == 0 ? 1 : idx - 1)) * row_stride;
  const T* b = (idx > 0 && idx + 1 < n_rows) ? x + (idx + 1) * row_stride : nullptr;
  for (int t = threadIdx.x; t < n_t; t += blockDim.x) dst[t] = b ? (T)(a[t] + b[t]) : a[t];
  __syncthreads();
  block_row_stats(dst, n_t, stats + 2 * idx);
}

// data /= np.linalg.norm(data, axis=-1, keepdims=True)
template <typename T>
__global__ __launch_bounds__(256) void row_normalize_kernel(T* __restrict__ x, int64_t row_stride, int32_t n_t,
                                                            const double* __restrict__ stats) {
  const int64_t r = blockIdx.y;
  const double nrm = sqrt(stats[2 * r]);
  T* row = x + r * row_stride;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n_t; t += gridDim.x * blockDim.x)
    row[t] = (T)((double)row[t] / nrm);
}

template <typename T>
static int trace_cleanup(T* x, int64_t n_rows, int64_t row_stride, int32_t n_t, int32_t flags, double thr,
                         double* stats, int32_t* idx_out, hipStream_t s) {
  hipLaunchKernelGGL(row_stats_kernel<T>, dim3((unsigned)n_rows), dim3(kStatBlock), 0, s, x, row_stride, n_t, stats);
  if (flags & 1)
    hipLaunchKernelGGL(impute_kernel<T>, dim3(1), dim3(kStatBlock), 0, s, x, n_rows, row_stride, n_t, 1, thr, stats,
                       idx_out);
  if (flags & 2)
    hipLaunchKernelGGL(impute_kernel<T>, dim3(1), dim3(kStatBlock), 0, s, x, n_rows, row_stride, n_t, 0, thr, stats,
                       idx_out ? idx_out + 1 : nullptr);
  if (flags & 4)
    hipLaunchKernelGGL(row_normalize_kernel<T>, dim3((unsigned)((n_t + 255) / 256), (unsigned)n_rows), dim3(256), 0,
                       s, x, row_stride, n_t, stats);
  return last_launch();
}

// SurfaceWaveSelector.locate_windows' cut (apis/data_classes.py:208-209, deepcopy of
// data[x_start:x_start + n_ch, t_start[w]:t_start[w] + n_t]) for all accepted passes at once:
// out[w][c][t] (contiguous batch, converted to Out).  Reads are guarded against the record's
// extent; a window outside it sets *status and is left unwritten.
template <typename In, typename Out>
__global__ __launch_bounds__(256) void cut_windows_kernel(const In* __restrict__ rec, int64_t n_rows,
                                                          int64_t row_stride, int64_t rec_n_t,
                                                          const int64_t* __restrict__ t_start, int64_t x_start,
                                                          int32_t n_ch, int32_t n_t, Out* __restrict__ out,
                                                          int32_t* __restrict__ status) {
  const int64_t w = blockIdx.z;
  const int c = blockIdx.y;
  const int64_t ts = t_start[w];
  if (ts < 0 || ts + n_t > rec_n_t || x_start < 0 || x_start + n_ch > n_rows) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && c == 0 && status) atomicOr(status, 1);
    return;
  }
  const In* src = rec + (x_start + c) * row_stride + ts;
  Out* dst = out + (w * n_ch + c) * (int64_t)n_t;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n_t; t += gridDim.x * blockDim.x) dst[t] = (Out)src[t];
}

template <typename In, typename Out>
static int cut_windows(const void* rec, int64_t n_rows, int64_t row_stride, int64_t rec_n_t, const int64_t* t_start,
                       int32_t n_win, int64_t x_start, int32_t n_ch, int32_t n_t, void* out, int32_t* status,
                       hipStream_t s) {
  const unsigned gx = (unsigned)((n_t + 255) / 256 < 64 ? (n_t + 255) / 256 : 64);
  for (int32_t w0 = 0; w0 < n_win; w0 += 65535) {  // gridDim.z limit
    const int32_t nw = n_win - w0 < 65535 ? n_win - w0 : 65535;
    hipLaunchKernelGGL((cut_windows_kernel<In, Out>), dim3(gx, n_ch, nw), dim3(256), 0, s, (const In*)rec, n_rows,
                       row_stride, rec_n_t, t_start + w0, x_start, n_ch, n_t,
                       (Out*)out + (int64_t)w0 * n_ch * n_t, status);
  }
  return last_launch();
}

}  // namespace dvh

using namespace dvh;

DVH_API int dvh_trace_cleanup(void* x, int32_t dtype, int64_t n_rows, int64_t row_stride, int32_t n_t, int32_t flags,
                              double noise_threshold, double* stats, int32_t* idx_out, void* stream) {
  if (!x || !stats) return set_error(-2, "null pointer argument");
  if (n_rows <= 0 || n_t <= 0) return 0;
  if (n_rows > 65535 && (flags & 4)) return set_error(-4, "too many traces for one launch");
  if (dtype == 0)
    return trace_cleanup<float>((float*)x, n_rows, row_stride, n_t, flags, noise_threshold, stats, idx_out,
                                (hipStream_t)stream);
  if (dtype == 1)
    return trace_cleanup<double>((double*)x, n_rows, row_stride, n_t, flags, noise_threshold, stats, idx_out,
                                 (hipStream_t)stream);
  return set_error(-2, "dtype must be 0 (float32) or 1 (float64)");
}

DVH_API int dvh_sosfiltfilt(void* x, int32_t dtype, int64_t n_rows, int64_t row_stride, int32_t n_t,
                            const double* sos, int32_t n_sec, int32_t padlen, const double* zi, double* work,
                            void* stream) {
  if (!x || !sos || !zi || !work) return set_error(-2, "null pointer argument");
  if (n_sec <= 0 || n_sec > kMaxSec) return set_error(-4, "unsupported number of second-order sections");
  if (n_t <= padlen) return set_error(-4, "The length of the input vector x must be greater than padlen");
  if (padlen < 0 || n_t < 2) return set_error(-2, "invalid padlen / length");
  if (n_rows <= 0) return 0;
  const dim3 grid((unsigned)((n_rows + 63) / 64));
  if (dtype == 0)
    hipLaunchKernelGGL(sosfiltfilt_kernel<float>, grid, dim3(64), 0, (hipStream_t)stream, (float*)x, n_rows,
                       row_stride, n_t, sos, n_sec, padlen, zi, work);
  else if (dtype == 1)
    hipLaunchKernelGGL(sosfiltfilt_kernel<double>, grid, dim3(64), 0, (hipStream_t)stream, (double*)x, n_rows,
                       row_stride, n_t, sos, n_sec, padlen, zi, work);
  else
    return set_error(-2, "dtype must be 0 (float32) or 1 (float64)");
  return last_launch();
}

DVH_API int dvh_mute_traj(void* data, int32_t dtype, int32_t n_pass, int64_t pass_stride, int32_t n_ch, int32_t n_t,
                          const int32_t* tab, const double* taper, void* stream) {
  if (!data || !tab || !taper) return set_error(-2, "null pointer argument");
  if (n_pass <= 0 || n_ch <= 0 || n_t <= 0) return 0;
  const dim3 grid((n_t + 255) / 256, n_ch, n_pass);
  if (dtype == 0)
    hipLaunchKernelGGL(mute_traj_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, (float*)data, pass_stride,
                       n_ch, n_t, tab, taper);
  else if (dtype == 1)
    hipLaunchKernelGGL(mute_traj_kernel<double>, grid, dim3(256), 0, (hipStream_t)stream, (double*)data, pass_stride,
                       n_ch, n_t, tab, taper);
  else
    return set_error(-2, "dtype must be 0 (float32) or 1 (float64)");
  return last_launch();
}

DVH_API int dvh_mute_time(void* data, int32_t dtype, int64_t n_rows, int32_t n_t, const double* taper, void* stream) {
  if (!data || !taper) return set_error(-2, "null pointer argument");
  if (n_rows <= 0 || n_t <= 0) return 0;
  const int64_t n = n_rows * n_t;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (dtype == 0)
    hipLaunchKernelGGL(mute_time_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, (float*)data, n_rows, n_t,
                       taper);
  else if (dtype == 1)
    hipLaunchKernelGGL(mute_time_kernel<double>, grid, dim3(256), 0, (hipStream_t)stream, (double*)data, n_rows, n_t,
                       taper);
  else
    return set_error(-2, "dtype must be 0 (float32) or 1 (float64)");
  return last_launch();
}

DVH_API int dvh_cut_windows(const void* rec, int32_t in_dtype, int64_t n_rows, int64_t row_stride, int64_t rec_n_t,
                            const int64_t* t_start, int32_t n_win, int64_t x_start, int32_t n_ch, int32_t n_t,
                            void* out, int32_t out_dtype, int32_t* status, void* stream) {
  if (!rec || !t_start || !out) return set_error(-2, "null pointer argument");
  if (n_win < 0 || n_ch < 0 || n_t < 0) return set_error(-2, "invalid sizes");
  if (n_win == 0 || n_ch == 0 || n_t == 0) return 0;
  if (n_ch > 65535) return set_error(-4, "too many channels for one launch");
  if (x_start < 0 || x_start + n_ch > n_rows || n_t > rec_n_t) return set_error(-2, "window outside the record");
  const hipStream_t s = (hipStream_t)stream;
  if (in_dtype == 0 && out_dtype == 0)
    return cut_windows<float, float>(rec, n_rows, row_stride, rec_n_t, t_start, n_win, x_start, n_ch, n_t, out, status, s);
  if (in_dtype == 1 && out_dtype == 0)
    return cut_windows<double, float>(rec, n_rows, row_stride, rec_n_t, t_start, n_win, x_start, n_ch, n_t, out, status, s);
  if (in_dtype == 0 && out_dtype == 1)
    return cut_windows<float, double>(rec, n_rows, row_stride, rec_n_t, t_start, n_win, x_start, n_ch, n_t, out, status, s);
  if (in_dtype == 1 && out_dtype == 1)
    return cut_windows<double, double>(rec, n_rows, row_stride, rec_n_t, t_start, n_win, x_start, n_ch, n_t, out, status,
                                       s);
  return set_error(-2, "dtype must be 0 (float32) or 1 (float64)");
}
