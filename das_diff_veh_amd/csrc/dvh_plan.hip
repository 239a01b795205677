// Per-pass index tables derived on the device, in float64 with the reference's own expressions.
//
// Replaces the per-pass host arithmetic of
//   preprocessing_window            apis/virtual_shot_gather.py:111-126
//       f = interp1d(veh_state_x, veh_state_t, fill_value='extrapolate')      (:115)
//       pt = np.argmax(t_axis >= f(pivot) + delta_t)                           (:117)
//   xcorr_two_traces_based_on_traj   apis/virtual_shot_gather.py:24-35
//       t_idx = np.argmax(t_axis >= f(x_axis[row]) +- delta_t); slices [t_idx, t_idx + nsamp)
//       (forward) / [t_idx - nsamp, t_idx) (other side), Python slice semantics
//   XCORR_vshot's shared slice       apis/virtual_shot_gather.py:152, 172
// so that a batch's seg_tab (the tables dvh_vsg_* consume) is formed inside the measured pipeline
// instead of by das_diff_veh_amd.plan.pass_geometry on the host (bit-identical: tests/test_plan_gpu.py).
//
// interp1d (SciPy 1.15 _call_linear): i = clip(searchsorted(x, xq, 'left'), 1, n - 1), lo = i - 1,
//   slope = (y[i] - y[lo]) / (x[i] - x[lo]),  f = slope * (xq - x[lo]) + y[lo]
// evaluated without contraction (no FMA), so every rounding is the one numpy performs.
// np.argmax(t >= v) on an ascending t is the first index with t[i] >= v, and 0 when none (v above
// the axis, or NaN).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>

#include "dvh_common.h"
#include "dvh.h"

#pragma clang fp contract(off)

namespace dvh {
namespace {

constexpr int kGeomBlock = 1024;  // one row per thread at R = 1023: the rows' dependent-load chains run side by side

// first index i in [0, n) with !(a[i] < v); n when every a[i] < v.  For an ascending a this is
// searchsorted(a, v, 'left'); a NaN v gives 0.
__device__ __forceinline__ int lower_bound(const double* __restrict__ a, int n, double v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// lower_bound for an ascending a, started from the index a straight line through (a[0], a[n-1])
// predicts: the answer is checked against its definition (a[i-1] < v <= a[i]) with two loads, and
// only a miss falls back to the bisection, narrowed to the side of the guess the answer lies on.
// Same result as lower_bound for every ascending a (uniform axes and tracking grids hit the guess
// or its neighbour, so the 13-step chain of dependent loads over an 8192-sample axis becomes 2-4).
__device__ __forceinline__ int lower_bound_guess(const double* __restrict__ a, int n, double v) {
  if (n <= 0) return 0;
  const double a0 = a[0], a1 = a[n - 1];
  double gd = (n > 1 && a1 > a0) ? (v - a0) / (a1 - a0) * (double)(n - 1) + 1.0 : 0.0;
  if (!(gd >= 0.0)) gd = 0.0;  // NaN v lands here
  if (gd > (double)n) gd = (double)n;
  const int g = (int)gd;
  const bool lo_ok = g == 0 || a[g - 1] < v;
  const bool hi_ok = g == n || !(a[g] < v);
  if (lo_ok && hi_ok) return g;
  if (lo_ok) {  // a[g] < v: the answer is above g; try g + 1 before bisecting
    if (g + 1 == n || !(a[g + 1] < v)) return g + 1;
    int lo = g + 2, hi = n;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (a[mid] < v) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  }
  // !(a[g-1] < v): the answer is at most g - 1
  if (g - 1 == 0 || a[g - 2] < v) return g - 1;
  int lo = 0, hi = g - 2;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// np.argmax(t >= v) for ascending t
__device__ __forceinline__ int first_ge(const double* __restrict__ t, int n, double v) {
  const int i = lower_bound_guess(t, n, v);
  return i >= n ? 0 : i;
}

// interp1d(x, y, kind='linear', fill_value='extrapolate')(xq) for strictly ascending x, n >= 2
__device__ __forceinline__ double interp_extrap(const double* __restrict__ x, const double* __restrict__ y, int n,
                                                double xq) {
  int i = lower_bound_guess(x, n, xq);
  i = i < 1 ? 1 : (i > n - 1 ? n - 1 : i);
  const int lo = i - 1;
  const double slope = __ddiv_rn(__dsub_rn(y[i], y[lo]), __dsub_rn(x[i], x[lo]));
  return __dadd_rn(__dmul_rn(slope, __dsub_rn(xq, x[lo])), y[lo]);
}

// (start, length) of s[a:b] for len(s) == n (Python slice semantics, step 1)
__device__ __forceinline__ int2 py_slice(int64_t a, int64_t b, int64_t n) {
  a = a < 0 ? (a + n > 0 ? a + n : 0) : (a < n ? a : n);
  b = b < 0 ? (b + n > 0 ? b + n : 0) : (b < n ? b : n);
  return make_int2((int)a, (int)(b > a ? b - a : 0));
}

// One block per pass: every thread evaluates f(pivot) (a handful of loads, identical result) and
// then the rows i = tid, tid + blockDim.x, ...
__global__ __launch_bounds__(kGeomBlock) void pass_geometry_kernel(
    const double* __restrict__ x_axis, int64_t x_stride, const double* __restrict__ t_axis, int64_t t_stride,
    int32_t n_t, const double* __restrict__ trk_x, const double* __restrict__ trk_t, int64_t trk_stride,
    const int32_t* __restrict__ trk_len, const double* __restrict__ pivot_x, const int32_t* __restrict__ pass_tab,
    int32_t R, double delta_t, int32_t nsamp, int32_t flags, int32_t* __restrict__ seg_tab,
    int32_t* __restrict__ status) {
  const int p = blockIdx.x;
  const double* xa = x_axis + (int64_t)p * x_stride;
  const double* ta = t_axis + (int64_t)p * t_stride;
  const double* tx = trk_x + (int64_t)p * trk_stride;
  const double* tt = trk_t + (int64_t)p * trk_stride;
  const int L = trk_len[p];
  // interp1d needs >= 2 points; the search assumes strictly ascending abscissae (the tracking grid
  // emits them so; interp1d's mergesort is then the identity)
  int bad = L < 2;
  for (int k = threadIdx.x + 1; k < L; k += blockDim.x) bad |= !(tx[k] > tx[k - 1]);
  bad = __syncthreads_or(bad);
  if (threadIdx.x == 0) status[p] = bad ? 1 : 0;
  int32_t* seg = seg_tab + (int64_t)p * R * 4;
  if (bad) {
    for (int i = threadIdx.x; i < R * 4; i += blockDim.x) seg[i] = 0;
    return;
  }
  const int row0 = pass_tab[2 * p], pivot_idx = pass_tab[2 * p + 1];
  const double fp = interp_extrap(tx, tt, L, pivot_x[p]);
  const bool other = (flags & 1) != 0;
  const int pt_f = first_ge(ta, n_t, __dadd_rn(fp, delta_t));
  const int pt_o = first_ge(ta, n_t, __dadd_rn(fp, -delta_t));
  for (int i = threadIdx.x; i < R; i += blockDim.x) {
    const int ch = row0 + i;
    const bool fwd_shared = ch <= pivot_idx, oth_shared = ch >= pivot_idx;
    double fx = 0.0;
    if (!fwd_shared || (other && !oth_shared)) fx = interp_extrap(tx, tt, L, xa[ch]);
    const int a = fwd_shared ? pt_f : first_ge(ta, n_t, __dadd_rn(fx, delta_t));
    const int2 sf = py_slice(a, (int64_t)a + nsamp, n_t);
    int2 so = make_int2(0, 0);
    if (other) {
      const int b = oth_shared ? pt_o : first_ge(ta, n_t, __dsub_rn(fx, delta_t));
      so = py_slice((int64_t)b - nsamp, b, n_t);
    }
    int32_t* s = seg + 4 * i;
    s[0] = sf.x;
    s[1] = sf.y;
    s[2] = so.x;
    s[3] = so.y;
  }
}

}  // namespace
}  // namespace dvh

using namespace dvh;

DVH_API int dvh_pass_geometry(const double* x_axis, int64_t x_stride, const double* t_axis, int64_t t_stride,
                              int32_t n_t, const double* trk_x, const double* trk_t, int64_t trk_stride,
                              const int32_t* trk_len, const double* pivot_x, const int32_t* pass_tab, int32_t n_pass,
                              int32_t R, double delta_t, int32_t nsamp, int32_t flags, int32_t* seg_tab,
                              int32_t* status, void* stream) {
  if (!x_axis || !t_axis || !trk_x || !trk_t || !trk_len || !pivot_x || !pass_tab || !seg_tab || !status)
    return set_error(-2, "null pointer argument");
  if (n_pass < 0 || R <= 0 || n_t < 1 || nsamp < 0 || x_stride < 0 || t_stride < 0 || trk_stride < 0)
    return set_error(-2, "invalid geometry (n_pass, R, n_t, nsamp, strides)");
  if (n_pass == 0) return 0;
  // one thread per row (whole waves): a narrow gather (configs[1]: R = 48) gets one wave per pass, not 16 idle ones
  const int block = std::min(kGeomBlock, std::max(64, (R + 63) / 64 * 64));
  hipLaunchKernelGGL(pass_geometry_kernel, dim3(n_pass), dim3(block), 0, (hipStream_t)stream, x_axis, x_stride,
                     t_axis, t_stride, n_t, trk_x, trk_t, trk_stride, trk_len, pivot_x, pass_tab, R, delta_t, nsamp,
                     flags, seg_tab, status);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_error(-3, hipGetErrorString(e));
}
