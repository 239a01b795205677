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
#include <stdlib.h>

#include <algorithm>

#include "vsg_engines.h"
#include "dvh_common.h"
#include "dvh.h"

namespace dvh {

constexpr int kBlock = 512;  // sumsq kernel
// waves per SIMD the kernels are compiled for: the Stockham engines are register-limited to 3,
// EngF500 fits 4
template <class E> struct Occ { static constexpr int v = 3; };
template <> struct Occ<EngF500> { static constexpr int v = 4; };
// Occupancy target of the stack kernels: 4 waves/SIMD for the exact Stockham engines up to N = 500
// (their spills at 128 VGPRs sit in the rare time-domain fallback only), else the engine default.
template <class E> struct OccF {
  static constexpr int v = E::kWaves == 4 && E::NFFT <= 500 ? 4 : Occ<E>::v;
};

// The engines with fused first / last stages (FusedOps: EngF500, EngP1024) take a per-pass pivot-slice
// spectra table in the stack kernels and pack single-sided tasks across passes.
template <class E> struct Fused { static constexpr bool v = false; };
template <> struct Fused<EngF500> { static constexpr bool v = true; };
template <> struct Fused<EngP1024> { static constexpr bool v = true; };

// Per-kernel engine setup: the sub-window length (the padded engines mask their loads with it) and the
// pivot-slice table (stack kernels; nullptr elsewhere).
template <class E>
__device__ __forceinline__ void bind_engine(E& e, const VsgArgs& A, const float2* tab) {
  if constexpr (Fused<E>::v) {
    e.w = A.w;
    e.tab = tab;
  }
}

// One row task's cross spectra: a fused engine with a bound pivot-spectra table uses it (stack kernels).
template <class E>
__device__ __forceinline__ void engine_spectra(E& eng, const VsgArgs& A, const RowTask& t, const RowTask& tn,
                                               bool has_next, float2 (&Cf)[E::NH], float2 (&Co)[E::NH]) {
  if constexpr (Fused<E>::v) {
    if (eng.tab && eng.tab_usable(t.p, A.n_pass)) {
      eng.spectra_tab(t, A.n_pass, A.hop, Cf, Co);
      return;
    }
  }
  eng.spectra(t, tn, has_next, A.w, A.hop, Cf, Co);
}

// A row task whose passes have only a table-served forward side, transformed across passes.  RAMP: the exact
// engines' output-spectrum form; otherwise the forward spectrum sum (*shared: its lag convention).
template <class E, bool RAMP>
__device__ __forceinline__ bool engine_direct(E& eng, const VsgArgs& A, const float* scales, const int32_t* order,
                                              const float* weight, int b, int e, int i, float2 (&Gh)[E::NH],
                                              bool* shared = nullptr) {
  if constexpr (Fused<E>::v) {
    return eng.tab && eng.template direct_task<RAMP>(A, scales, order, weight, b, e, i, Gh, shared);
  } else {
    return false;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// the next index from a global work counter (one atomic per wave)
__device__ __forceinline__ int pull_unit(uint32_t* counter, int lane) {
  int u = 0;
  if (lane == 0) u = (int)atomicAdd(counter, 1u);
  return __builtin_amdgcn_readfirstlane(__shfl(u, 0));
}


// XCD-aware block order (blocks are dealt round robin over the 8 XCDs, each with its own L2):
// consecutive logical blocks -- the row tasks of one pass chunk, which all read that chunk's pivot
// channel -- run on the same XCD.  A bijection on [0, gridDim.x).
__device__ __forceinline__ int xcd_block() {
  const int G = gridDim.x, b = blockIdx.x;
  const int q = G / 8, r = G % 8, x = b % 8, k = b / 8;
  return x < r ? x * (q + 1) + k : r * (q + 1) + (x - r) * q + k;
}

// The row tasks [0, n) of a stack launch as one wave takes them: a static stride (t0, t0 + stride, ...), or pulled
// from a global counter.  (Eight per-XCD counters, each XCD draining its own eighth of the tasks before the others'
// leftovers, measured no faster on the padded engine: w = 499 synth10k launch 15.05 vs 14.99 ms, weights 1.80-1.83
// vs 1.81-1.83 ms.)
struct TaskSource {
  uint32_t* q = nullptr;  // nullptr: static stride
  int64_t n = 0, stride = 1;
  __device__ int64_t first(int64_t t0, int lane) { return q ? pull_unit(q, lane) : t0; }
  __device__ int64_t next(int64_t t, int lane) { return q ? pull_unit(q, lane) : t + stride; }
};

template <class E>
__device__ __forceinline__ E make_engine(char* lds) {
  E::block_init(lds);
  __syncthreads();
  return E(lds, threadIdx.x >> 6, threadIdx.x & 63);
}

// The reference divides every window by ||data||_F first (preprocessing_window,
// apis/virtual_shot_gather.py:125): a window holding a NaN / inf, or all zero (0 / 0), turns the
// whole gather into NaN.  With win_sumsq = ||data||_F^2 given, such a pass gets NaN scales, which
// the gather / stack kernels carry into every computed row exactly as that division does.
__device__ __forceinline__ bool window_invalid(const double* __restrict__ sumsq, int p) {
  if (!sumsq) return false;
  const double s = sumsq[p];
  return !(s > 0.0) || !isfinite(s);
}

// Per-pass scale of each side: 1 / max(pivot autocorrelation row) after the optional row norm
// (post_processing_XCF with norm_amp=True); 1 / ||window||_F^2 when neither norm is requested.
template <class E>
__global__ __launch_bounds__(64 * E::kWaves, Occ<E>::v) void vsg_scales_kernel(VsgArgs A, const double* __restrict__ sumsq,
                                                             float* __restrict__ scales) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  E eng = make_engine<E>(lds);
  bind_engine(eng, A, nullptr);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const bool other = (A.flags & kFlagOtherSide) != 0;
  const bool norm = (A.flags & kFlagNorm) != 0;
  const bool norm_amp = (A.flags & kFlagNormAmp) != 0;
  constexpr int NJ = E::NJ;
  const int stride = gridDim.x * E::kWaves;
  for (int p = blockIdx.x * E::kWaves + wave; p < A.n_pass; p += stride) {
    if (!norm_amp || window_invalid(sumsq, p)) {
      if (lane == 0) {
        const float s = window_invalid(sumsq, p) ? NAN : (norm ? 1.0f : (float)(1.0 / sumsq[p]));
        scales[2 * p] = s;
        scales[2 * p + 1] = s;
      }
      continue;
    }
    const RowTask t = make_task(A, p, uni(A.pass_tab[2 * p + 1] - A.pass_tab[2 * p]));  // the pivot row
    RowTask tn = t;
    const bool has_next = norm_amp && p + stride < A.n_pass;
    if (has_next) tn = make_task(A, p + stride, uni(A.pass_tab[2 * (p + stride) + 1] - A.pass_tab[2 * (p + stride)]));
    const float2* Y = eng.correlate(t, tn, has_next, A.w, A.hop);
    float mf = -INFINITY, mo = -INFINITY, sf = 0.f, so = 0.f;
    bool nanf = false, nano = false;
    // a side with nothing accumulated is exactly zero in the reference (the packed inverse FFT
    // would otherwise leak the other side's rounding into it)
    const float2 live = make_float2(eng.live_f ? 1.f : 0.f, eng.live_o ? 1.f : 0.f);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int k = lane + 64 * j;
      if (k < A.w) {
        float2 c = eng.c(Y, k, A.w);
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
      amax_f = t.nwin_f > 0 ? mf / ((float)E::NFFT * (float)t.nwin_f) : 0.f;
      amax_o = t.nwin_o > 0 ? mo / ((float)E::NFFT * (float)t.nwin_o) : 0.f;
    }
    if (anynanf) amax_f = NAN;
    if (anynano) amax_o = NAN;
    if (lane == 0) {
      scales[2 * p] = 1.0f / amax_f;
      scales[2 * p + 1] = other ? 1.0f / amax_o : 0.f;
    }
  }
}

// Applies the per-pass scales to the row factors.  With neither norm the reference scales the DATA
// (data / ||data||, virtual_shot_gather.py:124), so a side without sub-windows stays exactly 0 even
// when the window is all zero or holds a NaN; otherwise the scale divides the finished row and
// 0 * (1 / amax) reproduces its 0 / amax.
__device__ __forceinline__ void side_scale(int flags, const RowTask& t, float sf, float so, float& ff, float& fo) {
  if (!(flags & (kFlagNorm | kFlagNormAmp))) {
    ff = t.nwin_f > 0 ? ff * sf : 0.f;
    fo = t.nwin_o > 0 ? fo * so : 0.f;
  } else {
    ff *= sf;
    fo *= so;
  }
}

// Time-domain epilogue of a row: lag permutation, per-pass scales, optional row norm, two-sided
// average -> G[m] for output lag j = lane + 64 m (post_processing_XCF + VirtualShotGather.__init__).

template <class E>
__device__ __forceinline__ void row_epilogue(const E& eng, const VsgArgs& A, const float2* Y, const RowTask& t,
                                             float sf, float so, int lane_, float (&G)[E::NJ]) {
  constexpr int NJ = E::NJ;
  const int lane = opaque(lane_);  // cold path (norms / NaN fallback): keep its index math local
  const bool other = (A.flags & kFlagOtherSide) != 0;
  const bool norm = (A.flags & kFlagNorm) != 0;
  const int w = A.w, h = w / 2;
  // a side with nothing accumulated is exactly zero in the reference (see vsg_scales_kernel)
  const float2 live = make_float2(eng.live_f ? 1.f : 0.f, eng.live_o ? 1.f : 0.f);
  float ff, fo;
  if (norm) {
    float s2f = 0.f, s2o = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int k = lane + 64 * j;
      if (k < w) {
        float2 c = eng.c(Y, k, w);
        c.x *= live.x;
        c.y *= live.y;
        s2f += c.x * c.x;
        s2o += c.y * c.y;
      }
    }
    ff = 1.0f / sqrtf(wave_sum(s2f));
    fo = 1.0f / sqrtf(wave_sum(s2o));
  } else {
    ff = t.nwin_f > 0 ? 1.0f / ((float)E::NFFT * (float)t.nwin_f) : 0.f;
    fo = t.nwin_o > 0 ? 1.0f / ((float)E::NFFT * (float)t.nwin_o) : 0.f;
  }
  side_scale(A.flags, t, sf, so, ff, fo);
  const bool fwd_shared = t.ch <= t.pivot;
  const bool oth_shared = t.ch >= t.pivot;
  float O[NJ];
  bool nan_o = false, nz_o = false;
#pragma unroll
  for (int m = 0; m < NJ; ++m) {
    const int j = lane + 64 * m;
    G[m] = 0.f;
    O[m] = 0.f;
    if (j < w) {
      const int kf = fwd_shared ? pmod(w - 1 - j - h, w) : pmod(j + h + 1, w);
      G[m] = (eng.c(Y, kf, w).x * live.x) * ff;
      if (other) {
        const int ko = oth_shared ? pmod(h - 1 - j, w) : pmod(j - h, w);
        O[m] = (eng.c(Y, ko, w).y * live.y) * fo;
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

template <class E>
__device__ __forceinline__ void gather_row(E& eng, const VsgArgs& A, const float* __restrict__ scales, int p,
                                           const RowTask& t, const RowTask& nt, bool has_next, int lane,
                                           float (&G)[E::NJ]) {
  const float2* Y = eng.correlate(t, nt, has_next, A.w, A.hop);
  row_epilogue<E>(eng, A, Y, t, sld(scales + 2 * p), sld(scales + 2 * p + 1), lane, G);
}

template <class E>
__global__ __launch_bounds__(64 * E::kWaves, Occ<E>::v) void vsg_gather_kernel(VsgArgs A, const float* __restrict__ scales,
                                                             float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  E eng = make_engine<E>(lds);
  bind_engine(eng, A, nullptr);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  constexpr int NJ = E::NJ;
  const int64_t n_task = (int64_t)A.n_pass * A.R;
  const int64_t stride = (int64_t)gridDim.x * E::kWaves;
  for (int64_t t = (int64_t)xcd_block() * E::kWaves + wave; t < n_task; t += stride) {
    const int p = uni((int)(t / A.R)), i = uni((int)(t % A.R));
    const RowTask task = make_task(A, p, i);
    RowTask tn = task;
    const bool has_next = t + stride < n_task;
    if (has_next) tn = make_task(A, (int)((t + stride) / A.R), (int)((t + stride) % A.R));
    float G[NJ];
    gather_row<E>(eng, A, scales, p, task, tn, has_next, lane, G);
    float* o = out + t * A.w;
#pragma unroll
    for (int m = 0; m < NJ; ++m) {
      const int j = lane + 64 * m;
      if (j < A.w) o[j] = G[m];
    }
  }
}

// Stack mode, exact transforms (N == w): every pass's contribution is accumulated directly as the
// spectrum of its output row, Ghat[m] += w_p (alpha f_f Phase_F(Cf) + beta f_o Phase_O(Co)), where
// each lag convention of the reference is a conjugation and a phase ramp:
//   c[(a - j) mod w]  ->  W^(a m) conj(C[m]),      c[(j + b) mod w]  ->  W^(-b m) C[m]
// (alpha, beta) = (1/2, 1/2) when the other side is finite and non-zero, else (1, 0).  One inverse
// transform per (chunk, row) replaces the per-pass inverse transform and epilogue.  Passes with a
// non-finite scale or NaN data go through the exact time-domain path (row_epilogue) instead.
// The row tasks t0, t0 + stride, ... < n_chunk * R of one wave (task = (chunk, row)).
template <class E>
__device__ __forceinline__ void stackf_tasks(E& eng, const VsgArgs& A, const float* __restrict__ scales,
                                             const int32_t* __restrict__ order, const int32_t* __restrict__ chunk_tab,
                                             int32_t n_chunk, const float* __restrict__ weight,
                                             float* __restrict__ stack, int64_t t0, TaskSource src) {
  const int lane_ = threadIdx.x & 63;
  constexpr int NJ = E::NJ;
  constexpr int NH = E::NH;
  constexpr int N = E::NFFT;
  const bool other = (A.flags & kFlagOtherSide) != 0;
  const bool norm = (A.flags & kFlagNorm) != 0;
  const int h = N / 2;
  const int64_t n_task = (int64_t)n_chunk * A.R;
  // tasks from src (static stride or pulled); the next index fetched at the top of the task so that `continue`
  // moves on
  const int lane_t = threadIdx.x & 63;
  src.n = n_task;
  int64_t tn = src.first(t0, lane_t);
  for (int64_t t = tn; t < n_task; t = tn) {
    tn = src.next(t, lane_t);
    const int c = uni((int)(t / A.R)), i = uni((int)(t % A.R));
    const int b = sld(chunk_tab + 3 * c), e = sld(chunk_tab + 3 * c + 1), slot = sld(chunk_tab + 3 * c + 2);
    float* o = stack + ((int64_t)slot * A.R + i) * A.w;
    float2 Gh[NH];
#pragma unroll
    for (int m = 0; m < NH; ++m) Gh[m] = make_float2(0.f, 0.f);
    const bool direct = !norm && engine_direct<E, true>(eng, A, scales, order, weight, b, e, i, Gh);
    for (int q = direct ? e : b; q < e; ++q) {
      const int p = sld(order + q);
      const RowTask task = make_task(A, p, i);
      float2 Cf[NH], Co[NH];
      engine_spectra(eng, A, task, task, false, Cf, Co);
      const float sf = sld(scales + 2 * p), so = sld(scales + 2 * p + 1), wp = sld(weight + p);
      // per-pass bin / twiddle-index math recomputed here (hoisted, it only spills)
      const int lane = opaque(lane_);
      // sums of |.| over the half spectra: NaN iff some bin is NaN (sums of non-negative values never
      // turn infinities into NaN); the other side is non-zero iff its sum is
      float af = 0.f, ao = 0.f;
#pragma unroll
      for (int m = 0; m < NH; ++m) {
        if (E::bin(lane, m) >= 0) {
          af += fabsf(Cf[m].x) + fabsf(Cf[m].y);
          ao += fabsf(Co[m].x) + fabsf(Co[m].y);
        }
      }
      const bool bad = __ballot(isnan(af + ao)) != 0;
      const bool nzo = other && (__ballot(ao != 0.f) != 0);
      if constexpr (Fused<E>::v) {  // covered-span scan: a non-finite sample among this pass's loaded slices
        if (eng.vflag && __ballot(!isfinite(af + ao)) != 0 && lane_ == 0) atomicMax(eng.vflag + p, kInfBits);
      }
      float ff, fo;
      if (norm) {  // ||c||^2 = sum_m |C[m]|^2 / N (Parseval over all N bins: interior bins count twice)
        float s2f = 0.f, s2o = 0.f;
#pragma unroll
        for (int m = 0; m < NH; ++m) {
          const int f = E::bin(lane, m);
          if (f >= 0) {
            const float wgt = (f == 0 || f == h) ? 1.f : 2.f;
            s2f += wgt * (Cf[m].x * Cf[m].x + Cf[m].y * Cf[m].y);
            s2o += wgt * (Co[m].x * Co[m].x + Co[m].y * Co[m].y);
          }
        }
        ff = sqrtf((float)N) / sqrtf(wave_sum(s2f));
        fo = sqrtf((float)N) / sqrtf(wave_sum(s2o));
      } else {
        ff = task.nwin_f > 0 ? 1.0f / (float)task.nwin_f : 0.f;
        fo = task.nwin_o > 0 ? 1.0f / (float)task.nwin_o : 0.f;
      }
      side_scale(A.flags, task, sf, so, ff, fo);
      if (bad || !isfinite(ff) || (nzo && !isfinite(fo))) {
        // exact time-domain path (NaN / inf semantics of the reference), added straight to the stack
        const float2* Y = eng.inverse(Cf, Co);
        float G[NJ];
        row_epilogue<E>(eng, A, Y, task, sf, so, lane, G);
#pragma unroll
        for (int m = 0; m < NJ; ++m) {
          const int j = lane + 64 * m;
          if (j < A.w) atomicAdd(o + j, G[m] * wp);
        }
        wave_sync();
      } else {
        // other row finite and not identically zero (row_epilogue's test)
        const bool ok = nzo && fo != 0.f;
        // lag shifts as phase ramps W^(s f): forward s = h - 1 on both row types (conj on the shared
        // window), other side s = h - 1 (shared, conj) or h (trajectory window).  W^(h f) = (-1)^f and
        // every engine's bins have the lane's parity, so W^((h-1) f) = (-1)^lane conj(tw[f]).
        const float sg = (lane & 1) ? -1.f : 1.f;
        const float cf = sg * wp * (ok ? 0.5f : 1.f) * ff;
        const float co = ok ? sg * wp * 0.5f * fo : 0.f;
        const bool fwd_shared = task.ch <= task.pivot;
        const bool oth_shared = task.ch >= task.pivot;
#pragma unroll
        for (int m = 0; m < NH; ++m) {
          const int f = E::bin(lane, m);
          if (f >= 0) {
            const float2 t = eng.twiddle(f);
            const float2 tc = make_float2(t.x, -t.y);
            float2 x = fwd_shared ? make_float2(Cf[m].x, -Cf[m].y) : Cf[m];
            x = cmul(x, tc);
            Gh[m].x += cf * x.x;
            Gh[m].y += cf * x.y;
            if (ok) {
              float2 y = Co[m];
              if (oth_shared) y = cmul(make_float2(y.x, -y.y), tc);
              Gh[m].x += co * y.x;
              Gh[m].y += co * y.y;
            }
          }
        }
      }
    }
    float2 Z[NH];
#pragma unroll
    for (int m = 0; m < NH; ++m) Z[m] = make_float2(0.f, 0.f);
    const float2* Y = eng.inverse(Gh, Z);
    const float inv_n = 1.0f / (float)N;
    const int lane = opaque(lane_);  // per-task addresses formed here, not held across the task loop
#pragma unroll
    for (int m = 0; m < NJ; ++m) {
      const int j = lane + 64 * m;
      if (j < A.w) atomicAdd(o + j, eng.c(Y, j, A.w).x * inv_n);
    }
    wave_sync();
  }
}

// Stack mode, zero-padded transforms (N >= 2w - 1, w without an exact engine, e.g. w = 499 on real time axes):
// the circular correlation is the fold c[k] = lin[k] + lin[k - w] of the linear one, so it cannot be phase-
// ramped in the N-point domain; but folding, the lag permutations and the class sum are linear.  The passes of
// a (chunk, row) task whose row has the same lag conventions as the chunk's first pass (every pass but those
// whose pivot row lies on the other side of this row) accumulate their weighted side spectra in registers,
//   Af += w_p alpha_p f_f,p Cf_p,   Ao += w_p beta_p f_o,p Co_p,
// then ONE inverse transform of Af + i Ao per task yields both sides' summed, folded correlations, which the
// epilogue permutes with the chunk's conventions and adds to the stack.  Passes with a row norm (the row's
// norm needs its own folded correlation), NaN data, non-finite factors or other conventions take the exact
// per-pass time-domain path.
template <class E>
__device__ __forceinline__ void stackp_tasks(E& eng, const VsgArgs& A, const float* __restrict__ scales,
                                             const int32_t* __restrict__ order, const int32_t* __restrict__ chunk_tab,
                                             int32_t n_chunk, const float* __restrict__ weight,
                                             float* __restrict__ stack, int64_t t0, TaskSource src) {
  const int lane_ = threadIdx.x & 63;
  constexpr int NJ = E::NJ;
  constexpr int NH = E::NH;
  constexpr int N = E::NFFT;
  const bool other = (A.flags & kFlagOtherSide) != 0;
  const bool norm = (A.flags & kFlagNorm) != 0;
  const int w = A.w, h = w / 2;
  const int64_t n_task = (int64_t)n_chunk * A.R;
  // tasks from src (static stride or pulled); the next index fetched at the top of the task so that `continue`
  // moves on
  const int lane_t = threadIdx.x & 63;
  src.n = n_task;
  int64_t tn = src.first(t0, lane_t);
  for (int64_t t = tn; t < n_task; t = tn) {
    tn = src.next(t, lane_t);
    const int c = uni((int)(t / A.R)), i = uni((int)(t % A.R));
    const int b = sld(chunk_tab + 3 * c), e = sld(chunk_tab + 3 * c + 1), slot = sld(chunk_tab + 3 * c + 2);
    float* o = stack + ((int64_t)slot * A.R + i) * A.w;
    float2 Af[NH], Ao[NH];
#pragma unroll
    for (int m = 0; m < NH; ++m) Af[m] = Ao[m] = make_float2(0.f, 0.f);
    bool fs0 = false, os0 = false, any = false, anyo = false;
    if (b < e) {
      const RowTask t0 = make_task(A, sld(order + b), i);
      fs0 = t0.ch <= t0.pivot;
      os0 = t0.ch >= t0.pivot;
    }
    // single-sided tasks with table-served forward slices: receivers packed across passes (fused engines)
    bool dshared = fs0;
    const bool direct = !norm && engine_direct<E, false>(eng, A, scales, order, weight, b, e, i, Af, &dshared);
    if (direct) {
      fs0 = dshared;
      any = true;
    }
    for (int q = direct ? e : b; q < e; ++q) {
      const int p = sld(order + q);
      const RowTask task = make_task(A, p, i);
      float2 Cf[NH], Co[NH];
      engine_spectra(eng, A, task, task, false, Cf, Co);
      const float sf = sld(scales + 2 * p), so = sld(scales + 2 * p + 1), wp = sld(weight + p);
      const int lane = opaque(lane_);
      float af = 0.f, ao = 0.f;
#pragma unroll
      for (int m = 0; m < NH; ++m) {
        if (E::bin(lane, m) >= 0) {
          af += fabsf(Cf[m].x) + fabsf(Cf[m].y);
          ao += fabsf(Co[m].x) + fabsf(Co[m].y);
        }
      }
      const bool bad = __ballot(isnan(af + ao)) != 0;
      const bool nzo = other && eng.live_o && (__ballot(ao != 0.f) != 0);
      if constexpr (Fused<E>::v) {  // covered-span scan: a non-finite sample among this pass's loaded slices
        if (eng.vflag && __ballot(!isfinite(af + ao)) != 0 && lane_ == 0) atomicMax(eng.vflag + p, kInfBits);
      }
      float ff = task.nwin_f > 0 ? 1.0f / (float)task.nwin_f : 0.f;
      float fo = task.nwin_o > 0 ? 1.0f / (float)task.nwin_o : 0.f;
      side_scale(A.flags, task, sf, so, ff, fo);
      const bool same = (task.ch <= task.pivot) == fs0 && (task.ch >= task.pivot) == os0;
      if (norm || bad || !same || !isfinite(ff) || (nzo && !isfinite(fo))) {
        // exact per-pass time-domain path, added straight to the stack
        const float2* Y = eng.inverse(Cf, Co);
        float G[NJ];
        row_epilogue<E>(eng, A, Y, task, sf, so, lane, G);
#pragma unroll
        for (int m = 0; m < NJ; ++m) {
          const int j = lane + 64 * m;
          if (j < A.w) atomicAdd(o + j, G[m] * wp);
        }
        wave_sync();
        continue;
      }
      // other row finite and not identically zero (row_epilogue's test): the two-sided average
      const bool ok = nzo && fo != 0.f;
      const float cf = wp * (ok ? 0.5f : 1.f) * ff, co = ok ? wp * 0.5f * fo : 0.f;
#pragma unroll
      for (int m = 0; m < NH; ++m) {
        Af[m].x += cf * Cf[m].x;
        Af[m].y += cf * Cf[m].y;
        Ao[m].x += co * Co[m].x;
        Ao[m].y += co * Co[m].y;
      }
      any = true;
      anyo |= ok;
    }
    if (!any) continue;
    // N * (sum of folded forward correlations, sum of folded other-side correlations) at lag k: eng.c(Y, k, w)
    const float2* Y = eng.inverse(Af, Ao);
    const float inv_n = 1.0f / (float)N;
#pragma unroll
    for (int m = 0; m < NJ; ++m) {
      const int j = lane_ + 64 * m;
      if (j < w) {
        const int kf = fs0 ? pmod(w - 1 - j - h, w) : pmod(j + h + 1, w);
        float g = eng.c(Y, kf, w).x;
        if (other && anyo) {  // (an all-zero Ao's inverse is rounding noise, not the exact 0 the reference adds)
          const int ko = os0 ? pmod(h - 1 - j, w) : pmod(j - h, w);
          g += eng.c(Y, ko, w).y;
        }
        atomicAdd(o + j, g * inv_n);
      }
    }
    wave_sync();
  }
}

// occupancy of the padded stack kernel: the N >= 1024 engines hold two accumulated side spectra besides the
// sub-window's (4 x 9 complex per lane at N = 1024) and would spill at 3 waves / SIMD
template <class E> struct OccP { static constexpr int v = E::NFFT >= 1000 ? 2 : Occ<E>::v; };

template <class E>
__global__ __launch_bounds__(64 * E::kWaves, OccP<E>::v) void vsg_stackp_kernel(
    VsgArgs A, const float* __restrict__ scales, const int32_t* __restrict__ order,
    const int32_t* __restrict__ chunk_tab, int32_t n_chunk, const float* __restrict__ weight,
    float* __restrict__ stack, const float2* __restrict__ ptab) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  E eng = make_engine<E>(lds);
  bind_engine(eng, A, ptab);
  const int wave = threadIdx.x >> 6;
  TaskSource src;
  src.stride = (int64_t)gridDim.x * E::kWaves;
  stackp_tasks<E>(eng, A, scales, order, chunk_tab, n_chunk, weight, stack, (int64_t)xcd_block() * E::kWaves + wave, src);
}

template <class E>
__global__ __launch_bounds__(64 * E::kWaves, OccF<E>::v) void vsg_stackf_kernel(
    VsgArgs A, const float* __restrict__ scales, const int32_t* __restrict__ order,
    const int32_t* __restrict__ chunk_tab, int32_t n_chunk, const float* __restrict__ weight,
    float* __restrict__ stack, const float2* __restrict__ ptab) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  E eng = make_engine<E>(lds);
  bind_engine(eng, A, ptab);
  const int wave = threadIdx.x >> 6;
  TaskSource src;
  src.stride = (int64_t)gridDim.x * E::kWaves;
  stackf_tasks<E>(eng, A, scales, order, chunk_tab, n_chunk, weight, stack, (int64_t)xcd_block() * E::kWaves + wave, src);
}

// The pivot-slice spectra table of every pass (FusedOps::spectra_tab) for engine E: one wave per pass forms the
// entries' (start, nwin) from the pivot row and the first / last gather rows and transforms their slices
// pairwise with the engine's transform (zero-padded past w for the padded engines), writing P[f] / 2, f <= N / 2,
// and each slice's non-zero flag at bin kTabBins - 1.
template <class E>
__global__ __launch_bounds__(256) void vsg_pivot_table_kernel(VsgArgs A, float2* __restrict__ tab) {
  constexpr int N = E::N, BINS = E::kTabBins;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float2* tw = reinterpret_cast<float2*>(lds);
  init_twiddles<N>(tw);
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float2* bufA = reinterpret_cast<float2*>(lds + sizeof(float2) * N + (size_t)wave * sizeof(float2) * 2 * N);
  float2* bufB = bufA + N;
  int32_t* head = reinterpret_cast<int32_t*>(tab + (int64_t)A.n_pass * tab_pass_f2<BINS>());
  for (int p = blockIdx.x * 4 + wave; p < A.n_pass; p += gridDim.x * 4) {
    const int row0 = sld(A.pass_tab + 2 * p), pivot = sld(A.pass_tab + 2 * p + 1);
    const RowTask tp = make_task(A, p, pivot - row0), tl = make_task(A, p, A.R - 1), t0 = make_task(A, p, 0);
    int st0 = tp.a_f, st1 = tp.a_o, st2 = tl.a_f, st3 = t0.a_o;
    int nw0 = tp.nwin_f, nw1 = tp.nwin_o, nw2 = tl.ch > pivot ? tl.nwin_f : 0, nw3 = t0.ch < pivot ? t0.nwin_o : 0;
    // an entry holds kTabSub sub-windows: a pass with more (time_window_to_xcorr > 2 wlen) is marked unusable
    // (every head nwin = -1, nothing transformed) and its row tasks take the plain z = P + i R path
    static_assert(kTabEnt == 4, "entries: pivot forward / other side, far-row forward / other side");
    if (!(nw0 <= kTabSub && nw1 <= kTabSub && nw2 <= kTabSub && nw3 <= kTabSub)) nw0 = nw1 = nw2 = nw3 = -1;
    // entry values by selects among scalars (a run-time index into a stack array went to scratch)
    auto pick = [](int e, int a0, int a1, int a2, int a3) { return e == 0 ? a0 : e == 1 ? a1 : e == 2 ? a2 : a3; };
    if (lane < 2 * kTabEnt)
      head[(int64_t)p * 2 * kTabEnt + lane] = (lane & 1) ? pick(lane >> 1, nw0, nw1, nw2, nw3) : pick(lane >> 1, st0, st1, st2, st3);
    // the slices (e, q), q < kTabSub, two per transform; absent ones are zero.  The next pair's samples are loaded
    // before this pair's transform (one load latency per pass instead of one per transform)
    constexpr int NL = (N + 63) / 64;
    auto load_pair = [&](int s0, float (&v0)[NL], float (&v1)[NL], bool& h0, bool& h1) {
      const int e0 = s0 / kTabSub, q0 = s0 % kTabSub, e1 = (s0 + 1) / kTabSub, q1 = (s0 + 1) % kTabSub;
      h0 = q0 < pick(e0, nw0, nw1, nw2, nw3);
      h1 = q1 < pick(e1, nw0, nw1, nw2, nw3);
      const float* x0 = tp.piv + pick(e0, st0, st1, st2, st3) + q0 * A.hop;
      const float* x1 = tp.piv + pick(e1, st0, st1, st2, st3) + q1 * A.hop;
#pragma unroll
      for (int k = 0; k < NL; ++k) {
        const int n = lane + 64 * k;
        const bool in = n < A.w;  // the padded engines' zeros past the sub-window (and n < N, as A.w <= N)
        v0[k] = (h0 && in) ? x0[n] : 0.f;
        v1[k] = (h1 && in) ? x1[n] : 0.f;
      }
    };
    float c0[NL], c1[NL];
    bool ch0, ch1;
    load_pair(0, c0, c1, ch0, ch1);
#pragma unroll 1
    for (int s0 = 0; s0 < kTabSub * kTabEnt; s0 += 2) {
      const int e0 = s0 / kTabSub, q0 = s0 % kTabSub, e1 = (s0 + 1) / kTabSub, q1 = (s0 + 1) % kTabSub;
      const bool h0 = ch0, h1 = ch1;
      uint32_t nz0 = 0, nz1 = 0;
      const float2* X = nullptr;
      if (h0 || h1) {
#pragma unroll
        for (int k = 0; k < NL; ++k) {
          const int n = lane + 64 * k;
          nz0 |= nzbits(c0[k]);
          nz1 |= nzbits(c1[k]);
          if (n < N) bufA[n] = make_float2(c0[k], c1[k]);
        }
      }
      if (s0 + 2 < kTabSub * kTabEnt) load_pair(s0 + 2, c0, c1, ch0, ch1);
      if (h0 || h1) {
        wave_sync();
        X = FftPlan<N>::T::run(bufA, bufB, tw, lane);
      }
      const bool l0 = __ballot(nz0 != 0) != 0, l1 = __ballot(nz1 != 0) != 0;
      float2* o0 = tab + (((int64_t)p * kTabEnt + e0) * kTabSub + q0) * BINS;
      float2* o1 = tab + (((int64_t)p * kTabEnt + e1) * kTabSub + q1) * BINS;
      for (int f = lane; f < BINS; f += 64) {
        float2 p0 = make_float2(0.f, 0.f), p1 = p0;
        if (X && f <= N / 2) {
          const float2 za = X[f], zc = X[f == 0 ? 0 : N - f];
          // P / 2 of each slice (the consumers separate 2 R from their own transforms)
          p0 = make_float2(0.25f * (za.x + zc.x), 0.25f * (za.y - zc.y));
          p1 = make_float2(0.25f * (za.y + zc.y), -0.25f * (za.x - zc.x));
        }
        if (f == BINS - 1) {
          p0 = make_float2(l0 ? 1.f : 0.f, 0.f);
          p1 = make_float2(l1 ? 1.f : 0.f, 0.f);
        }
        o0[f] = p0;
        o1[f] = p1;
      }
      wave_sync();
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Window validity fused into the stack launch.  The reference divides every window by ||data||_F
// (preprocessing_window, apis/virtual_shot_gather.py:125): a NaN or inf anywhere in the window, or
// an all-zero window, makes the whole gather NaN (norm / norm_amp divide by a NaN or zero maximum
// afterwards), and so its class mean.  Deciding that needs every sample of the window, 4x - 130x the
// bytes the correlations read.  In the validated stack launch, besides the correlation waves, one
// wave per block streams the windows (16 x 16-byte loads per lane in flight) and keeps the maximum
// of |x| as a bit pattern, max(bits & 0x7fffffff): >= 0x7f800000 means a NaN / inf, 0 means all
// zero.  Work is pulled in units of kScanRows channel rows from a global counter, by the scan waves
// from the start and by the correlation waves once their row tasks are done, so the HBM-bound scan
// runs under the VALU-bound transforms.  vsg_invalid_fill_kernel then sets the class slots holding an
// invalid pass to NaN.
//
// Scan windows: by default window s is pass s (win + s * pass_stride, n_ch rows), scanned in the
// correlation's class-sorted order so that both fronts start on the same passes (3.51 vs 3.53 ms per
// synth10k launch).  A unit launch (plan.UnitPlan: (pass, pivot) units over one flattened record) names
// its windows instead: scan_tab[s] = first record row of window s, and unit_scan[u] = the window whose
// flag unit u takes, so a pass imaged at several pivots is validated once per launch.
constexpr int kScanRows = 16;
constexpr int kScanDepth = 16;  // 16-byte loads per lane in flight (8 / 12 / 24 measured no better)
constexpr int kScanAux = 2;     // cache policy of the scan's buffer loads (nt; allocating loads measured 4 % slower on
                                // synth10k)

__device__ __forceinline__ uint32_t absbits(float x) { return __builtin_bit_cast(uint32_t, x) & 0x7fffffffu; }


// Buffer descriptor over [p, p + bytes) built from wave-uniform values (no waterfall loops around the
// loads); out-of-range loads return 0, which leaves a max |x| unchanged.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t scan_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* pu = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(pu, 0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// max |x| bit pattern over nf4 consecutive float4 (16-byte aligned): unconditional 16-byte buffer
// loads, kScanDepth per lane in flight (the descriptor's range check zeroes the tail)
template <int D = kScanDepth>
__device__ __forceinline__ uint32_t scan_span(const float* __restrict__ q, int nf4, int lane) {
  const __amdgpu_buffer_rsrc_t rs = scan_rsrc(q, (uint32_t)nf4 * 16u);
  const int nsteps = (nf4 + 63) >> 6;
  uint32_t m = 0;
  int off = lane * 16;
  u32x4 r[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    r[d] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kScanAux);
    off += 1024;
  }
  for (int s0 = 0; s0 < nsteps; s0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const u32x4 v = r[d] & 0x7fffffffu;
      m = max(m, max(max(v.x, v.y), max(v.z, v.w)));
      r[d] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kScanAux);
      off += 1024;
    }
  }
  return m;
}

// rows [c0, c1) of a window (n_t samples each): max |x| bit pattern over the wave
template <int D = kScanDepth>
__device__ __forceinline__ uint32_t scan_rows(const float* __restrict__ base, int64_t ch_stride, int c0, int c1,
                                              int n_t, bool vec, int lane) {
  uint32_t m = 0;
  if (vec && ch_stride == n_t) {  // the unit's rows are one contiguous span
    m = scan_span<D>(base + (int64_t)c0 * ch_stride, ((c1 - c0) * n_t) >> 2, lane);
  } else if (vec) {
    for (int c = c0; c < c1; ++c) m = max(m, scan_span<D>(base + (int64_t)c * ch_stride, n_t >> 2, lane));
  } else {
    for (int c = c0; c < c1; ++c)
      for (int t = lane; t < n_t; t += 64) m = max(m, absbits(base[(int64_t)c * ch_stride + t]));
  }
  return wave_max_u32(m);
}

struct ScanArgs {
  const int32_t* tab;  // nullptr: window s = pass s; else first record row of window s
  int32_t n_win;       // scan windows
  int32_t n_ch, n_t;   // rows and samples of one window
};

// ---- covered-span scan: the scan leaves out, per gather row, the float4s inside the row's correlated slices
// [a, a + (nwin - 1) hop + w) (both sides), which the correlation waves load and validate themselves (non-finite
// samples reach their spectra, or are checked where a sub-window is not transformed: FusedOps::check_untransformed).
// A row's remaining float4s are at most three spans; the wave streams them as one virtual index range, each lane's
// load address mapped past the skipped ranges (two compares), with kScanDepth loads in flight across row boundaries.
// Windows whose flag ends at 0 (nothing non-zero in the scanned part) or kSuspect are rescanned whole afterwards
// (window_fixup_kernel), so all-zero windows and non-finite spectra without a pass stay exact.
struct SpanRow {
  uint32_t base;  // byte offset of the row in the window (windows < 4 GiB)
  int U;         // float4s to scan
  int t0, d0;    // virtual index of the first skipped range, its length (float4)
  int s1, d1;    // start (real float4 index) and length of the second
};
// float4 range wholly inside side (a, L)'s correlated slices (empty when hop > w leaves gaps)
__device__ __forceinline__ void covered4(int a, int L, int w, int hop, int& b, int& e) {
  const int nw = n_subwin(L, w, hop);
  b = e = 0;
  if (nw <= 0 || hop > w) return;
  b = (a + 3) >> 2;
  e = (a + (nw - 1) * hop + w) >> 2;
  if (e < b) b = e = 0;
}
__device__ __forceinline__ SpanRow span_row(const VsgArgs& A, int p, int row0, int c, int n4) {
  SpanRow r;
  r.base = (uint32_t)((int64_t)c * A.ch_stride * 4);
  int b0 = 0, e0 = 0, b1 = 0, e1 = 0;
  const int i = c - row0;
  if (i >= 0 && i < A.R) {
    const int32_t* seg = A.seg_tab + ((int64_t)p * A.R + i) * 4;
    covered4(sld(seg), sld(seg + 1), A.w, A.hop, b0, e0);
    if (A.flags & kFlagOtherSide) covered4(sld(seg + 2), sld(seg + 3), A.w, A.hop, b1, e1);
  }
  if (e0 <= b0) b0 = e0 = n4;  // empty ranges sit past the row
  if (e1 <= b1) b1 = e1 = n4;
  if (b1 < b0) {  // ordered
    int t = b0; b0 = b1; b1 = t;
    t = e0; e0 = e1; e1 = t;
  }
  if (b1 < e0) {  // overlapping ranges merge
    e0 = max(e0, e1);
    b1 = e1 = n4;
  }
  e0 = min(e0, n4);
  e1 = min(e1, n4);
  r.t0 = b0;
  r.d0 = e0 - b0;
  r.s1 = b1;
  r.d1 = e1 - b1;
  r.U = n4 - r.d0 - r.d1;
  if (r.U == 0) r.U = 1;  // a wholly covered row reads one float4 again: no row is empty (one row switch per load)
  return r;
}
// rows [c0, c1) of pass p's window (n_t % 4 == 0, 16-byte aligned rows): max |x| bit pattern over the wave
// D: loads per lane in flight (the kernel's registers are sized for its correlation waves: EngF500's 128 VGPRs take
// 11, 12 spill)
template <int D>
__device__ __forceinline__ uint32_t scan_rows_span(const VsgArgs& A, const ScanArgs& S, int p, int c0, int c1, int lane) {
  const float* base = A.win + (int64_t)p * A.pass_stride;
  const int64_t wbytes = ((int64_t)(S.n_ch - 1) * A.ch_stride + S.n_t) * 4;  // < 0xfffffff0 (host)
  const __amdgpu_buffer_rsrc_t rs = scan_rsrc(base, (uint32_t)wbytes);
  const int row0 = sld(A.pass_tab + 2 * p), n4 = S.n_t >> 2;
  constexpr uint32_t kOut = 0xfffffff0u;  // past the descriptor's range: the load returns 0
  int c = c0, k = 0;
  SpanRow cur = span_row(A, p, row0, c, n4);
  auto issue = [&]() -> uint32_t {
    if (c < c1 && k * 64 >= cur.U) {  // next row (the loads in flight cover its table reads)
      ++c;
      k = 0;
      if (c < c1) cur = span_row(A, p, row0, c, n4);
    }
    if (c >= c1) return kOut;
    const int v = k * 64 + lane;
    ++k;
    int o = v + (v >= cur.t0 ? cur.d0 : 0);
    o += o >= cur.s1 ? cur.d1 : 0;
    return v < cur.U ? cur.base + (uint32_t)o * 16u : kOut;
  };
  uint32_t m = 0;
  u32x4 r[D];
#pragma unroll
  for (int d = 0; d < D; ++d) r[d] = __builtin_amdgcn_raw_buffer_load_b128(rs, issue(), 0, kScanAux);
  while (c < c1) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const u32x4 v = r[d] & 0x7fffffffu;
      m = max(m, max(max(v.x, v.y), max(v.z, v.w)));
      r[d] = __builtin_amdgcn_raw_buffer_load_b128(rs, issue(), 0, kScanAux);
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const u32x4 v = r[d] & 0x7fffffffu;
    m = max(m, max(max(v.x, v.y), max(v.z, v.w)));
  }
  return wave_max_u32(m);
}

// Windows the covered-span scan could not decide -- flag 0 (the scanned part all zero: the slices may not be) or
// kSuspect -- are rescanned whole: one block per window, nothing to do for the usual flag.
__global__ __launch_bounds__(256) void window_fixup_kernel(VsgArgs A, ScanArgs S, uint32_t* __restrict__ vflag) {
  const int s = blockIdx.x;
  const uint32_t f0 = vflag[s];
  if (f0 != 0 && !(f0 & kSuspect)) return;
  __shared__ uint32_t part[4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float* base = A.win + (int64_t)s * A.pass_stride;
  uint32_t m = 0;
  for (int c = wave; c < S.n_ch; c += 4)
    for (int t = lane; t < S.n_t; t += 64) m = max(m, absbits(base[(int64_t)c * A.ch_stride + t]));
  m = wave_max_u32(m);
  if (lane == 0) part[wave] = m;
  __syncthreads();
  if (threadIdx.x == 0) vflag[s] = max(max(part[0], part[1]), max(part[2], part[3]));
}

// Pull scan units (window, kScanRows channel rows) until none is left; atomicMax into vflag[window].  span: the
// covered-span scan (default windows of a launch whose chunks list every pass), DS loads per lane in flight.
template <int D = kScanDepth, int DS = 8>
__device__ __forceinline__ void scan_units(const VsgArgs& A, const ScanArgs& S, uint32_t* __restrict__ vflag,
                                           uint32_t* __restrict__ counter, int lane,
                                           const int32_t* __restrict__ sorder = nullptr, bool span = false) {
  const int upp = (S.n_ch + kScanRows - 1) / kScanRows;  // units per window
  const int n_units = S.n_win * upp;
  const bool vec = (S.n_t % 4 == 0) && (A.ch_stride % 4 == 0) && (A.pass_stride % 4 == 0) &&
                   (reinterpret_cast<uintptr_t>(A.win) % 16 == 0);
  int u = pull_unit(counter, lane);
  while (u < n_units) {
    const int un = pull_unit(counter, lane);  // the next unit's index, fetched under this unit's loads
    const int q = u / upp, c0 = (u - q * upp) * kScanRows;
    const int s = (sorder && !S.tab) ? sld(sorder + q) : q;
    const float* base = S.tab ? A.win + (int64_t)sld(S.tab + s) * A.ch_stride : A.win + (int64_t)s * A.pass_stride;
    const uint32_t m = span ? scan_rows_span<DS>(A, S, s, c0, min(c0 + kScanRows, S.n_ch), lane)
                            : scan_rows<D>(base, A.ch_stride, c0, min(c0 + kScanRows, S.n_ch), S.n_t, vec, lane);
    if (lane == 0) atomicMax(vflag + s, m);
    u = un;
  }
}

// correlation waves raise their issue priority while they correlate (scan waves stay at 0): the correlation is the
// critical path; 1 / 2 / 3 all measured 127.7 k -> 136 k windows/s on synth10k
constexpr int kCorrPrio = 2;

// The row tasks of a stack launch: frequency-domain stacking with the engine's exact (N = w) transforms, or
// with a zero-padded one (stackp_tasks).
template <class E, bool EXACT>
__device__ __forceinline__ void stack_tasks(E& eng, const VsgArgs& A, const float* __restrict__ scales,
                                            const int32_t* __restrict__ order, const int32_t* __restrict__ chunk_tab,
                                            int32_t n_chunk, const float* __restrict__ weight, float* __restrict__ stack,
                                            int64_t t0, TaskSource src) {
  if constexpr (EXACT) stackf_tasks<E>(eng, A, scales, order, chunk_tab, n_chunk, weight, stack, t0, src);
  else stackp_tasks<E>(eng, A, scales, order, chunk_tab, n_chunk, weight, stack, t0, src);
}

// Persistent validated stack launch: blocks of kFft correlation waves + kScan scan waves (EngF500: two per CU;
// the 1 024-point engines' LDS and registers allow one).
template <class E, int kFft, int kScan, int kOcc, bool EXACT = true, int kDepth = kScanDepth, int kSpanDepth = 8>
__global__ __launch_bounds__(64 * (kFft + kScan), kOcc) void vsg_stackv_kernel(
    VsgArgs A, const float* __restrict__ scales, const int32_t* __restrict__ order,
    const int32_t* __restrict__ chunk_tab, int32_t n_chunk, const float* __restrict__ weight,
    float* __restrict__ stack, ScanArgs S, uint32_t* __restrict__ vflag, uint32_t* __restrict__ counter,
    const float2* __restrict__ ptab, int32_t span_req) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  E eng = make_engine<E>(lds);
  bind_engine(eng, A, ptab);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // the chunks cover order[0, end of the last chunk): scan in that order when it lists every pass
  const int32_t* sorder = (n_chunk > 0 && sld(chunk_tab + 3 * (n_chunk - 1) + 1) == A.n_pass) ? order : nullptr;
  // covered-span scan (the host checked window layout and alignment): every pass's slices are loaded by the
  // correlation only when the chunks list every pass
  const bool span = Fused<E>::v && span_req && sorder && !S.tab;
  if constexpr (Fused<E>::v) {
    if (span) eng.vflag = vflag;
  }
  // the padded engines' correlation waves pull row tasks (w = 499: fused launch 4.80 -> 3.99 ms, their task costs vary
  // with the pivot-slice table's coverage); the exact ones keep the static stride (pulled, synth10k / weights measured
  // no better: balanced waves all join the scan at once)
  TaskSource src;
  src.stride = (int64_t)gridDim.x * kFft;
  if constexpr (!EXACT) src.q = counter + 1;
  if (wave < kFft) {
    __builtin_amdgcn_s_setprio(kCorrPrio);  // correlation waves issue first when both are ready
    stack_tasks<E, EXACT>(eng, A, scales, order, chunk_tab, n_chunk, weight, stack, (int64_t)xcd_block() * kFft + wave,
                          src);
    __builtin_amdgcn_s_setprio(0);
  }
  scan_units<kDepth, kSpanDepth>(A, S, vflag, counter, lane, sorder, span);
}

// The validity scan alone (correlation engines without a validated stack kernel).
__global__ __launch_bounds__(256) void window_scan_kernel(VsgArgs A, ScanArgs S, uint32_t* __restrict__ vflag,
                                                          uint32_t* __restrict__ counter) {
  scan_units(A, S, vflag, counter, threadIdx.x & 63);
}

// stack[slot] = NaN for every slot holding a pass whose window is invalid (vflag NaN / inf or 0).
// Block (slot, part): the slot's passes are found through chunk_tab; part j fills elements
// [j * 4096, (j + 1) * 4096) of the slot.
constexpr int kFillBlock = 256;
__global__ __launch_bounds__(kFillBlock) void vsg_invalid_fill_kernel(const int32_t* __restrict__ order,
                                                                      const int32_t* __restrict__ chunk_tab,
                                                                      int32_t n_chunk, const uint32_t* __restrict__ vflag,
                                                                      const int32_t* __restrict__ unit_scan,
                                                                      float* __restrict__ stack, int64_t slot_elems) {
  const int slot = blockIdx.y;
  int bad = 0;
  for (int c = threadIdx.x; c < n_chunk; c += kFillBlock) {
    if (chunk_tab[3 * c + 2] != slot) continue;
    for (int q = chunk_tab[3 * c]; q < chunk_tab[3 * c + 1]; ++q) {
      const int p = order[q];
      const uint32_t f = vflag[unit_scan ? unit_scan[p] : p];
      bad |= (f >= 0x7f800000u) || (f == 0u);
    }
  }
  if (!__syncthreads_or(bad)) return;
  float* o = stack + (int64_t)slot * slot_elems;
  const int64_t e0 = (int64_t)blockIdx.x * 4096;
  for (int64_t k = e0 + threadIdx.x; k < min(e0 + 4096, slot_elems); k += kFillBlock) o[k] = NAN;
}

// Sum of squares of each pass window (np.linalg.norm(window.data) ** 2), for norm=norm_amp=False.
// One block per pass; wave k takes rows k, k + 8, ...; 16-byte loads, 4 in flight per lane, fp64
// accumulation in a fixed order (deterministic run to run).
constexpr int kSumWaves = kBlock / 64;
__global__ __launch_bounds__(kBlock) void window_sumsq_kernel(const float* __restrict__ win, int64_t pass_stride,
                                                               int64_t ch_stride, int32_t n_ch, int32_t n_t,
                                                               double* __restrict__ out) {
  __shared__ double part[kSumWaves];
  const int p = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* base = win + (int64_t)p * pass_stride;
  const bool vec = (n_t % 4 == 0) && (ch_stride % 4 == 0) && (pass_stride % 4 == 0) &&
                   (reinterpret_cast<uintptr_t>(win) % 16 == 0);
  double s0 = 0.0, s1 = 0.0;
  for (int c = wave; c < n_ch; c += kSumWaves) {
    const float* row = base + (int64_t)c * ch_stride;
    if (vec) {
      const float4* r4 = reinterpret_cast<const float4*>(row);
      const int n4 = n_t / 4;
      int t = lane;
      for (; t + 192 < n4; t += 256) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = r4[t + 64 * u];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          s0 += (double)v[u].x * v[u].x + (double)v[u].y * v[u].y;
          s1 += (double)v[u].z * v[u].z + (double)v[u].w * v[u].w;
        }
      }
      for (; t < n4; t += 64) {
        const float4 v = r4[t];
        s0 += (double)v.x * v.x + (double)v.y * v.y;
        s1 += (double)v.z * v.z + (double)v.w * v.w;
      }
    } else {
      for (int t = lane; t < n_t; t += 64) {
        const double v = row[t];
        s0 += v * v;
      }
    }
  }
  double s = s0 + s1;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) part[wave] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < kSumWaves; ++k) t += part[k];
    out[p] = t;
  }
}

struct VsgKernels {
  const void* scales;
  const void* gather;
  const void* stack;
  size_t lds;
  int waves;
};

template <class E, bool EXACT>
VsgKernels vsg_kernels() {
  const void* st;
  if constexpr (EXACT) st = (const void*)vsg_stackf_kernel<E>;
  else st = (const void*)vsg_stackp_kernel<E>;
  return VsgKernels{(const void*)vsg_scales_kernel<E>, (const void*)vsg_gather_kernel<E>, st,
                    E::kBlockBytes + E::kWaves * E::kWaveBytes, E::kWaves};
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
    case 250: *k = vsg_kernels<EngStockham<250, false>, true>(); return true;
    case 500: *k = vsg_kernels<EngF500, true>(); return true;  // fused-stage Stockham
    case 1000: *k = vsg_kernels<EngStockham<1000, false>, true>(); return true;
    case 512: *k = vsg_kernels<EngStockham<512, true>, false>(); return true;
    case 1024: *k = vsg_kernels<EngP1024, false>(); return true;  // fused-stage padded Stockham
    case 2048: *k = vsg_kernels<EngStockham<2048, true>, false>(); return true;
    default: return false;
  }
}

static int check_common(const VsgArgs& A) {
  if (!A.win || !A.pass_tab || !A.seg_tab) return set_error(-2, "null pointer argument");
  if (A.n_pass < 0 || A.R <= 0 || A.w < 2 || A.hop < 1) return set_error(-2, "invalid geometry (R, w, hop)");
  return 0;
}

static int launch(const void* fn, int grid, int waves, size_t lds, void** args, hipStream_t s) {
  if (grid <= 0) return 0;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return set_error(-3, hipGetErrorString(e));
  e = hipLaunchKernel(fn, dim3(grid), dim3(64 * waves), args, lds, s);
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
  return launch(k.scales, (n_pass + k.waves - 1) / k.waves, k.waves, k.lds, args, (hipStream_t)stream);
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
  const int64_t grid = (tasks + k.waves - 1) / k.waves;
  void* args[] = {&A, &scales, &out};
  return launch(k.gather, (int)(grid > (1 << 30) ? (1 << 30) : grid), k.waves, k.lds, args, (hipStream_t)stream);
}

// Validated launch shapes.  EngF500: blocks of 7 correlation + 1 scan waves, 2 blocks per CU (4 waves per SIMD, the
// registers sized for it by the launch bounds).  EngP1024: 7 + 1 waves, one block per CU (LDS, registers), its scan
// waves keeping 32 loads per lane in flight (w = 499 synth10k launch 14.70 vs 15.08 ms at 16, 14.92 at 48).
constexpr int kVsFft = 7, kVsScan = 1, kVsBpc = 2, kVsOcc = 4;
constexpr int kVsSpan = 11;  // the covered-span scan's loads per lane in flight in the EngF500 launch: the most without
                             // spills (12 spill; 11 vs 8: synth10k 13.06 vs 13.09-13.13 ms, profiles/r6_ab)
constexpr int kP1Fft = 7, kP1Scan = 1, kP1Depth = 32;

// The fused (correlation + validity scan) launch of each transform length: kernel, correlation / scan waves per
// block, blocks per CU, LDS per block.
struct VStack {
  const void* fn;
  int fft, scan, bpc;
  size_t lds;
};
template <class E, int F, int SC, int OCC, bool EXACT, int DEPTH = kScanDepth, int SPAN = 8>
static VStack vstack(int bpc) {
  return VStack{(const void*)vsg_stackv_kernel<E, F, SC, OCC, EXACT, DEPTH, SPAN>, F, SC, bpc,
                E::kBlockBytes + F * E::kWaveBytes};
}
static bool get_vstack(int n, VStack* v) {
  switch (n) {
    case 500: *v = vstack<EngF500, kVsFft, kVsScan, kVsOcc, true, kScanDepth, kVsSpan>(kVsBpc); return true;
    case 512: *v = vstack<EngStockham<512, true>, 7, 1, 2, false>(1); return true;
    case 1024: *v = vstack<EngP1024, kP1Fft, kP1Scan, 2, false, kP1Depth>(1); return true;
    default: return false;
  }
}

// Transform lengths whose engine takes the pivot-slice table: 500 (EngF500) and the padded 1 024 (EngP1024).
static bool table_engine(int n) { return n == 500 || n == 1024; }

template <class E>
static int64_t table_bytes(int64_t n_pass) {
  return n_pass * (tab_pass_f2<E::kTabBins>() * (int64_t)sizeof(float2) + 2 * kTabEnt * (int64_t)sizeof(int32_t));
}
static int64_t stack_ws_bytes(int n, int64_t n_pass) {
  return n == 500 ? table_bytes<EngF500>(n_pass) : table_bytes<EngP1024>(n_pass);
}

static int launch_table(VsgArgs& A, int n, float2* tab, hipStream_t s) {
  const int grid = (int)std::min<int64_t>(((int64_t)A.n_pass + 3) / 4, 8 * (int64_t)cu_count());
  void* args[] = {&A, &tab};
  // the engine's block tables + 4 waves' buffers (EngP1024's padded buffer A and stage tables included)
  if (n == 500)
    return launch((const void*)vsg_pivot_table_kernel<EngF500>, grid, 4, EngF500::kBlockBytes + 4 * EngF500::kWaveBytes,
                  args, s);
  return launch((const void*)vsg_pivot_table_kernel<EngP1024>, grid, 4, EngP1024::kBlockBytes + 4 * EngP1024::kWaveBytes,
                args, s);
}

DVH_API int64_t dvh_vsg_stack_workspace(int32_t n_pass, int32_t w) {
  bool pad;
  const int n = choose_fft(w, &pad);
  if (n_pass <= 0 || !table_engine(n)) return 0;
  return stack_ws_bytes(n, n_pass);
}

DVH_API int dvh_vsg_stack_validated(const float* win, int64_t pass_stride, int64_t ch_stride, int32_t n_pass,
                                    int32_t n_ch, int32_t n_t, const int32_t* pass_tab, const int32_t* seg_tab, int32_t R,
                                    int32_t w, int32_t hop, int32_t flags, const float* scales, const int32_t* order,
                                    const int32_t* chunk_tab, int32_t n_chunk, int32_t n_slot, const float* weight,
                                    float* stack, const int32_t* scan_tab, int32_t n_scan, const int32_t* unit_scan,
                                    uint32_t* work, void* spec_ws, void* stream) {
  VsgArgs A{win, pass_stride, ch_stride, pass_tab, seg_tab, n_pass, R, w, hop, flags};
  if (int rc = check_common(A)) return rc;
  if (!scales || !order || !chunk_tab || !weight || !stack || !work) return set_error(-2, "null pointer argument");
  if (!(flags & (kFlagNorm | kFlagNormAmp)))
    return set_error(-2, "validated stacking needs norm or norm_amp (raw scales need ||data||_F: dvh_window_sumsq)");
  if (n_ch < R || n_t <= 0) return set_error(-2, "window smaller than the gather");
  if ((scan_tab == nullptr) != (unit_scan == nullptr)) return set_error(-2, "scan_tab and unit_scan go together");
  if (scan_tab && n_scan <= 0) return set_error(-2, "a scan table needs n_scan > 0");
  VsgKernels k;
  int n;
  if (!get_kernels(w, &k, &n)) return set_error(-4, "unsupported correlation window length");
  const ScanArgs S{scan_tab, scan_tab ? n_scan : n_pass, n_ch, n_t};
  hipStream_t s = (hipStream_t)stream;
  uint32_t* vflag = work;
  uint32_t* counter = work + S.n_win;
  float2* tab = (table_engine(n) && spec_ws) ? reinterpret_cast<float2*>(spec_ws) : nullptr;
  hipError_t e = hipMemsetAsync(work, 0, sizeof(uint32_t) * ((size_t)S.n_win + 2), s);
  if (e != hipSuccess) return set_error(-3, hipGetErrorString(e));
  // the covered-span scan: w = 500's fused engine, default windows, 16-byte aligned rows (the kernel also needs the
  // chunks to list every pass, and falls back to the whole-window scan otherwise).  synth10k launch 13.27-13.28 ->
  // 13.06-13.13 ms, weights 1.304-1.312 -> 1.263-1.289 ms; on the padded engine it lost (w = 499 synth10k 14.8-15.0
  // -> 16.3-17.1 ms at 8 or 16 loads per lane in flight against the whole-window scan's 32).  DVH_SCAN_SPAN=0: off.
  static const int span_env = getenv("DVH_SCAN_SPAN") ? atoi(getenv("DVH_SCAN_SPAN")) : 1;
  int32_t span = (span_env && n == 500 && !scan_tab && n_t % 4 == 0 && ch_stride % 4 == 0 && pass_stride % 4 == 0 &&
                  reinterpret_cast<uintptr_t>(win) % 16 == 0 &&
                  ((int64_t)(n_ch - 1) * ch_stride + n_t) * 4 < 0xfffffff0LL) ? 1 : 0;
  if (tab)
    if (int rc = launch_table(A, n, tab, s)) return rc;
  const int64_t tasks = (int64_t)n_chunk * R;
  VStack v{};
  if (get_vstack(n, &v)) {
    const int64_t need = (tasks + v.fft - 1) / v.fft;
    const int grid = (int)(need < v.bpc * cu_count() ? (need > 0 ? need : 1) : v.bpc * cu_count());
    void* args[] = {&A, &scales, &order, &chunk_tab, &n_chunk, &weight, &stack, (void*)&S, &vflag, &counter, &tab, &span};
    if (int rc = launch(v.fn, grid, v.fft + v.scan, v.lds, args, s)) return rc;
    if (span && S.n_win > 0) {  // the windows the covered-span scan could not decide, rescanned whole
      hipLaunchKernelGGL(window_fixup_kernel, dim3((unsigned)S.n_win), dim3(256), 0, s, A, S, vflag);
      if ((e = hipGetLastError()) != hipSuccess) return set_error(-3, hipGetErrorString(e));
    }
  } else {  // no fused form: the scan as its own launch, then the plain stack launch
    void* sargs[] = {&A, (void*)&S, &vflag, &counter};
    if (int rc = launch((const void*)window_scan_kernel, 4 * cu_count(), 4, 0, sargs, s)) return rc;
    const int64_t grid = (tasks + k.waves - 1) / k.waves;
    void* args[] = {&A, &scales, &order, &chunk_tab, &n_chunk, &weight, &stack, &tab};
    if (int rc = launch(k.stack, (int)(grid > (1 << 30) ? (1 << 30) : grid), k.waves, k.lds, args, s)) return rc;
  }
  if (n_slot <= 0 || n_chunk <= 0) return 0;
  const int64_t slot_elems = (int64_t)R * w;
  hipLaunchKernelGGL(vsg_invalid_fill_kernel, dim3((unsigned)((slot_elems + 4095) / 4096), n_slot), dim3(kFillBlock), 0,
                     s, order, chunk_tab, n_chunk, (const uint32_t*)vflag, unit_scan, stack, slot_elems);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : set_error(-3, hipGetErrorString(e));
}

DVH_API int dvh_vsg_stack(const float* win, int64_t pass_stride, int64_t ch_stride, int32_t n_pass,
                          const int32_t* pass_tab, const int32_t* seg_tab, int32_t R, int32_t w, int32_t hop,
                          int32_t flags, const float* scales, const int32_t* order, const int32_t* chunk_tab,
                          int32_t n_chunk, const float* weight, float* stack, void* spec_ws, void* stream) {
  VsgArgs A{win, pass_stride, ch_stride, pass_tab, seg_tab, n_pass, R, w, hop, flags};
  if (int rc = check_common(A)) return rc;
  if (!scales || !order || !chunk_tab || !weight || !stack) return set_error(-2, "null pointer argument");
  VsgKernels k;
  int n;
  if (!get_kernels(w, &k, &n)) return set_error(-4, "unsupported correlation window length");
  const int64_t tasks = (int64_t)n_chunk * R;
  hipStream_t s = (hipStream_t)stream;
  float2* tab = (table_engine(n) && spec_ws) ? reinterpret_cast<float2*>(spec_ws) : nullptr;
  if (tab)
    if (int rc = launch_table(A, n, tab, s)) return rc;
  const int64_t grid = (tasks + k.waves - 1) / k.waves;
  void* args[] = {&A, &scales, &order, &chunk_tab, &n_chunk, &weight, &stack, &tab};
  return launch(k.stack, (int)(grid > (1 << 30) ? (1 << 30) : grid), k.waves, k.lds, args, s);
}
