// Per-wave correlation engines of the VSG kernels (gfx950).
//
// An engine turns one gather row task (pass p, row i) into the raw circular correlations of both
// sides, c_f[k] and c_o[k] (k < w), summed over the row's sub-windows and scaled by N * nwin:
//   for every sub-window, z = pivot + i * receiver -> one complex FFT -> cross spectrum
//   P conj(R) = (i/4)(Z[f] + conj Z[-f]) conj(Z[f] - conj Z[-f]) accumulated per side in registers,
//   then ONE inverse FFT of Cf + i Co (real part -> forward side, imaginary -> other side).
// The cross spectra of real correlations are Hermitian, so only bins f <= N/2 are accumulated
// (NH per lane, f = lane + 64 j); the inverse writes both W[f] and W[N - f].
// A sub-window whose pivot or receiver slice is identically zero contributes exactly zero in the
// reference; the engines test every loaded sample (bit pattern, so NaN counts as non-zero) and skip
// such sub-windows, and report per side whether anything was accumulated (live_f / live_o), so that
// an all-zero side is exactly zero (and yields the reference's 0/0 = NaN where it normalises).
//
//   EngStockham<N, PAD>  any supported N: LDS ping-pong Stockham transform (fft_wave.h), sub-window
//                        loads staged in registers one sub-window ahead.  PAD: N >= 2w - 1 zero padded,
//                        linear correlation folded back to circular in c().
//   EngF500              N = w = 500 (wlen = 2 s at 250 Hz, the reference's operating point): the
//                        4 x 5 x 5 x 5 Stockham transform with its first and last stages in registers.
// (Engine variants measured and not kept -- 20 x 25 register transform, paired in-place 20 x 5 x 5,
// register twiddles -- are kept for reference in tools/variants/vsg_engine_variants.h.)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fft_wave.h"
#include "tw_tables.h"

#ifndef DVH_RCV_AHEAD
#define DVH_RCV_AHEAD 1  // sub-windows of receiver samples EngF500 keeps in flight (1 or 2)
#endif

namespace dvh {

#ifndef DVH_XPASS_PF
#define DVH_XPASS_PF 0  // EngF500: prefetch the next task's first sub-window during the last transform of a call
#endif
#ifndef DVH_RCV_NT
#define DVH_RCV_NT 0  // 1: receiver samples (read once per (pass, row)) loaded non-temporal, sparing the L2 lines
                      // of the pivot channel every row of a chunk re-reads
#endif
__device__ __forceinline__ float rcv_load(const float* p) {
#if DVH_RCV_NT
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}

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
__device__ __forceinline__ float unif(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

// Everything a row task needs, wave-uniform.
struct RowTask {
  const float* piv;
  const float* rcv;
  int a_f, nwin_f, a_o, nwin_o;
  int ch, pivot;
  int p, row0;
};

__device__ __forceinline__ RowTask make_task(const VsgArgs& A, int p, int i) {
  p = uni(p);
  i = uni(i);
  RowTask t;
  const int row0 = uni(A.pass_tab[2 * p]);
  t.p = p;
  t.row0 = row0;
  t.pivot = uni(A.pass_tab[2 * p + 1]);
  t.ch = row0 + i;
  const float* base = A.win + (int64_t)p * A.pass_stride;
  t.piv = base + (int64_t)t.pivot * A.ch_stride;
  t.rcv = base + (int64_t)t.ch * A.ch_stride;
  const int32_t* seg = A.seg_tab + ((int64_t)p * A.R + i) * 4;
  t.a_f = uni(seg[0]);
  t.nwin_f = n_subwin(uni(seg[1]), A.w, A.hop);
  const bool other = (A.flags & kFlagOtherSide) != 0;
  t.a_o = uni(seg[2]);
  t.nwin_o = other ? n_subwin(uni(seg[3]), A.w, A.hop) : 0;
  return t;
}

// |x| != 0 as a bit mask (NaN included); OR-accumulate, test once per sub-window
__device__ __forceinline__ uint32_t nzbits(float x) { return __builtin_bit_cast(uint32_t, x) & 0x7fffffffu; }

__device__ __forceinline__ void accumulate_cross(float2 Az, float2 Bc, float2& C) {
  // P = (A + B) / 2, R = (A - B) / 2i with B = conj(Bc)  ->  P conj(R) = (i / 4) (A + B) conj(A - B)
  const float bx = Bc.x, by = -Bc.y;
  C.x += 0.5f * (bx * Az.y - by * Az.x);
  C.y += 0.25f * ((Az.x * Az.x + Az.y * Az.y) - (bx * bx + by * by));
}

// conj(W) for W = Cf + i Co over all N bins from the half spectra held in the engine's slots
// (slot j of a lane is bin E::bin(lane, j) <= N/2, or -1): the input of the inverse transform
// conj(FFT(conj(W))).  W[N - f] = conj(Cf[f]) + i conj(Co[f]).
template <class E>
__device__ __forceinline__ void store_conj_hermitian(float2* buf, const float2 (&Cf)[E::NH], const float2 (&Co)[E::NH],
                                                     int lane) {
  constexpr int N = E::NFFT;
#pragma unroll
  for (int j = 0; j < E::NH; ++j) {
    const int f = E::bin(lane, j);
    if (f >= 0) {
      buf[E::slot(f)] = make_float2(Cf[j].x - Co[j].y, -(Cf[j].y + Co[j].x));
      if (f > 0 && f < N / 2) buf[E::slot(N - f)] = make_float2(Cf[j].x + Co[j].y, Cf[j].y - Co[j].x);
    }
  }
}

// ------------------------------------------------------------------------------------------------
template <int N, bool PAD>
struct EngStockham {
  static constexpr int NFFT = N;
  static constexpr int kWaves = 4;
  static constexpr bool kNextTask = false;
  static constexpr int NJ = (N + 63) / 64;
  static constexpr int NH = (N / 2 + 1 + 63) / 64;
  static_assert(N % 2 == 0, "Hermitian half spectra assume an even length");
  static constexpr size_t kBlockBytes = sizeof(float2) * N;        // twiddle table
  static constexpr size_t kWaveBytes = sizeof(float2) * 2 * N;     // ping-pong buffers
  float2* tw;
  float2* bufA;
  float2* bufB;
  int lane;
  bool live_f, live_o;  // some sub-window of the side had non-zero pivot and receiver slices
  uint32_t rmax;        // this lane's max |receiver sample| bit pattern over the last spectra() call

  __device__ EngStockham(char* lds, int wave, int lane_) : lane(lane_), live_f(false), live_o(false), rmax(0) {
    tw = reinterpret_cast<float2*>(lds);
    bufA = reinterpret_cast<float2*>(lds + kBlockBytes + (size_t)wave * kWaveBytes);
    bufB = bufA + N;
  }
  static __device__ void block_init(char* lds) { init_twiddles<N>(reinterpret_cast<float2*>(lds)); }

  __device__ void load(const RowTask& t, int a, int w, float2 (&z)[NJ]) const {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = lane + 64 * j;
      z[j] = (n < w) ? make_float2(t.piv[a + n], t.rcv[a + n]) : make_float2(0.f, 0.f);
    }
  }

  // accumulated cross spectra of both sides: Cf[j], Co[j] at bins f = lane + 64 j
  __device__ void spectra(const RowTask& t, const RowTask&, bool, int w, int hop, float2 (&Cf)[NH],
                          float2 (&Co)[NH]) {
    const int nq = t.nwin_f + t.nwin_o;
    float2 z[NJ];
#pragma unroll
    for (int j = 0; j < NH; ++j) {
      Cf[j] = make_float2(0.f, 0.f);
      Co[j] = make_float2(0.f, 0.f);
    }
    live_f = live_o = false;
    rmax = 0;
    if (nq > 0) load(t, t.nwin_f > 0 ? t.a_f : t.a_o, w, z);
    for (int q = 0; q < nq; ++q) {
      uint32_t bp = 0, br = 0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = lane + 64 * j;
        if (n < N) bufA[n] = z[j];
        bp |= nzbits(z[j].x);
        br |= nzbits(z[j].y);
        rmax = max(rmax, nzbits(z[j].y));
      }
      const bool live = (__ballot(bp != 0) != 0) && (__ballot(br != 0) != 0);
      if (q + 1 < nq) {
        const int qn = q + 1;
        load(t, qn < t.nwin_f ? t.a_f + qn * hop : t.a_o + (qn - t.nwin_f) * hop, w, z);
      }
      if (!live) continue;  // exactly zero in the reference
      if (q < t.nwin_f) live_f = true;
      else live_o = true;
      wave_sync();
      const float2* X = FftPlan<N>::T::run(bufA, bufB, tw, lane);
      if (q < t.nwin_f) {
#pragma unroll
        for (int j = 0; j < NH; ++j) {
          const int f = lane + 64 * j;
          if (f <= N / 2) accumulate_cross(X[f], X[f == 0 ? 0 : N - f], Cf[j]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < NH; ++j) {
          const int f = lane + 64 * j;
          if (f <= N / 2) accumulate_cross(X[f], X[f == 0 ? 0 : N - f], Co[j]);
        }
      }
      wave_sync();
    }
  }

  // Y with Y[k].x = N * IDFT(Cf)[k], -Y[k].y = N * IDFT(Co)[k] (read through c())
  // half-spectrum slot j of a lane holds bin f = lane + 64 j (f <= N/2)
  static __device__ __forceinline__ int bin(int lane, int j) {
    const int f = lane + 64 * j;
    return f <= N / 2 ? f : -1;
  }
  static __device__ __forceinline__ int slot(int n) { return n; }

  __device__ const float2* inverse(const float2 (&Cf)[NH], const float2 (&Co)[NH]) {
    store_conj_hermitian<EngStockham>(bufA, Cf, Co, lane);
    wave_sync();
    return FftPlan<N>::T::run(bufA, bufB, tw, lane);
  }

  __device__ const float2* correlate(const RowTask& t, const RowTask& nt, bool has_next, int w, int hop) {
    float2 Cf[NH], Co[NH];
    spectra(t, nt, has_next, w, hop, Cf, Co);
    return inverse(Cf, Co);
  }

  // twiddle exp(-2 pi i m / N), m in [0, N)
  __device__ float2 twiddle(int m) const { return tw[m]; }

  // (N * sum_s c_f[k], N * sum_s c_o[k])
  __device__ float2 c(const float2* Y, int k, int w) const {
    float2 v = Y[k];
    if (PAD && k > 0) {
      const float2 u = Y[N - w + k];
      v.x += u.x;
      v.y += u.y;
    }
    return make_float2(v.x, -v.y);
  }
};

// ------------------------------------------------------------------------------------------------
// EngF500: N = w = 500 Stockham (4 x 5 x 5 x 5) with the first and last stages fused into registers.
//   stage 1 (radix 4, span 1) reads its inputs straight from the prefetched sub-window samples
//     (lane i < 125 of round r holds samples i + 125 t) -- no LDS store of the raw window;
//   stages 2-3 go through LDS (one twiddle read per butterfly, powers by recurrence);
//   stage 4 (radix 5, span 100) runs butterflies k and 100 - k in the same lane (l <= 50), so the
//     lane holds X[k + 100 q] and its Hermitian partners X[N - f] and forms the cross spectra of its
//     five bins in registers -- no LDS write of the spectrum and no partner reads.
// Half-spectrum slots per lane l: j < 3 -> f = l + 100 j (l <= 50); j = 3, 4 -> f = 100 - l + 100 (j - 3)
// (1 <= l <= 49): each of the 251 bins f <= 250 exactly once.
struct EngF500 {
  static constexpr int N = 500;
  static constexpr int NFFT = 500;
  static constexpr int NJ = 8;
  static constexpr int NH = 5;
  static constexpr int kWaves = 4;
  static constexpr bool kNextTask = DVH_XPASS_PF != 0;  // the cross-pass prefetch variant takes the next task
  static constexpr size_t kBlockBytes = sizeof(float2) * N;     // twiddle table
  static constexpr size_t kWaveBytes = sizeof(float2) * 2 * N;  // ping-pong buffers
  float2* tw;
  float2* bufA;
  float2* bufB;
  int lane;
  bool live_f, live_o;
  uint32_t rmax;  // this lane's max |receiver sample| bit pattern over the last spectra() call

  __device__ EngF500(char* lds, int wave, int lane_) : lane(lane_), live_f(false), live_o(false), rmax(0) {
    tw = reinterpret_cast<float2*>(lds);
    bufA = reinterpret_cast<float2*>(lds + kBlockBytes + (size_t)wave * kWaveBytes);
    bufB = bufA + N;
  }
  static __device__ void block_init(char* lds) { init_twiddles<N>(reinterpret_cast<float2*>(lds)); }

  static __device__ __forceinline__ int bin(int l, int j) {
    if (j < 3) return l <= 50 ? l + 100 * j : -1;
    return (l >= 1 && l <= 49) ? 100 - l + 100 * (j - 3) : -1;
  }
  static __device__ __forceinline__ int slot(int n) { return n; }

  // stage-1 operands of a sub-window starting at a: z[4 r + t] = (pivot, receiver)[i + 125 t], i = lane + 64 r
  __device__ __forceinline__ void load(const RowTask& t, int a, float2 (&z)[8]) const {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = lane + 64 * r;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int n = a + i + 125 * u;
        z[4 * r + u] = (i < 125) ? make_float2(t.piv[n], rcv_load(t.rcv + n)) : make_float2(0.f, 0.f);
      }
    }
  }

  __device__ __forceinline__ void stage1(const float2 (&z)[8]) const {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = lane + 64 * r;
      if (r == 0 || i < 125) {
        float2 a[4] = {z[4 * r], z[4 * r + 1], z[4 * r + 2], z[4 * r + 3]};
        Dft<4>::run(a);
#pragma unroll
        for (int q = 0; q < 4; ++q) bufB[4 * i + q] = a[q];
      }
    }
  }

  // stages 2-4 of the transform whose stage-1 output is in bufB; cross spectra into C
  __device__ __forceinline__ void finish(float2 (&C)[NH]) const {
    finish_with([&](int j, float2 a, float2 b) { accumulate_cross(a, b, C[j]); });
  }

  // stages 2-4 of the transform whose stage-1 output is in bufB; for every half-spectrum slot j of
  // the lane (compile-time j, valid slots only), acc(j, Z[f], Z[N - f]) with f = bin(lane, j)
  template <class F>
  __device__ __forceinline__ void finish_with(F&& acc) const {
    wave_sync();
    stockham_stage<N, 4, 5>(bufB, bufA, tw, lane);
    wave_sync();
    stockham_stage<N, 20, 5>(bufA, bufB, tw, lane);
    wave_sync();
    if (lane <= 50) {
      float2 XA[5], XB[5];
      const bool pair = lane >= 1 && lane <= 49;
      last_bfly_from(bufB, lane, XA);
      if (pair) last_bfly_from(bufB, 100 - lane, XB);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        // partner X[N - f] of f = l + 100 j is X[(100 - l) + 100 (4 - j)]
        const float2 p0 = XA[(5 - j) % 5], p50 = XA[4 - j], pb = XB[4 - j];
        float2 pa;  // value selects (a select of array elements would become a scratch pointer)
        pa.x = lane == 0 ? p0.x : (lane == 50 ? p50.x : pb.x);
        pa.y = lane == 0 ? p0.y : (lane == 50 ? p50.y : pb.y);
        acc(j, XA[j], pa);
      }
      if (pair) {
#pragma unroll
        for (int q = 0; q < 2; ++q) acc(3 + q, XB[q], XA[4 - q]);
      }
    }
    wave_sync();
  }

  // radix-5 butterfly k of the last stage (span 100): X[k + 100 q], q < 5
  __device__ __forceinline__ void last_bfly_from(const float2* src, int k, float2 (&x)[5]) const {
#pragma unroll
    for (int t = 0; t < 5; ++t) x[t] = lds_ld(src, k + 100 * t);
#if DVH_TW_RECUR
    const float2 w1 = tw[k];
    float2 wt = w1;
#pragma unroll
    for (int t = 1; t < 5; ++t) {
      x[t] = cmul(x[t], wt);
      if (t < 4) wt = cmul(wt, w1);
    }
#else
#pragma unroll
    for (int t = 1; t < 5; ++t) x[t] = cmul(x[t], tw[t * k]);
#endif
    Dft<5>::run(x);
  }

  // receiver samples of the sub-window starting at a, in load()'s lane layout
  __device__ __forceinline__ void load_rcv(const RowTask& t, int a, float (&zr)[8]) const {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = lane + 64 * r;
#pragma unroll
      for (int u = 0; u < 4; ++u) zr[4 * r + u] = (i < 125) ? t.rcv[a + i + 125 * u] : 0.f;
    }
  }
  __device__ __forceinline__ void load_piv(const RowTask& t, int a, float2 (&z)[8]) const {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = lane + 64 * r;
#pragma unroll
      for (int u = 0; u < 4; ++u) z[4 * r + u].x = (i < 125) ? t.piv[a + i + 125 * u] : 0.f;
    }
  }

  // Sub-window q's pivot and receiver samples are loaded one sub-window ahead; with
  // DVH_RCV_AHEAD == 2 the receiver samples (the HBM-missing stream: pivot slices are shared by the
  // chunk's rows and mostly hit L2) two sub-windows ahead, for more latency tolerance when the
  // launch also streams whole windows (vsg_stackv_kernel).  With DVH_XPASS_PF the last sub-window of a
  // call loads the FIRST sub-window of the caller's next task (tn) into zc, so the first transform of
  // every pass is prefetched too; a call whose task is not the one prefetched loads its own.
  float2 zc[8];
  const float* pre_rcv = nullptr;
  int pre_a = -1;
  __device__ void spectra(const RowTask& t, const RowTask& tn, bool has_next, int, int hop, float2 (&Cf)[NH],
                          float2 (&Co)[NH]) {
    const int nq = t.nwin_f + t.nwin_o;
#pragma unroll
    for (int j = 0; j < NH; ++j) {
      Cf[j] = make_float2(0.f, 0.f);
      Co[j] = make_float2(0.f, 0.f);
    }
    live_f = live_o = false;
    auto start = [&](int q) { return q < t.nwin_f ? t.a_f + q * hop : t.a_o + (q - t.nwin_f) * hop; };
#if DVH_XPASS_PF
    const int nqn = has_next ? tn.nwin_f + tn.nwin_o : 0;
    const int an = tn.nwin_f > 0 ? tn.a_f : tn.a_o;
    if (nq > 0 && !(pre_rcv == t.rcv && pre_a == start(0))) load(t, start(0), zc);
    pre_rcv = nullptr;
#else
    if (nq > 0) load(t, start(0), zc);
#endif
    float2 (&z)[8] = zc;
#if DVH_RCV_AHEAD == 2
    float zr[8];
    if (nq > 1) load_rcv(t, start(1), zr);
#endif
    rmax = 0;
    for (int q = 0; q < nq; ++q) {
      uint32_t bp = 0, br = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bp |= nzbits(z[j].x);
        br |= nzbits(z[j].y);
        rmax = max(rmax, nzbits(z[j].y));
      }
      const bool live = (__ballot(bp != 0) != 0) && (__ballot(br != 0) != 0);
      if (live) stage1(z);
      if (q + 1 < nq) {
#if DVH_RCV_AHEAD == 2
        load_piv(t, start(q + 1), z);
#pragma unroll
        for (int j = 0; j < 8; ++j) z[j].y = zr[j];
        if (q + 2 < nq) load_rcv(t, start(q + 2), zr);
#else
        load(t, start(q + 1), z);
#endif
      }
#if DVH_XPASS_PF
      else if (nqn > 0) {  // the next task's first sub-window, under this one's stages 2-4
        load(tn, an, z);
        pre_rcv = tn.rcv;
        pre_a = an;
      }
#endif
      if (!live) continue;  // exactly zero in the reference
      if (q < t.nwin_f) {
        live_f = true;
        finish(Cf);
      } else {
        live_o = true;
        finish(Co);
      }
    }
#if DVH_XPASS_PF
    if (nq == 0 && nqn > 0) {
      load(tn, an, z);
      pre_rcv = tn.rcv;
      pre_a = an;
    }
#endif
  }

  __device__ const float2* inverse(const float2 (&Cf)[NH], const float2 (&Co)[NH]) {
    store_conj_hermitian<EngF500>(bufA, Cf, Co, lane);
    wave_sync();
    return FftPlan<N>::T::run(bufA, bufB, tw, lane);
  }

  __device__ const float2* correlate(const RowTask& t, const RowTask& nt, bool has_next, int w, int hop) {
    float2 Cf[NH], Co[NH];
    spectra(t, nt, has_next, w, hop, Cf, Co);
    return inverse(Cf, Co);
  }

  __device__ float2 twiddle(int m) const { return tw[m]; }

  __device__ float2 c(const float2* Y, int k, int) const {
    const float2 v = Y[k];
    return make_float2(v.x, -v.y);
  }
};


}  // namespace dvh
