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
//   EngP1024             w <= 512 without an exact engine (w = 499): zero-padded 4^5 transform, first and
//                        last stages in registers, as EngF500 (pivot-slice table, cross-pass packing).
// (Engine variants measured and not kept are listed in DESIGN.md.)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fft_wave.h"
#include "tw_tables.h"


namespace dvh {


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

// Wave-uniform load through the scalar cache (s_load).  The tables the kernels read (pass / segment / chunk
// tables, order, scales, weights, the pivot-spectra table) are written only by earlier launches, so the
// constant address space is safe; it keeps these dependent loads off the vector memory pipe, where they
// queued behind the receiver loads.  The address must be wave-uniform.
template <class T>
__device__ __forceinline__ T sld(const T* p) {
  return *(const __attribute__((address_space(4))) T*)p;
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
  const int row0 = sld(A.pass_tab + 2 * p);
  t.p = p;
  t.row0 = row0;
  t.pivot = sld(A.pass_tab + 2 * p + 1);
  t.ch = row0 + i;
  const float* base = A.win + (int64_t)p * A.pass_stride;
  t.piv = base + (int64_t)t.pivot * A.ch_stride;
  t.rcv = base + (int64_t)t.ch * A.ch_stride;
  const int32_t* seg = A.seg_tab + ((int64_t)p * A.R + i) * 4;
  t.a_f = sld(seg);
  t.nwin_f = n_subwin(sld(seg + 1), A.w, A.hop);
  const bool other = (A.flags & kFlagOtherSide) != 0;
  t.a_o = sld(seg + 2);
  t.nwin_o = other ? n_subwin(sld(seg + 3), A.w, A.hop) : 0;
  return t;
}

// Opaque copy of a per-lane value: index arithmetic derived from it stays where it is used instead
// of being hoisted to the kernel entry (where, for per-task paths, it only occupies registers across the
// whole task loop and gets spilled once per wave).
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// |x| != 0 as a bit mask (NaN included); OR-accumulate, test once per sub-window
__device__ __forceinline__ uint32_t nzbits(float x) { return __builtin_bit_cast(uint32_t, x) & 0x7fffffffu; }
// OR-accumulated non-zero bits of the loaded samples (one v_and_or per sample)
__device__ __forceinline__ uint32_t maxbits(uint32_t b, float x) { return b | nzbits(x); }
// Validity flags of the covered-span scan (dvh_vsg.hip): per pass the max |x| bit pattern of the samples the scan
// read (>= kInfBits: a NaN / inf), or'ed with kSuspect when a correlation wave saw a non-finite spectrum it cannot
// attribute to one pass (the window is then rescanned whole).
constexpr uint32_t kInfBits = 0x7f800000u, kSuspect = 0x80000000u;

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
                                                     int lane_) {
  constexpr int N = E::NFFT;
  const int lane = opaque(lane_);
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

  __device__ EngStockham(char* lds, int wave, int lane_) : lane(lane_), live_f(false), live_o(false) {
    tw = reinterpret_cast<float2*>(lds);
    bufA = reinterpret_cast<float2*>(lds + kBlockBytes + (size_t)wave * kWaveBytes);
    bufB = bufA + N;
  }
  static __device__ void block_init(char* lds) { init_twiddles<N>(reinterpret_cast<float2*>(lds)); }

  // sub-window samples staged in registers; a padded transform (w <= N / 2) only has samples n < N / 2, the
  // upper half of its input is zero (stored once per sub-window, no registers)
  static constexpr int NZ = PAD ? (N / 2 + 63) / 64 : NJ;
  __device__ void load(const RowTask& t, int a, int w, float2 (&z)[NZ]) const {
#pragma unroll
    for (int j = 0; j < NZ; ++j) {
      const int n = lane + 64 * j;
      z[j] = (n < w) ? make_float2(t.piv[a + n], t.rcv[a + n]) : make_float2(0.f, 0.f);
    }
  }

  // accumulated cross spectra of both sides: Cf[j], Co[j] at bins f = lane + 64 j
  __device__ void spectra(const RowTask& t, const RowTask&, bool, int w, int hop, float2 (&Cf)[NH],
                          float2 (&Co)[NH]) {
    const int nq = t.nwin_f + t.nwin_o;
    float2 z[NZ];
#pragma unroll
    for (int j = 0; j < NH; ++j) {
      Cf[j] = make_float2(0.f, 0.f);
      Co[j] = make_float2(0.f, 0.f);
    }
    live_f = live_o = false;
    if (nq > 0) load(t, t.nwin_f > 0 ? t.a_f : t.a_o, w, z);
    for (int q = 0; q < nq; ++q) {
      uint32_t bp = 0, br = 0;
#pragma unroll
      for (int j = 0; j < NZ; ++j) {
        const int n = lane + 64 * j;
        if (n < N) bufA[n] = z[j];
        bp |= nzbits(z[j].x);
        br |= nzbits(z[j].y);
      }
      if (PAD) {
#pragma unroll
        for (int j = NZ; j < NJ; ++j) {
          const int n = lane + 64 * j;
          if (n < N) bufA[n] = make_float2(0.f, 0.f);
        }
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
    this->spectra(t, nt, has_next, w, hop, Cf, Co);
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
// Per-pass table of pivot-slice spectra (FusedOps::spectra_tab).  A pass's rows read the pivot channel at
// few distinct slices: every row of a shared side (channel <= pivot forward, >= pivot other side,
// apis/virtual_shot_gather.py:145-180) at the pivot's own time window, and the trajectory rows whose
// trajectory time lies outside the record at the clamped window (argmax of an all-False mask is 0,
// virtual_shot_gather.py:29, so they all slice [0, nsamp)).  Entry e of pass p holds the spectra of the
// slices [start_e + q hop, + w), q < nwin_e:
//   e = 0: the forward shared window (the pivot row's forward slice), e = 1: the other side's,
//   e = 2: the forward trajectory window of the last gather row, e = 3: the other-side trajectory window
//   of the first gather row (the far rows' clamped windows).
// A row side whose (start, nwin) equals its entry's transforms only its receivers, two per complex FFT.
// An entry holds kTabSub = 3 sub-windows (the reference's default time_window_to_xcorr = 2 wlen: nwin = 3).
// A pass with a longer side is marked unusable in the head (every nwin = -1; tab_usable() is false) and
// its row tasks take the plain path.  BINS (per engine): the half-spectrum bins f <= N / 2 of P / 2 (the
// halving of z's separation folded in, exact), and at [BINS - 1].x a 1 when the slice has a non-zero sample.
constexpr int kTabEnt = 4;
constexpr int kTabSub = 3;

template <int BINS>
__device__ __forceinline__ const float2* tab_slice(const float2* tab, int p, int e, int q) {
  return tab + (((int64_t)p * kTabEnt + e) * kTabSub + q) * BINS;
}
template <int BINS>
constexpr int64_t tab_pass_f2() {
  return (int64_t)kTabEnt * kTabSub * BINS;  // float2 per pass
}
// (start, nwin) of every entry: int32 [n_pass][kTabEnt][2] after the spectra
template <int BINS>
__device__ __forceinline__ const int32_t* tab_head(const float2* tab, int n_pass) {
  return reinterpret_cast<const int32_t*>(tab + (int64_t)n_pass * tab_pass_f2<BINS>());
}

// ------------------------------------------------------------------------------------------------
// FusedOps<E>: the row-task logic of the engines whose first and last transform stages run in registers
// (EngF500, EngP1024).  E provides the transform: N / NFFT, NJ (sample registers), NH (half-spectrum slots
// per lane), kTabBins, bin(l, j), load_ri() (a sub-window's samples into registers), stage1() (registers ->
// LDS), finish_with(acc) (the remaining stages, then acc(j, Z[f], Z[N - f]) for every half-spectrum slot j
// of the lane), inverse() and c() (the correlation at lag k after the inverse).  FusedOps holds the per-wave
// state and the three ways a row task forms its accumulated cross spectra:
//   spectra():     one complex transform per sub-window, z = pivot + i receiver;
//   spectra_tab(): the sub-windows whose pivot slices the pass table holds cost only their receivers, two
//                  per transform (z = R_a + i R_b, separated in the last stage and multiplied into the
//                  table's P conj(R)); the others keep z = P + i R.  On the configs[2] geometry that is 2
//                  transforms for a row whose only side is shared and 3 for a far row with both sides,
//                  against 3 and 6;
//   direct_task(): a task whose passes have only a table-served forward side packs receivers two per
//                  transform ACROSS its passes.
template <class E, int kNJ, int kNH>
struct FusedOps {
  float2* tw;
  float2* bufA;
  float2* bufB;
  int lane;
  bool live_f, live_o;
  const float2* tab = nullptr;  // the pass table of pivot spectra (stack kernels), or none
  int w;                        // sub-window length: the padded engines load samples n < w
  uint32_t* vflag = nullptr;    // validated launch with the covered-span scan: the passes' validity flags, to which
                                // the correlation reports the non-finite samples it loads (the scan leaves them out)

  __device__ FusedOps(char* lds, int wave, int lane_, int w_) : lane(lane_), live_f(false), live_o(false), w(w_) {
    tw = reinterpret_cast<float2*>(lds);
    bufA = reinterpret_cast<float2*>(lds + E::kBlockBytes + (size_t)wave * E::kWaveBytes);
    bufB = bufA + E::kBufA;
  }
  __device__ __forceinline__ const E& self() const { return *static_cast<const E*>(this); }

  __device__ __forceinline__ void load(const RowTask& t, int a, float2 (&z)[kNJ]) const {
    self().load_ri(t.piv + a, t.rcv + a, z);
  }
  // the stages after stage 1 of the transform whose stage-1 output is in bufB; cross spectra into C
  __device__ __forceinline__ void finish(float2 (&C)[kNH]) const {
    self().finish_with([&](int j, float2 a, float2 b) { accumulate_cross(a, b, C[j]); });
  }

  // Covered-span scan: a loaded sub-window that is not transformed (a zero pivot or receiver slice) is checked here
  // for non-finite samples (rare); a transformed one carries them into the accumulated spectra, which the stack
  // tasks test.  p2 < 0: both halves of z belong to pass p; else the real half to p, the imaginary half to p2.
  __device__ void check_untransformed(const float2 (&z)[kNJ], int p, int p2 = -1) const {
    if (!vflag) return;
    uint32_t ma = 0, mb = 0;
#pragma unroll
    for (int j = 0; j < kNJ; ++j) {
      ma = max(ma, nzbits(z[j].x));
      mb = max(mb, nzbits(z[j].y));
    }
    const bool ba = __ballot(ma >= kInfBits) != 0, bb = __ballot(mb >= kInfBits) != 0;
    if (lane == 0) {
      if (p2 < 0) {
        if (ba || bb) atomicMax(vflag + p, kInfBits);
      } else {
        if (ba) atomicMax(vflag + p, kInfBits);
        if (bb) atomicMax(vflag + p2, kInfBits);
      }
    }
  }

  // the pass's table entries hold all its sub-windows (head nwin of entry 0 >= 0)
  __device__ __forceinline__ bool tab_usable(int p, int n_pass) const {
    return sld(tab_head<E::kTabBins>(tab, n_pass) + (int64_t)p * kTabEnt * 2 + 1) >= 0;
  }

  // Sub-window q's pivot and receiver samples are loaded one sub-window ahead.
  __device__ void spectra(const RowTask& t, const RowTask&, bool, int, int hop, float2 (&Cf)[kNH],
                          float2 (&Co)[kNH]) {
    constexpr int NH_ = kNH;
    const int nq = t.nwin_f + t.nwin_o;
#pragma unroll
    for (int j = 0; j < NH_; ++j) {
      Cf[j] = make_float2(0.f, 0.f);
      Co[j] = make_float2(0.f, 0.f);
    }
    live_f = live_o = false;
    auto start = [&](int q) { return q < t.nwin_f ? t.a_f + q * hop : t.a_o + (q - t.nwin_f) * hop; };
    float2 z[kNJ];
    if (nq > 0) load(t, start(0), z);
    for (int q = 0; q < nq; ++q) {
      uint32_t bp = 0, br = 0;
#pragma unroll
      for (int j = 0; j < kNJ; ++j) {
        bp = maxbits(bp, z[j].x);
        br = maxbits(br, z[j].y);
      }
      const bool live = (__ballot(bp != 0) != 0) && (__ballot(br != 0) != 0);
      if (live) self().stage1(z);
      else check_untransformed(z, t.p);
      if (q + 1 < nq) load(t, start(q + 1), z);
      if (!live) continue;  // exactly zero in the reference
      if (q < t.nwin_f) {
        live_f = true;
        finish(Cf);
      } else {
        live_o = true;
        finish(Co);
      }
    }
  }

  // ---- spectra_tab: the sub-windows whose pivot slices the table holds cost only their receivers ----
  // Transforms of a row task (wave-uniform): jobs k < npair pack the table-served receivers h = 2k, 2k + 1
  // (h < nrf: forward side, sub-window h, entry ef; then the other side, entry eo); the remaining nt
  // trajectory sub-windows (side ts, start at) are z = P + i R as in spectra().
  struct TabJobs {
    int nrf, nr, ef, eo, ts, at, nt, npair;
  };
  static __device__ __forceinline__ TabJobs tab_jobs(const RowTask& t, const int32_t* head) {
    TabJobs J;
    const bool shf = t.ch <= t.pivot, sho = t.ch >= t.pivot;
    // a trajectory side matches its far-row entry when its slices are the same
    const bool mf = shf || (t.nwin_f > 0 && t.a_f == sld(head + 4) && t.nwin_f == sld(head + 5));
    const bool mo = sho || (t.nwin_o > 0 && t.a_o == sld(head + 6) && t.nwin_o == sld(head + 7));
    J.ef = shf ? 0 : 2;
    J.eo = sho ? 1 : 3;
    J.nrf = mf ? t.nwin_f : 0;
    J.nr = J.nrf + (mo ? t.nwin_o : 0);
    J.ts = !mf ? 0 : 1;
    J.nt = !mf ? t.nwin_f : (!mo ? t.nwin_o : 0);
    J.at = J.ts == 0 ? t.a_f : t.a_o;
    J.npair = (J.nr + 1) >> 1;
    return J;
  }
  // table-served receiver h: side, sub-window, slice start
  __device__ __forceinline__ void tab_half(const RowTask& t, const TabJobs& J, int h, int hop, int& side, int& q,
                                           int& a) const {
    side = h < J.nrf ? 0 : 1;
    q = h < J.nrf ? h : h - J.nrf;
    a = (side == 0 ? t.a_f : t.a_o) + q * hop;
  }
  __device__ __forceinline__ void tab_load(const RowTask& t, const TabJobs& J, int k, int hop,
                                           float2 (&z)[kNJ]) const {
    if (k < J.npair) {
      int s0, q0, a0, s1, q1, a1;
      tab_half(t, J, 2 * k, hop, s0, q0, a0);
      tab_half(t, J, 2 * k + 1, hop, s1, q1, a1);
      self().load_ri(t.rcv + a0, 2 * k + 1 < J.nr ? t.rcv + a1 : nullptr, z);
    } else {
      const int a = J.at + (k - J.npair) * hop;
      self().load_ri(t.piv + a, t.rcv + a, z);
    }
  }

  __device__ void spectra_tab(const RowTask& t, int n_pass, int hop, float2 (&Cf)[kNH], float2 (&Co)[kNH]) {
    constexpr int NH_ = kNH, BINS = E::kTabBins;
#pragma unroll
    for (int j = 0; j < NH_; ++j) {
      Cf[j] = make_float2(0.f, 0.f);
      Co[j] = make_float2(0.f, 0.f);
    }
    live_f = live_o = false;
    const int32_t* head = tab_head<BINS>(tab, n_pass) + (int64_t)t.p * kTabEnt * 2;
    const TabJobs J = tab_jobs(t, head);
    const int nj = J.npair + J.nt;
    float2 z[kNJ];
    if (nj > 0) tab_load(t, J, 0, hop, z);
    for (int k = 0; k < nj; ++k) {
      const bool pairjob = k < J.npair;
      uint32_t bp = 0, br = 0;
#pragma unroll
      for (int j = 0; j < kNJ; ++j) {
        bp = maxbits(bp, z[j].x);
        br = maxbits(br, z[j].y);
      }
      const bool nzp = __ballot(bp != 0) != 0, nzr = __ballot(br != 0) != 0;
      int s0 = 0, q0 = 0, a0 = 0, s1 = 0, q1 = 0, a1 = 0;
      bool la = false, lb = false;
      const float2 *Pa = nullptr, *Pb = nullptr;
      if (pairjob) {
        tab_half(t, J, 2 * k, hop, s0, q0, a0);
        tab_half(t, J, 2 * k + 1, hop, s1, q1, a1);
        Pa = tab_slice<BINS>(tab, t.p, s0 == 0 ? J.ef : J.eo, q0);
        Pb = tab_slice<BINS>(tab, t.p, s1 == 0 ? J.ef : J.eo, q1);
        // a receiver slice or its pivot slice identically zero: exactly zero in the reference
        la = nzp && sld(&Pa[BINS - 1].x) != 0.f;
        lb = (2 * k + 1 < J.nr) && nzr && sld(&Pb[BINS - 1].x) != 0.f;
      }
      const bool live = pairjob ? (la || lb) : (nzp && nzr);
      if (live) self().stage1(z);
      else check_untransformed(z, t.p);
      if (k + 1 < nj) tab_load(t, J, k + 1, hop, z);
      if (!live) continue;
      if (pairjob) {
        // the table's P at this lane's bins, loaded under the middle stages
        float2 pa[NH_], pb[NH_];
#pragma unroll
        for (int j = 0; j < NH_; ++j) {
          const int f = max(E::bin(lane, j), 0);
          pa[j] = Pa[f];
          pb[j] = Pb[f];
        }
        if (la) {
          if (s0 == 0) live_f = true;
          else live_o = true;
        }
        if (lb) {
          if (s1 == 0) live_f = true;
          else live_o = true;
        }
        const bool fa = s0 == 0, fb = s1 == 0;
        self().finish_with([&](int j, float2 za, float2 zc) {
          // z = R_a + i R_b: R_a = (Z[f] + conj Z[-f]) / 2, R_b = (Z[f] - conj Z[-f]) / 2i; P conj(R)
          if (la) {
            const float2 r = make_float2(za.x + zc.x, za.y - zc.y);  // 2 R_a (the table holds P / 2)
            const float2 c = make_float2(pa[j].x * r.x + pa[j].y * r.y, pa[j].y * r.x - pa[j].x * r.y);
            float2& C = fa ? Cf[j] : Co[j];
            C.x += c.x;
            C.y += c.y;
          }
          if (lb) {
            const float2 r = make_float2(za.y + zc.y, zc.x - za.x);  // 2 R_b
            const float2 c = make_float2(pb[j].x * r.x + pb[j].y * r.y, pb[j].y * r.x - pb[j].x * r.y);
            float2& C = fb ? Cf[j] : Co[j];
            C.x += c.x;
            C.y += c.y;
          }
        });
      } else if (J.ts == 0) {
        live_f = true;
        finish(Cf);
      } else {
        live_o = true;
        finish(Co);
      }
    }
  }

  // ---- direct_task: a row task whose passes have only a table-served forward side ----
  // (no row norm; every pass's other side empty, its forward slices in the table, the same sub-window count
  // W and shared/far-window kind on every pass, finite factors).  The passes' receivers are then packed two
  // per transform ACROSS passes -- ceil(W n / 2) transforms for n passes instead of n ceil(W / 2) -- and each
  // pass's weight w_p = weight / W * scale is applied per half:  U = sum_p w_p sum_q P_pq conj(R_pq).
  // RAMP (exact engines): Gh += (-1)^lane ramp(U), the forward epilogue of stackf_tasks (ok = false: no
  // other side) summed over the passes; otherwise (padded engines) Gh += U, the forward side's accumulated
  // spectrum, and *shared = the passes' common lag convention.  On the configs[2] geometry these are the
  // rows below the pivot (3 receivers per pass).  Returns false (nothing done) when the task does not qualify.
  template <bool RAMP>
  __device__ bool direct_task(const VsgArgs& A, const float* __restrict__ scales, const int32_t* __restrict__ order,
                              const float* __restrict__ weight, int b, int e, int i, float2 (&Gh)[kNH],
                              bool* shared = nullptr) {
    constexpr int NH_ = kNH, BINS = E::kTabBins;
    const int n = e - b;
    if (n <= 1 || n > 64) return false;
    const bool other = (A.flags & kFlagOtherSide) != 0;
    // lane k < n: pass order[b + k] (the passes' table entries in flight together: one load latency)
    const bool act = lane < n;
    int p = 0, row0 = 0, piv = 0, a = 0, L = 0, Lo = 0, h1 = 0, h4 = -1, h5 = -1;
    float sf = 0.f, wp = 0.f;
    if (act) {
      p = order[b + lane];
      row0 = A.pass_tab[2 * p];
      piv = A.pass_tab[2 * p + 1];
      const int32_t* seg = A.seg_tab + ((int64_t)p * A.R + i) * 4;
      a = seg[0];
      L = seg[1];
      Lo = seg[3];
      const int32_t* head = tab_head<BINS>(tab, A.n_pass) + (int64_t)p * kTabEnt * 2;
      h1 = head[1];
      h4 = head[4];
      h5 = head[5];
      sf = scales[2 * p];
      wp = weight[p];
    }
    const int ch = row0 + i;
    const int nwf = n_subwin(L, A.w, A.hop), nwo = other ? n_subwin(Lo, A.w, A.hop) : 0;
    const bool shf = ch <= piv;
    const int W = uni(nwf);
    const bool shf0 = uni(shf ? 1 : 0) != 0;
    const bool mf = shf || (nwf > 0 && a == h4 && nwf == h5);
    // the epilogue's forward factor: ff = 1 / nwin_f, times the scale (side_scale), times the class weight
    float wgt = 0.f;
    if (W > 0) {
      float ff = 1.0f / (float)W;
      ff *= sf;
      wgt = wp * ff;
    }
    const bool good = !act || (h1 >= 0 && nwo == 0 && nwf == W && shf == shf0 && mf && isfinite(wgt));
    if (__ballot(!good) != 0) return false;
    if (shared) *shared = shf0;
    if (W == 0) return true;  // no sub-windows on any pass: the row adds nothing
    // per-pass sources in lane k: receiver slice and table slice of sub-window 0, factor
    const uint64_t rp = reinterpret_cast<uint64_t>(A.win + (int64_t)p * A.pass_stride + (int64_t)ch * A.ch_stride + a);
    const uint64_t pp = reinterpret_cast<uint64_t>(tab_slice<BINS>(tab, p, shf ? 0 : 2, 0));
    const uint32_t rlo = (uint32_t)rp, rhi = (uint32_t)(rp >> 32), plo = (uint32_t)pp, phi = (uint32_t)(pp >> 32);
    const uint32_t wv = __builtin_bit_cast(uint32_t, wgt);
    // halves in order: pass k, sub-window s (cursor of the next half to hand out)
    int hk = 0, hs = 0;
    auto take = [&](const float*& r, const float2*& P, float& wt) {
      const int k = hk;
      r = reinterpret_cast<const float*>(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)rhi, k) << 32) |
                                         (uint32_t)__builtin_amdgcn_readlane((int)rlo, k)) + hs * A.hop;
      P = reinterpret_cast<const float2*>(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)phi, k) << 32) |
                                          (uint32_t)__builtin_amdgcn_readlane((int)plo, k)) + hs * BINS;
      wt = __builtin_bit_cast(float, __builtin_amdgcn_readlane((int)wv, k));
      if (++hs == W) {
        hs = 0;
        ++hk;
      }
    };
    const int M = W * n, nj = (M + 1) >> 1;
    float2 U[NH_];
#pragma unroll
    for (int j = 0; j < NH_; ++j) U[j] = make_float2(0.f, 0.f);
    const float *ra, *rb;
    const float2 *Pa, *Pb;
    float wa, wb = 0.f;
    take(ra, Pa, wa);
    bool hb = hk < n;
    if (hb) take(rb, Pb, wb);
    else {
      rb = ra;
      Pb = Pa;
    }
    float2 z[kNJ];
    self().load_ri(ra, rb, z);
    for (int jb = 0; jb < nj; ++jb) {
      uint32_t bp = 0, br = 0;
#pragma unroll
      for (int j = 0; j < kNJ; ++j) {
        bp = maxbits(bp, z[j].x);
        br = maxbits(br, z[j].y);
      }
      // a receiver slice or its pivot slice identically zero: exactly zero in the reference
      const bool la = (__ballot(bp != 0) != 0) && sld(&Pa[BINS - 1].x) != 0.f;
      const bool lb = hb && (__ballot(br != 0) != 0) && sld(&Pb[BINS - 1].x) != 0.f;
      const bool live = la || lb;
      if (live) self().stage1(z);
      else check_untransformed(z, __builtin_amdgcn_readlane(p, (2 * jb) / W),
                               hb ? __builtin_amdgcn_readlane(p, (2 * jb + 1) / W) : __builtin_amdgcn_readlane(p, (2 * jb) / W));
      const float2 *Pa_c = Pa, *Pb_c = Pb;
      const float wa_c = wa, wb_c = wb;
      if (jb + 1 < nj) {  // the next pair's samples, loaded under this transform
        take(ra, Pa, wa);
        hb = hk < n;
        if (hb) take(rb, Pb, wb);
        else {
          rb = ra;
          Pb = Pa;
        }
        self().load_ri(ra, rb, z);
      }
      if (!live) continue;
      float2 pa[NH_], pb[NH_];
#pragma unroll
      for (int j = 0; j < NH_; ++j) {
        const int f = max(E::bin(lane, j), 0);
        pa[j] = Pa_c[f];
        pb[j] = Pb_c[f];
      }
      self().finish_with([&](int j, float2 za, float2 zc) {
        // z = R_a + i R_b: R_a = (Z[f] + conj Z[-f]) / 2, R_b = (Z[f] - conj Z[-f]) / 2i; w P conj(R)
        if (la) {
          const float2 r = make_float2(za.x + zc.x, za.y - zc.y);  // 2 R_a (the table holds P / 2)
          U[j].x += wa_c * (pa[j].x * r.x + pa[j].y * r.y);
          U[j].y += wa_c * (pa[j].y * r.x - pa[j].x * r.y);
        }
        if (lb) {
          const float2 r = make_float2(za.y + zc.y, zc.x - za.x);  // 2 R_b
          U[j].x += wb_c * (pb[j].x * r.x + pb[j].y * r.y);
          U[j].y += wb_c * (pb[j].y * r.x - pb[j].x * r.y);
        }
      });
    }
    if (vflag) {  // a non-finite sample of some pass reached U: each of the task's passes is rescanned whole
      bool nf = false;
#pragma unroll
      for (int j = 0; j < NH_; ++j) nf |= !isfinite(U[j].x) || !isfinite(U[j].y);
      if (__ballot(nf) != 0 && act) atomicOr(vflag + p, kSuspect);
    }
    if constexpr (RAMP) {
      // Gh = (-1)^lane (conj on the shared window) U conj(tw[f])
      const int ln = opaque(lane);
      const float sg = (ln & 1) ? -1.f : 1.f;
#pragma unroll
      for (int j = 0; j < NH_; ++j) {
        const int f = E::bin(ln, j);
        if (f >= 0) {
          const float2 t = tw[f];
          const float2 x = cmul(shf0 ? make_float2(U[j].x, -U[j].y) : U[j], make_float2(t.x, -t.y));
          Gh[j].x += sg * x.x;
          Gh[j].y += sg * x.y;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < NH_; ++j) {
        Gh[j].x += U[j].x;
        Gh[j].y += U[j].y;
      }
    }
    return true;
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
struct EngF500 : FusedOps<EngF500, 8, 5> {
  static constexpr int N = 500;
  static constexpr int NFFT = 500;
  static constexpr int NJ = 8;
  static constexpr int NH = 5;
  static constexpr int kWaves = 4;
  static constexpr bool kNextTask = false;
  static constexpr int kTabBins = 256;  // bins f <= 250; [255].x: the slice's non-zero flag
  static constexpr size_t kBlockBytes = sizeof(float2) * N;     // twiddle table
  static constexpr size_t kWaveBytes = sizeof(float2) * 2 * N;  // ping-pong buffers
  static constexpr int kBufA = N;                               // bufB = bufA + kBufA

  __device__ EngF500(char* lds, int wave, int lane_) : FusedOps<EngF500, 8, 5>(lds, wave, lane_, N) {}
  static __device__ void block_init(char* lds) { init_twiddles<N>(reinterpret_cast<float2*>(lds)); }

  static __device__ __forceinline__ int bin(int l, int j) {
    if (j < 3) return l <= 50 ? l + 100 * j : -1;
    return (l >= 1 && l <= 49) ? 100 - l + 100 * (j - 3) : -1;
  }
  static __device__ __forceinline__ int slot(int n) { return n; }

  // stage-1 operands z[4 r + t] = (re, im)[i + 125 t], i = lane + 64 r, of the slices starting at re / im
  // Branch-free: lanes past the 125 stage-1 butterflies (round 1, lane >= 61) load lane 60's samples
  // again, which stage1() does not store and which leave the non-zero tests unchanged; with im ==
  // nullptr the receiver is loaded into both halves (the second half's result is discarded).
  __device__ __forceinline__ void load_ri(const float* re, const float* im, float2 (&z)[8]) const {
    const float* ip = im ? im : re;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = r == 0 ? lane : min(lane + 64, 124);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int n = i + 125 * u;
        z[4 * r + u] = make_float2(re[n], ip[n]);
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
        // the four outputs are two 16-byte stores, X[4i..4i+1] and X[4i+2..4i+3]; with both in that order an
        // 8-lane store group hits banks 8i mod 32 twice (2-way conflict, the engine's only one).  Lanes with
        // i & 4 store their second pair first, so each store's eight 16-byte pieces tile the 32 banks.
        const bool sw = (lane & 4) != 0;
        const int o = sw ? 2 : 0;
        float4* d = reinterpret_cast<float4*>(bufB + 4 * i);
        d[o >> 1] = sw ? make_float4(a[2].x, a[2].y, a[3].x, a[3].y) : make_float4(a[0].x, a[0].y, a[1].x, a[1].y);
        d[(2 - o) >> 1] = sw ? make_float4(a[0].x, a[0].y, a[1].x, a[1].y) : make_float4(a[2].x, a[2].y, a[3].x, a[3].y);
      }
    }
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
    const int ln = opaque(lane);  // the stage's addresses formed per call, not held in registers between calls
    if (ln <= 50) {
      float2 XA[5], XB[5];
      const bool pair = ln >= 1 && ln <= 49;
      last_bfly_from(bufB, ln, XA);
      if (pair) last_bfly_from(bufB, 100 - ln, XB);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        // partner X[N - f] of f = l + 100 j is X[(100 - l) + 100 (4 - j)]
        const float2 p0 = XA[(5 - j) % 5], p50 = XA[4 - j], pb = XB[4 - j];
        float2 pa;  // value selects (a select of array elements would become a scratch pointer)
        pa.x = ln == 0 ? p0.x : (ln == 50 ? p50.x : pb.x);
        pa.y = ln == 0 ? p0.y : (ln == 50 ? p50.y : pb.y);
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
    const float2 w1 = tw[k];
    float2 wt = w1;
#pragma unroll
    for (int t = 1; t < 5; ++t) {
      x[t] = cmul(x[t], wt);
      if (t < 4) wt = cmul(wt, w1);
    }
    Dft<5>::run(x);
  }

  __device__ const float2* inverse(const float2 (&Cf)[NH], const float2 (&Co)[NH]) {
    store_conj_hermitian<EngF500>(bufA, Cf, Co, lane);
    wave_sync();
    return FftPlan<N>::T::run(bufA, bufB, tw, lane);
  }

  __device__ const float2* correlate(const RowTask& t, const RowTask& nt, bool has_next, int w, int hop) {
    float2 Cf[NH], Co[NH];
    this->spectra(t, nt, has_next, w, hop, Cf, Co);
    return inverse(Cf, Co);
  }

  __device__ float2 twiddle(int m) const { return tw[m]; }

  __device__ float2 c(const float2* Y, int k, int) const {
    const float2 v = Y[k];
    return make_float2(v.x, -v.y);
  }
};


// ------------------------------------------------------------------------------------------------
// EngP1024: zero-padded N = 1024 Stockham for the window lengths without an exact engine, w <= 512 (w = int(wlen /
// dt) = 499 at the reference's other operating point, dt = 0.004000000000001336): the linear correlation of the
// zero-padded sub-windows (N >= 2w - 1) is folded back to the circular one in c().  The transform is fused like
// EngF500's:
//   the first stage from the prefetched samples: a lane holds z[j] = x[lane + 64 j], j < 8 (only samples n < w <=
//     512 can be non-zero: half the registers of a 1 024-sample stage), and its butterflies drop the zero inputs;
//   the last stage (radix 4, span 256) runs butterflies k and 256 - k in one lane -- round A: (l, 256 - l) for l >= 1
//     and (0, 128) on lane 0, both self-partnered; round B: (64 + l, 192 - l) -- so each lane holds X[f] and X[N - f]
//     of its bins and forms their cross spectra in registers.
// Half-spectrum slots per lane l (each bin f <= 512 exactly once):
//   j = 0, 1: l, l + 256;  j = 2, 3: 256 - l, 512 - l (lane 0: 128, 384);  j = 4..7: 64 + l, 320 + l, 192 - l,
//   448 - l;  j = 8: 512 (lane 0 only).
// The transforms run as radix-16 stages: forward = radix 16 (span 1, from the registers, zero-padded half) -> LDS A ->
// radix 16 (span 16) -> LDS B -> the paired radix-4 last stage (span 256) in registers; inverse = radix 4 (span 1,
// from the registers) -> LDS B -> radix 16 (span 4) -> LDS A -> radix 16 (span 64) -> Y in LDS B.  Two LDS round trips
// per transform instead of four radix-4 ones, one wave synchronisation per stage boundary, and the twiddle products of
// two radix-4 stages merged into one radix-16 stage.  Buffer A is padded (the span-1 forward stage's 16 outputs per
// lane at n + n / 16, the span-4 inverse stage's at n + 4 (n / 64)), so the stores and reads of every stage are
// conflict free; buffer B is plain.  (An XOR-swizzled radix-4 layout cut the conflicts further but cost 25 % more VALU
// for no gain)
struct EngP1024 : FusedOps<EngP1024, 8, 9> {
  static constexpr int N = 1024;
  static constexpr int NFFT = 1024;
  static constexpr int NJ = 8;  // sample registers: n < N / 2
  static constexpr int NH = 9;
  static constexpr int kWaves = 4;
  static constexpr bool kNextTask = false;
  static constexpr int kTabBins = 520;  // bins f <= 512; [519].x: the slice's non-zero flag
  static constexpr int kBufA = N + N / 16;
  static constexpr size_t kWaveBytes = sizeof(float2) * (kBufA + N);  // buffers A and B
  // Radix-16 stage twiddles, contiguous per stage after the main table: stage Ls holds w^k, w^4k, w^8k (w = e^(-2 pi
  // i Ls' / N), Ls' = N / (16 Ls)) for k < Ls at r16_tw(Ls) + {0, Ls, 2 Ls} + k, so that a stage's reads by lanes of
  // consecutive k are consecutive (read from the main table at stride 4 k, 16 k, 32 k they cost 1.6 bank-conflict
  // cycles per LDS instruction of the whole launch).
  static constexpr int kR16Tw = N;
  static constexpr int kR16TwEntries = 3 * (16 + 4 + 64);
  static constexpr int r16_tw(int Ls) { return kR16Tw + (Ls == 16 ? 0 : (Ls == 4 ? 48 : 60)); }
  static constexpr size_t kBlockBytes = sizeof(float2) * (N + kR16TwEntries);

  __device__ EngP1024(char* lds, int wave, int lane_) : FusedOps<EngP1024, 8, 9>(lds, wave, lane_, N / 2) {}
  static __device__ void block_init(char* lds) {
    float2* t = reinterpret_cast<float2*>(lds);
    init_twiddles<N>(t);
    for (int e = threadIdx.x; e < kR16TwEntries; e += blockDim.x) {
      const int Ls = e < 48 ? 16 : (e < 60 ? 4 : 64), o = e - (Ls == 16 ? 0 : (Ls == 4 ? 48 : 60));
      const int j = o / Ls, k = o % Ls, mult = j == 0 ? 1 : (j == 1 ? 4 : 8);
      const int m = mult * k * (N / (16 * Ls));
      double sn, cs;
      sincospi(2.0 * (double)m / (double)N, &sn, &cs);  // init_twiddles' formula: the same float values as tw[m]
      t[kR16Tw + e] = make_float2((float)cs, (float)(-sn));
    }
  }

  static __device__ __forceinline__ int bin(int l, int j) {
    switch (j) {
      case 0: return l;
      case 1: return l + 256;
      case 2: return l == 0 ? 128 : 256 - l;
      case 3: return l == 0 ? 384 : 512 - l;
      case 4: return 64 + l;
      case 5: return 320 + l;
      case 6: return 192 - l;
      case 7: return 448 - l;
      default: return l == 0 ? 512 : -1;
    }
  }
  static __device__ __forceinline__ int slot(int n) { return n; }

  // z[j] = (re, im)[lane + 64 j], j < 8, zero past the sub-window (n >= w); im == nullptr: the receiver in
  // both halves (the second half's result is discarded)
  __device__ __forceinline__ void load_ri(const float* re, const float* im, float2 (&z)[8]) const {
    const float* ip = im ? im : re;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = lane + 64 * j;
      z[j] = n < w ? make_float2(re[n], ip[n]) : make_float2(0.f, 0.f);
    }
  }

  // the four outputs of radix-4 butterfly i of a span-1 stage (out[4 i + q]) as two 16-byte stores at a 32-byte
  // lane stride; lanes with i & 4 store their second pair first so that every 8-lane store group tiles the 32 banks
  // (as EngF500's stage 1)
  static __device__ __forceinline__ void store4(float2* out, int i, float2 x0, float2 x1, float2 x2, float2 x3) {
    const bool sw = (i & 4) != 0;
    const int o = sw ? 2 : 0;
    float4* d = reinterpret_cast<float4*>(out + 4 * i);
    d[o >> 1] = sw ? make_float4(x2.x, x2.y, x3.x, x3.y) : make_float4(x0.x, x0.y, x1.x, x1.y);
    d[(2 - o) >> 1] = sw ? make_float4(x0.x, x0.y, x1.x, x1.y) : make_float4(x2.x, x2.y, x3.x, x3.y);
  }

  __device__ __forceinline__ void stage1(const float2 (&z)[8]) const {
    // radix-16 butterfly i = lane of x[i + 64 t], t < 16: the prefetched z[t] for t < 8, zero above; outputs
    // out[16 i + q] at the padded index 17 i + q (16 lanes of a store group: 16 distinct banks)
    float2 a[16];
#pragma unroll
    for (int t = 0; t < 8; ++t) a[t] = z[t];
    dft16<true>(a);
    float2* o = bufA + 17 * lane;
#pragma unroll
    for (int q = 0; q < 16; ++q) o[q] = a[q];
  }

  // radix-16 Stockham stage (span Ls = 16, 4 or 64) of butterfly i = lane: inputs in[ia(i + 64 t)], twiddles
  // w^t with w = tw[k N / (16 Ls)] (k = i % Ls), outputs out[oa((i - k) 16 + k + Ls q)]
  template <int Ls, class IA, class OA>
  __device__ __forceinline__ void stage16(const float2* in, float2* out, IA ia, OA oa) const {
    const int i = lane, k = i % Ls;
    float2 a[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) a[t] = lds_ld(in, ia(i + 64 * t));
    const float2* st = tw + r16_tw(Ls);
    twiddle16(a, st[k], st[Ls + k], st[2 * Ls + k]);
    dft16<false>(a);
    const int base = (i - k) * 16 + k;
#pragma unroll
    for (int q = 0; q < 16; ++q) out[oa(base + Ls * q)] = a[q];
  }

  // radix-4 butterfly k of the last stage (span 256): X[k + 256 q], q < 4
  __device__ __forceinline__ void last_bfly_from(const float2* src, int k, float2 (&x)[4]) const {
#pragma unroll
    for (int t = 0; t < 4; ++t) x[t] = lds_ld(src, k + 256 * t);
    const float2 w1 = tw[k];
    float2 wt = w1;
#pragma unroll
    for (int t = 1; t < 4; ++t) {
      x[t] = cmul(x[t], wt);
      if (t < 3) wt = cmul(wt, w1);
    }
    Dft<4>::run(x);
  }

  static __device__ __forceinline__ float2 sel(bool c, float2 a, float2 b) {
    return make_float2(c ? a.x : b.x, c ? a.y : b.y);  // value selects (no scratch pointer)
  }

  // stages 2-5 of the transform whose stage-1 output is in bufB; acc(j, Z[f], Z[N - f]) for every valid
  // half-spectrum slot j of the lane (compile-time j)
  template <class F>
  __device__ __forceinline__ void finish_with(F&& acc) const {
    wave_sync();
    stage16<16>(bufA, bufB, [](int n) { return n + (n >> 4); }, [](int n) { return n; });
    const float2* src = bufB;  // the span-256 stage's input
    wave_sync();
    const int ln = opaque(lane);  // the stage's addresses formed per call, not held in registers between calls
    const bool l0 = ln == 0;
    {
      float2 XA[4], XB[4];
      last_bfly_from(src, ln, XA);
      last_bfly_from(src, l0 ? 128 : 256 - ln, XB);
      acc(0, XA[0], sel(l0, XA[0], XB[3]));
      acc(1, XA[1], sel(l0, XA[3], XB[2]));
      acc(2, XB[0], sel(l0, XB[3], XA[3]));
      acc(3, XB[1], sel(l0, XB[2], XA[2]));
      if (l0) acc(8, XA[2], XA[2]);
    }
    {
      float2 XA[4], XB[4];
      last_bfly_from(src, 64 + ln, XA);
      last_bfly_from(src, 192 - ln, XB);
      acc(4, XA[0], XB[3]);
      acc(5, XA[1], XB[2]);
      acc(6, XB[0], XA[3]);
      acc(7, XB[1], XA[2]);
    }
    wave_sync();
  }

  // The inverse transform conj(FFT(conj(W))) of W = Cf + i Co (W[N - f] = conj Cf[f] + i conj Co[f]).  Its first
  // stage (span 1: butterfly i of x[i + 256 t], t < 4, no twiddles) runs from the registers: the inputs of each
  // butterfly are four of ONE lane's half-spectrum slots or their Hermitian partners -- lane l >= 1 holds those of
  // butterflies l, 64 + l, 192 - l and 256 - l, lane 0 those of 0, 64, 128 and 192 -- so the spectrum is never
  // stored and re-read; then stages 2-5 in the swizzled layout.  Returns Y (bufB), read through c().
  __device__ const float2* inverse(const float2 (&Cf)[NH], const float2 (&Co)[NH]) {
    const int ln = opaque(lane);
    const bool l0 = ln == 0;
    // x[f] = conj W[f] = A(j), x[N - f] = conj W[N - f] = B(j) for slot j's bin f
    auto A = [&](int j) { return make_float2(Cf[j].x - Co[j].y, -(Cf[j].y + Co[j].x)); };
    auto B = [&](int j) { return make_float2(Cf[j].x + Co[j].y, Cf[j].y - Co[j].x); };
    auto bfly = [&](int i, float2 a0, float2 a1, float2 a2, float2 a3) {
      float2 a[4] = {a0, a1, a2, a3};
      Dft<4>::run(a);
      store4(bufB, i, a[0], a[1], a[2], a[3]);
    };
    // lane 0: x[512] is bin 512 itself (slot 8), x[768] the partner of bin 256 (slot 1); lanes >= 1: partners of
    // 512 - l (slot 3) and 256 - l (slot 2)
    bfly(ln, A(0), A(1), l0 ? A(8) : B(3), l0 ? B(1) : B(2));
    bfly(64 + ln, A(4), A(5), B(7), B(6));
    // lanes >= 1: butterflies 192 - l and 256 - l; lane 0: 128 and 192 (value selects, no divergent branch)
    bfly(l0 ? 128 : 192 - ln, sel(l0, A(2), A(6)), sel(l0, A(3), A(7)), sel(l0, B(3), B(5)), sel(l0, B(2), B(4)));
    bfly(l0 ? 192 : 256 - ln, sel(l0, A(6), A(2)), sel(l0, A(7), A(3)), sel(l0, B(5), B(1)), sel(l0, B(4), B(0)));
    wave_sync();
    stage16<4>(bufB, bufA, [](int n) { return n; }, [](int n) { return n + 4 * (n >> 6); });
    wave_sync();
    stage16<64>(bufA, bufB, [](int n) { return n + 4 * (n >> 6); }, [](int n) { return n; });
    wave_sync();
    return bufB;
  }

  __device__ const float2* correlate(const RowTask& t, const RowTask& nt, bool has_next, int w_, int hop) {
    float2 Cf[NH], Co[NH];
    this->spectra(t, nt, has_next, w_, hop, Cf, Co);
    return inverse(Cf, Co);
  }

  __device__ float2 twiddle(int m) const { return tw[m]; }

  // (N * sum_s c_f[k], N * sum_s c_o[k]): the linear correlation folded to the circular one of period w
  __device__ float2 c(const float2* Y, int k, int w_) const {
    float2 v = Y[k];
    if (k > 0) {
      const float2 u = Y[N - w_ + k];
      v.x += u.x;
      v.y += u.y;
    }
    return make_float2(v.x, -v.y);
  }
};

}  // namespace dvh
