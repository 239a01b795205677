// EngQ500: the correlation engine of the stack kernels at the reference's operating point
// (w = 500: wlen = 2 s at 250 Hz), gfx950 wave64.
//
// A row task (pass p, gather row i) needs the spectra of up to 12 real 500-sample slices: on each
// side s in {forward, other} and sub-window q < nwin_s, the pivot slice P and the receiver slice R
// (XCORR_vshot / XCORR_two_traces, modules/utils.py:253-314).  On a side whose rows share the pivot's
// time window ("shared": channel <= pivot forward, >= pivot other side, apis/virtual_shot_gather.py:
// 145-180) the pivot slices are the same for every row of the pass: their spectra come from a per-pass
// table (vsg_pivot_spectra_kernel) and only the receiver is transformed.  The remaining real slices
// (3 shared receivers, 3 + 3 trajectory pivot / receiver slices) are packed two per complex
// transform: at most 5 "slots" per row task (one per shared receiver pair, one per trajectory
// sub-window), against 6 complex transforms of the per-sub-window engine (EngF500).
//
// The slots are transformed together as a four-step 500 = 20 x 25 FFT whose passes run in
// registers: pass 1, lane task (slot k, column n2): DFT-20 of x[25 n1 + n2] (loaded straight from
// global memory), times exp(-2 pi i n2 f1 / 500), written to LDS at [k][25 f1 + n2]; pass 2, lane
// task (slot k, row f1): DFT-25 of that row, written back in natural order X[f1 + 20 f2].  One LDS
// round trip per transform (a radix-4/5 Stockham makes three) and 25 / 20 independent butterflies
// per lane.  With 5 slots, pass 1 is 125 lane tasks (2 rounds of 64) and pass 2 100: the slots are
// processed as phase A (slots 0, 1 and the first 14 columns of slot 2) and phase B (slot 2's other
// columns, slots 3, 4), so a wave holds three 4 KB transform buffers (slots 3 and 4 reuse A's) and
// every pass-2 phase is a single round.  Rows with only a shared side (2 slots: most rows below the
// pivot when the trajectory leaves the window) run phase A only.
//
// Spectral phase: lane l owns bins f = l + 64 j (j < 4, f <= 250) and reads Z[f], Z[500 - f] of each
// slot from LDS: a trajectory slot z = P + i R gives P conj(R) = (i/4)(Z[f] + conj Z[-f]) conj(Z[f] -
// conj Z[-f]) (accumulate_cross); a shared slot z = R_a + i R_b gives R_a = (Z[f] + conj Z[-f]) / 2,
// R_b = (Z[f] - conj Z[-f]) / 2i, each multiplied into the table's P conj(R).  A slice that is
// identically zero contributes exactly zero in the reference and is skipped (bit test of every loaded
// sample, NaN counted as non-zero); slices of different sides never share a slot, so a NaN on one
// side cannot leak into the other (the reference keeps the forward row when the other side is NaN).
//
// The accumulated half spectra Cf / Co (bins l + 64 j, as EngStockham<500>) feed the same per-pass
// epilogue and one inverse transform per (pass chunk, row) as before (stackf_tasks).
#pragma once
#include "vsg_engines.h"

#ifndef DVH_Q_XPF
#define DVH_Q_XPF 0  // 1: load the next row task's first slices during this task's pass 2
#endif

namespace dvh {

// ------------------------------------------------------------------------------------------------
// register DFTs (forward, X[f] = sum_n x[n] exp(-2 pi i n f / N)), constant twiddles from tw_tables.h

__device__ __forceinline__ float2 cmul_c(float2 a, float c, float s) {  // a * (c + i s)
  return make_float2(a.x * c - a.y * s, a.x * s + a.y * c);
}

// DFT-20 in place, output index f = fa + 4 fb: n = 5 na + nb, step 1 DFT-4 over na, twiddle
// W20^(nb fa), step 2 DFT-5 over nb.
__device__ __forceinline__ void dft20(float2 (&a)[20]) {
  float2 u[5][4];
#pragma unroll
  for (int nb = 0; nb < 5; ++nb) {
    float2 t[4] = {a[nb], a[5 + nb], a[10 + nb], a[15 + nb]};
    Dft<4>::run(t);
#pragma unroll
    for (int fa = 0; fa < 4; ++fa) u[nb][fa] = (nb && fa) ? cmul_c(t[fa], Tw20::c[nb * fa], Tw20::s[nb * fa]) : t[fa];
  }
#pragma unroll
  for (int fa = 0; fa < 4; ++fa) {
    float2 t[5] = {u[0][fa], u[1][fa], u[2][fa], u[3][fa], u[4][fa]};
    Dft<5>::run(t);
#pragma unroll
    for (int fb = 0; fb < 5; ++fb) a[fa + 4 * fb] = t[fb];
  }
}

// DFT-25 in place, output index f = fa + 5 fb: n = 5 na + nb, step 1 DFT-5 over na, twiddle
// W25^(nb fa), step 2 DFT-5 over nb.
__device__ __forceinline__ void dft25(float2 (&a)[25]) {
  float2 u[5][5];
#pragma unroll
  for (int nb = 0; nb < 5; ++nb) {
    float2 t[5] = {a[nb], a[5 + nb], a[10 + nb], a[15 + nb], a[20 + nb]};
    Dft<5>::run(t);
#pragma unroll
    for (int fa = 0; fa < 5; ++fa) u[nb][fa] = (nb && fa) ? cmul_c(t[fa], Tw25::c[nb * fa], Tw25::s[nb * fa]) : t[fa];
  }
#pragma unroll
  for (int fa = 0; fa < 5; ++fa) {
    float2 t[5] = {u[0][fa], u[1][fa], u[2][fa], u[3][fa], u[4][fa]};
    Dft<5>::run(t);
#pragma unroll
    for (int fb = 0; fb < 5; ++fb) a[fa + 5 * fb] = t[fb];
  }
}

// ------------------------------------------------------------------------------------------------
// Per-pass pivot spectra of the shared sides: ptab[(p * 2 + side) * 3 + q][f], f <= 250, and at
// [.][255].x = 1 when the pivot slice has a non-zero sample (else 0: the sub-window contributes zero).
constexpr int kPtabBins = 256;
constexpr int kPtabPerPass = 2 * 3 * kPtabBins;  // float2 entries per pass

__device__ __forceinline__ const float2* ptab_of(const float2* ptab, int p, int side, int q) {
  return ptab + ((int64_t)p * 6 + side * 3 + q) * kPtabBins;
}

// A slot: up to two real slices packed as z = re + i im, each given as a byte offset into the
// pass's buffer descriptor (kNoSlice: absent, reads as zeros).
constexpr uint32_t kNoSlice = 0x80000000u;
enum : int { kSlotEmpty = 0, kSlotTraj = 1, kSlotShared = 2 };

struct QSlots {  // wave-uniform; every array is indexed with compile-time slot numbers only
  int n;
  uint32_t re[5], im[5];
  int code[5];  // kind | side_re << 2 | q_re << 3 | side_im << 5 | q_im << 6 (shared halves: (side, sub-window))
};

// ------------------------------------------------------------------------------------------------
struct EngQ500 {
  static constexpr int N = 500;
  static constexpr int NFFT = 500;
  static constexpr int NJ = 8;  // output lags k = lane + 64 j
  static constexpr int NH = 4;  // half-spectrum bins f = lane + 64 j <= 250
  static constexpr int kWaves = 4;  // waves per block of the plain stack kernel
  static constexpr bool kNextTask = DVH_Q_XPF != 0;
  static constexpr size_t kBlockBytes = sizeof(float2) * N;      // twiddle table (inverse, phase ramps)
  static constexpr size_t kWaveBytes = sizeof(float2) * 3 * N;   // three transform buffers
  float2* tw;
  float2* buf;  // [3][500]
  int lane;
  bool live_f, live_o;
  const float2* ptab = nullptr;  // the pass table of the shared pivot spectra (vsg_pivot_spectra_kernel)
  uint32_t vmax = 0;  // this lane's max |x| bit pattern over the slices the last spectra_q() loaded

  // Lane-derived indices are recomputed where they are used, from an opaque copy of the lane id
  // (hoisted to the kernel entry they would occupy registers across the task loop and spill).
  __device__ EngQ500(char* lds, int wave, int lane_) : lane(lane_), live_f(false), live_o(false) {
    tw = reinterpret_cast<float2*>(lds);
    buf = reinterpret_cast<float2*>(lds + kBlockBytes + (size_t)wave * kWaveBytes);
  }
  __device__ __forceinline__ int lid() const {
    int v = lane;
    asm volatile("" : "+v"(v));
    return v;
  }
  static __device__ void block_init(char* lds) { init_twiddles<N>(reinterpret_cast<float2*>(lds)); }

  static __device__ __forceinline__ int bin(int l, int j) {
    const int f = l + 64 * j;
    return f <= N / 2 ? f : -1;
  }
  static __device__ __forceinline__ int slot(int n) { return n; }

  // ---- slot layout of a row task (wave-uniform) ----
  // shared receivers first (side by side, two per slot), then the trajectory sub-windows
  static __device__ __forceinline__ QSlots make_slots(const VsgArgs& A, const RowTask& t, int row0) {
    QSlots S;
    const bool shf = t.ch <= t.pivot && t.nwin_f > 0;
    const bool sho = t.ch >= t.pivot && t.nwin_o > 0;
    const bool trf = t.ch > t.pivot && t.nwin_f > 0;
    const bool tro = t.ch < t.pivot && t.nwin_o > 0;
    // first shared side sa (n_a sub-windows), second shared side (pivot row only)
    const int sa = shf ? 0 : 1;
    const int n_a = shf ? t.nwin_f : (sho ? t.nwin_o : 0);
    const int n_b = (shf && sho) ? t.nwin_o : 0;
    const int a_a = sa == 0 ? t.a_f : t.a_o;
    const int slots_a = (n_a + 1) >> 1, slots_b = (n_b + 1) >> 1;
    const int ts = trf ? 0 : 1;  // trajectory side
    const int n_t = trf ? t.nwin_f : (tro ? t.nwin_o : 0);
    const int a_t = ts == 0 ? t.a_f : t.a_o;
    const int64_t rcv = (int64_t)(t.ch - row0) * A.ch_stride, piv = (int64_t)(t.pivot - row0) * A.ch_stride;
    S.n = slots_a + slots_b + n_t;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      uint32_t re = kNoSlice, im = kNoSlice;
      int kind = kSlotEmpty, sre = 0, qre = 0, sim = 0, qim = 0;
      if (k < slots_a) {
        kind = kSlotShared;
        sre = sim = sa;
        qre = 2 * k;
        qim = 2 * k + 1;
        re = (uint32_t)(4 * (rcv + a_a + qre * A.hop));
        if (qim < n_a) im = (uint32_t)(4 * (rcv + a_a + qim * A.hop));
      } else if (k < slots_a + slots_b) {
        kind = kSlotShared;
        sre = sim = 1;
        qre = 2 * (k - slots_a);
        qim = qre + 1;
        re = (uint32_t)(4 * (rcv + t.a_o + qre * A.hop));
        if (qim < n_b) im = (uint32_t)(4 * (rcv + t.a_o + qim * A.hop));
      } else if (k < S.n) {
        kind = kSlotTraj;
        sre = ts;
        qre = k - slots_a - slots_b;
        re = (uint32_t)(4 * (piv + a_t + qre * A.hop));
        im = (uint32_t)(4 * (rcv + a_t + qre * A.hop));
      }
      S.re[k] = uni((int)re);
      S.im[k] = uni((int)im);
      S.code[k] = uni(kind | (sre << 2) | (qre << 3) | (sim << 5) | (qim << 6));
    }
    return S;
  }

  // ---- pass 1 ----
  // this lane's slice offsets in round r (slot k = (64 r + lane) / 25)
  __device__ __forceinline__ void round_offsets(const QSlots& S, int r, uint32_t& ore, uint32_t& oim) const {
    const int tau = 64 * r + lid();
    const int k = tau / 25;
    ore = kNoSlice;
    oim = kNoSlice;
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      if (k == s) {
        ore = S.re[s];
        oim = S.im[s];
      }
    }
    const uint32_t d = 4u * (uint32_t)(tau - 25 * k);
    if (ore != kNoSlice) ore += d;
    if (oim != kNoSlice) oim += d;
  }

  // the 20 samples x[25 n1 + n2] of this lane's column, re and im slices (zeros for absent slices)
  __device__ __forceinline__ void load_round(const __amdgpu_buffer_rsrc_t& rs, const QSlots& S, int r,
                                             float (&xr)[20], float (&xi)[20]) const {
    uint32_t ore, oim;
    round_offsets(S, r, ore, oim);
#pragma unroll
    for (int n1 = 0; n1 < 20; ++n1) {
      xr[n1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(ore + 100u * n1), 0, 0));
      xi[n1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(oim + 100u * n1), 0, 0));
    }
  }

  // DFT-20 of the column, times exp(-2 pi i n2 f1 / 500), stored at dst[25 f1] when `store`; returns
  // the lane's (re non-zero, im non-zero) bits
  __device__ __forceinline__ uint32_t pass1(const float (&xr)[20], const float (&xi)[20], int r, float2* dst,
                                            bool store) {
    uint32_t nzr = 0, nzi = 0;  // max |x| bit patterns (0: all zero; >= 0x7f800000: NaN / inf)
    float2 a[20];
#pragma unroll
    for (int n1 = 0; n1 < 20; ++n1) {
      nzr = max(nzr, __builtin_bit_cast(uint32_t, xr[n1]) & 0x7fffffffu);
      nzi = max(nzi, __builtin_bit_cast(uint32_t, xi[n1]) & 0x7fffffffu);
      a[n1] = make_float2(xr[n1], xi[n1]);
    }
    dft20(a);
    // twiddles w^(fa + 4 fb) = w^fa (w^4)^fb, w = exp(-2 pi i n2 / 500) from the block's table
    const int n2 = (64 * r + lid()) % 25;
    const float2 w = tw[n2], v = tw[4 * n2];
    float2 wp[4], vp[5];
    wp[0] = make_float2(1.f, 0.f);
    wp[1] = w;
    wp[2] = cmul(w, w);
    wp[3] = cmul(wp[2], w);
    vp[0] = make_float2(1.f, 0.f);
    vp[1] = v;
    vp[2] = cmul(v, v);
    vp[3] = cmul(vp[2], v);
    vp[4] = cmul(vp[2], vp[2]);
#pragma unroll
    for (int fb = 0; fb < 5; ++fb) {
#pragma unroll
      for (int fa = 0; fa < 4; ++fa) {
        const int f1 = fa + 4 * fb;
        float2 y = a[f1];
        if (fa) y = cmul(y, wp[fa]);
        if (fb) y = cmul(y, vp[fb]);
        if (store) dst[25 * f1] = y;
      }
    }
    vmax = max(vmax, max(nzr, nzi));
    return (nzr ? 1u : 0u) | (nzi ? 2u : 0u);
  }

  // ---- pass 2: lane (buffer lane / 20, row f1 = lane % 20) while lane < 20 * nbuf ----
  __device__ __forceinline__ void pass2(int nbuf) const {
    const int l = lid();
    const int b = l / 20, f1 = l - 20 * b;
    if (b < nbuf) {
      float2* base = buf + 500 * b;
      float2 a[25];
#pragma unroll
      for (int n2 = 0; n2 < 25; ++n2) a[n2] = base[25 * f1 + n2];
      dft25(a);
      // every lane's reads of the buffer precede its writes (one wave, in-order LDS; the DFT depends on
      // all reads), so the natural-order spectrum may overwrite the rows in place
#pragma unroll
      for (int f2 = 0; f2 < 25; ++f2) base[f1 + 20 * f2] = a[f2];
    }
  }

  // ---- spectral phase: accumulate the slots of buffers [0, nbuf) (slot of buffer b = sl[b]) ----
  // The table rows of the first shared side (slots 0, 1), loaded at the start of the task so that their
  // latency runs under pass 1 / pass 2: Pre.v[q][j] = P[side][q][lane + 64 j], Pre.live bit q = flag.
  struct PivotPre {
    float2 v[3][NH];
    int side;   // -1: no prefetch (slot 0 is not a shared slot)
    int live;   // bit q: the pivot slice q is not identically zero
  };

  __device__ __forceinline__ void prefetch_pivot(const QSlots& S, const float2* __restrict__ ptab, int p,
                                                 PivotPre& P) const {
    P.side = -1;
    P.live = 0;
    if ((S.code[0] & 3) != kSlotShared) return;
    P.side = (S.code[0] >> 2) & 1;
    const int l = lid();
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const float2* row = ptab_of(ptab, p, P.side, q);
      P.live |= (row[kPtabBins - 1].x != 0.f) ? (1 << q) : 0;
#pragma unroll
      for (int j = 0; j < NH; ++j) P.v[q][j] = row[min(l + 64 * j, kPtabBins - 2)];
    }
    P.live = uni(P.live);
  }

  // P[side][q][bin j of this lane]: from the prefetch when it holds that side, else from the table
  __device__ __forceinline__ float2 pivot_bin(const PivotPre& P, const float2* __restrict__ ptab, int p, int side, int q,
                                              int j, int f) const {
    if (side == P.side) {
      float2 v = P.v[0][j];
      if (q == 1) v = P.v[1][j];
      if (q == 2) v = P.v[2][j];
      return v;
    }
    return ptab_of(ptab, p, side, q)[f];
  }
  __device__ __forceinline__ bool pivot_live(const PivotPre& P, const float2* __restrict__ ptab, int p, int side,
                                             int q) const {
    if (side == P.side) return (P.live >> q) & 1;
    return ptab_of(ptab, p, side, q)[kPtabBins - 1].x != 0.f;
  }

  template <int NB>
  __device__ __forceinline__ void accumulate(const QSlots& S, const int (&sl)[NB], const uint32_t (&nz)[2],
                                             const float2* __restrict__ ptab, int p, const PivotPre& Pre,
                                             float2 (&Cf)[NH], float2 (&Co)[NH]) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int k = sl[b];
      if (k < 0) continue;
      // wave-uniform slot fields (compile-time k chains)
      int code = 0;
      bool has_im = false;
#pragma unroll
      for (int s = 0; s < 5; ++s) {
        if (k == s) {
          code = S.code[s];
          has_im = S.im[s] != kNoSlice;
        }
      }
      const int kind = code & 3, sre = (code >> 2) & 1, qre = (code >> 3) & 3, sim = (code >> 5) & 1,
                qim = (code >> 6) & 3;
      const bool nzr = (nz[0] >> k) & 1, nzi = (nz[1] >> k) & 1;
      const float2* X = buf + 500 * b;
      const int l = lid();
      if (kind == kSlotTraj) {
        if (!(nzr && nzi)) continue;  // exactly zero in the reference
        if (sre == 0) live_f = true;
        else live_o = true;
#pragma unroll
        for (int j = 0; j < NH; ++j) {
          const int f = l + 64 * j;
          if (f <= N / 2) {
            const float2 za = X[f], zb = X[f == 0 ? 0 : N - f];
            if (sre == 0) accumulate_cross(za, zb, Cf[j]);
            else accumulate_cross(za, zb, Co[j]);
          }
        }
      } else if (kind == kSlotShared) {
        const bool la = nzr && pivot_live(Pre, ptab, p, sre, qre);
        const bool lb = has_im && nzi && pivot_live(Pre, ptab, p, sim, qim);
        if (la) {
          if (sre == 0) live_f = true;
          else live_o = true;
        }
        if (lb) {
          if (sim == 0) live_f = true;
          else live_o = true;
        }
        if (!la && !lb) continue;
#pragma unroll
        for (int j = 0; j < NH; ++j) {
          const int f = l + 64 * j;
          if (f <= N / 2) {
            const float2 za = X[f], zc = X[f == 0 ? 0 : N - f];  // zc = Z[-f]
            // R_a = (Z[f] + conj Z[-f]) / 2, R_b = (Z[f] - conj Z[-f]) / 2i; P conj(R)
            if (la) {
              const float2 ra = make_float2(0.5f * (za.x + zc.x), 0.5f * (za.y - zc.y));
              const float2 pa = pivot_bin(Pre, ptab, p, sre, qre, j, f);
              const float2 c = make_float2(pa.x * ra.x + pa.y * ra.y, pa.y * ra.x - pa.x * ra.y);
              if (sre == 0) {
                Cf[j].x += c.x;
                Cf[j].y += c.y;
              } else {
                Co[j].x += c.x;
                Co[j].y += c.y;
              }
            }
            if (lb) {
              // (Z[f] - conj Z[-f]) / 2i = ((za.y + zc.y), -(za.x - zc.x)) / 2
              const float2 rb = make_float2(0.5f * (za.y + zc.y), -0.5f * (za.x - zc.x));
              const float2 pb = pivot_bin(Pre, ptab, p, sim, qim, j, f);
              const float2 c = make_float2(pb.x * rb.x + pb.y * rb.y, pb.y * rb.x - pb.x * rb.y);
              if (sim == 0) {
                Cf[j].x += c.x;
                Cf[j].y += c.y;
              } else {
                Co[j].x += c.x;
                Co[j].y += c.y;
              }
            }
          }
        }
      }
    }
  }

  // Round 0 of the wave's next row task (tn) is loaded at the end of this task's pass 1 (DVH_Q_XPF), so
  // its global-memory latency runs under this task's pass 2 and spectral phase instead of stalling the
  // next task's first transform.
  float pxr[20], pxi[20];
  int pre_p = -1, pre_ch = -1;  // the task pxr / pxi hold (wave-uniform)

  __device__ __forceinline__ void prefetch0(const VsgArgs& A, const RowTask& tn) {
    const QSlots S = make_slots(A, tn, tn.row0);
    pre_p = tn.p;
    pre_ch = tn.ch;
    if (S.n == 0) return;
    const float* base = A.win + (int64_t)tn.p * A.pass_stride + (int64_t)tn.row0 * A.ch_stride;
    load_round(scan_rsrc_q(base, (uint32_t)((int64_t)A.R * A.ch_stride * 4)), S, 0, pxr, pxi);
  }

  // accumulated cross spectra of both sides for row task t of pass p (bins f = lane + 64 j); tn: the
  // wave's next task when has_next
  __device__ void spectra_q(const VsgArgs& A, const RowTask& t, int p, int row0, const float2* __restrict__ ptab,
                            const RowTask& tn, bool has_next, float2 (&Cf)[NH], float2 (&Co)[NH]) {
#pragma unroll
    for (int j = 0; j < NH; ++j) {
      Cf[j] = make_float2(0.f, 0.f);
      Co[j] = make_float2(0.f, 0.f);
    }
    live_f = live_o = false;
    vmax = 0;
    const bool xpf = DVH_Q_XPF && has_next;
    const bool have = DVH_Q_XPF && pre_p == t.p && pre_ch == t.ch;
    pre_p = -1;
    const QSlots S = make_slots(A, t, row0);
    if (S.n == 0) {
      if (xpf) prefetch0(A, tn);
      return;
    }
    // the pass's gather rows as one buffer resource (byte offsets < 2^31, checked on the host)
    const float* base = A.win + (int64_t)p * A.pass_stride + (int64_t)row0 * A.ch_stride;
    const __amdgpu_buffer_rsrc_t rs = scan_rsrc_q(base, (uint32_t)((int64_t)A.R * A.ch_stride * 4));
    float yr[20], yi[20];
    const bool two = S.n > 2;
    if (!have) load_round(rs, S, 0, pxr, pxi);
    PivotPre Pre;
    prefetch_pivot(S, ptab, p, Pre);
    // per-slot non-zero bits (nz[0]: re slice, nz[1]: im slice)
    uint32_t nz[2] = {0u, 0u};
    // pass 1, round 0: slots 0, 1 -> buffers 0, 1; slot 2's first 14 columns -> buffer 2
    {
      const int l = lid(), k = l / 25;
      const uint32_t bits = pass1(pxr, pxi, 0, buf + 500 * k + (l - 25 * k), true);
      const uint64_t br = __ballot(bits & 1u), bi = __ballot(bits & 2u);
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const uint64_t m = s < 2 ? (0x1ffffffull << (25 * s)) : (~0ull << 50);
        nz[0] |= (br & m) ? (1u << s) : 0u;
        nz[1] |= (bi & m) ? (1u << s) : 0u;
      }
    }
    if (two) load_round(rs, S, 1, yr, yi);  // round 1's slices, in flight under phase A
    else if (xpf) prefetch0(A, tn);
    wave_sync();
    pass2(min(S.n, 2));
    wave_sync();
    const int slA[2] = {0, S.n > 1 ? 1 : -1};
    // phase B's nz bits of slot 2 are completed below; slots 0 and 1 are final here
    accumulate<2>(S, slA, nz, ptab, p, Pre, Cf, Co);
    if (!two) return;
    wave_sync();
    // pass 1, round 1: slot 2's columns 14..24 -> buffer 2, slots 3, 4 -> buffers 0, 1
    {
      const int tau = 64 + lid(), k = tau / 25;  // 2, 3, 4 (5 for lanes 61..63: no slice, writes suppressed)
      const int bsel = k == 2 ? 2 : k - 3;
      // lanes 61..63 (tasks past slot 4) compute zeros and must not store (they would land in slot 2)
      const uint32_t bits = pass1(yr, yi, 1, buf + 500 * (bsel < 0 ? 0 : bsel) + (tau - 25 * k), k < 5);
      const uint64_t br = __ballot(bits & 1u), bi = __ballot(bits & 2u);
#pragma unroll
      for (int s = 2; s < 5; ++s) {
        const uint64_t m = s == 2 ? 0x7ffull : (0x1ffffffull << (25 * s - 64));
        nz[0] |= (br & m) ? (1u << s) : 0u;
        nz[1] |= (bi & m) ? (1u << s) : 0u;
      }
    }
    if (xpf) prefetch0(A, tn);
    wave_sync();
    pass2(3);
    wave_sync();
    const int slB[3] = {S.n > 3 ? 3 : -1, S.n > 4 ? 4 : -1, 2};
    accumulate<3>(S, slB, nz, ptab, p, Pre, Cf, Co);
    wave_sync();
  }

  static __device__ __forceinline__ __amdgpu_buffer_rsrc_t scan_rsrc_q(const void* p, uint32_t bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* pu = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(pu, 0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
  }

  __device__ const float2* inverse(const float2 (&Cf)[NH], const float2 (&Co)[NH]) {
    store_conj_hermitian<EngQ500>(buf, Cf, Co, lane);
    wave_sync();
    return FftPlan<N>::T::run(buf, buf + N, tw, lane);
  }

  __device__ float2 twiddle(int m) const { return tw[m]; }

  __device__ float2 c(const float2* Y, int k, int) const {
    const float2 v = Y[k];
    return make_float2(v.x, -v.y);
  }
};

}  // namespace dvh
