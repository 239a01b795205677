// Correlation-engine variants measured on MI355X and NOT built into libdvh (kept for reference; see
// DESIGN.md "measured and rejected").  They were selectable in round 1 through DVH_VSG500 / DVH_TW_REG
// and are not compiled anywhere now; they depend on das_diff_veh_amd/csrc/vsg_engines.h.
//   Eng500   20 x 25 register transform, LDS-DMA staged slices (7-wave blocks)
//   EngP500  two sub-windows per pass, in-place 20 x 5 x 5 (0.54 vs 0.48 ms for EngF500)
//   EngF500 register-twiddle members (DVH_TW_REG: 0.494 / 0.622 vs 0.476 ms)
#pragma once
#include "vsg_engines.h"

namespace dvh {

// ------------------------------------------------------------------------------------------------
// 20 x 25 register transform for N = 500.
//   stage 1 (radix 20, span 1):  butterfly i < 25 reads x[i + 25 t], t < 20, writes X1[20 i + q]
//   stage 2 (radix 25, span 20): butterfly k < 20 reads X1[k + 20 t] * W500^(t k), t < 25,
//                                writes X[k + 20 q] (natural order, in place of what it read)
// Stage buffers use the rotation swizzle n = 20 a + b -> 20 a + (a + b) mod 20 (bank spread for the
// stage-1 stores, stage-2 accesses stay contiguous per row).

__device__ __forceinline__ float2 tw20(int m) { return make_float2(Tw20::c[m % 20], Tw20::s[m % 20]); }
__device__ __forceinline__ float2 tw25(int m) { return make_float2(Tw25::c[m % 25], Tw25::s[m % 25]); }

// in-place natural-order DFT of length 20 (4 x 5 Cooley-Tukey, n = 5 n1 + n2, k = k1 + 4 k2)
__device__ __forceinline__ void dft20(float2 (&x)[20]) {
  float2 y[4][5];
#pragma unroll
  for (int n2 = 0; n2 < 5; ++n2) {
    float2 v[4] = {x[n2], x[5 + n2], x[10 + n2], x[15 + n2]};
    Dft<4>::run(v);
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) y[k1][n2] = (n2 * k1 == 0) ? v[k1] : cmul(v[k1], tw20(n2 * k1));
  }
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    float2 u[5] = {y[k1][0], y[k1][1], y[k1][2], y[k1][3], y[k1][4]};
    Dft<5>::run(u);
#pragma unroll
    for (int k2 = 0; k2 < 5; ++k2) x[k1 + 4 * k2] = u[k2];
  }
}

// in-place natural-order DFT of length 25 (5 x 5, n = 5 n1 + n2, k = k1 + 5 k2)
__device__ __forceinline__ void dft25(float2 (&x)[25]) {
  float2 y[5][5];
#pragma unroll
  for (int n2 = 0; n2 < 5; ++n2) {
    float2 v[5] = {x[n2], x[5 + n2], x[10 + n2], x[15 + n2], x[20 + n2]};
    Dft<5>::run(v);
#pragma unroll
    for (int k1 = 0; k1 < 5; ++k1) y[k1][n2] = (n2 * k1 == 0) ? v[k1] : cmul(v[k1], tw25(n2 * k1));
  }
#pragma unroll
  for (int k1 = 0; k1 < 5; ++k1) {
    float2 u[5] = {y[k1][0], y[k1][1], y[k1][2], y[k1][3], y[k1][4]};
    Dft<5>::run(u);
#pragma unroll
    for (int k2 = 0; k2 < 5; ++k2) x[k1 + 5 * k2] = u[k2];
  }
}

// Stage buffers: natural index n = 20 a + b stored at 21 a + b (row pad: conflict-free stage-1
// stores, stage-2 column accesses at compile-time immediate offsets); buffers kBuf apart, kBuf = 20
// mod 32 so the two sub-windows a 32-lane half touches use disjoint banks.
__device__ __forceinline__ int pad500(int n) {
  const int a = n / 20;
  return n + a;
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

struct Eng500 {
  static constexpr int N = 500;
  static constexpr int NFFT = 500;
  static constexpr int NJ = 8;
  static constexpr int NH = 4;
  static constexpr int kWaves = 7;                                              // 448-thread blocks
  static constexpr int kSlab = 1024;                                            // floats per channel (64-lane DMA granules)
  static constexpr int kBuf = 532;                                              // float2 per stage buffer
  static constexpr size_t kBlockBytes = sizeof(float2) * N;                     // W500 twiddle table
  static constexpr size_t kWaveBytes = 2 * kSlab * sizeof(float) + 3 * kBuf * sizeof(float2);  // 20960 B
  float2* tw;
  float* sp;   // pivot slice
  float* sr;   // receiver slice
  float2* B;   // 3 stage buffers
  int lane;
  bool pref;   // slab already holds the first slice of the next task
  bool live_f, live_o;

  __device__ Eng500(char* lds, int wave, int lane_) : lane(lane_), pref(false), live_f(false), live_o(false) {
    tw = reinterpret_cast<float2*>(lds);
    char* base = lds + kBlockBytes + (size_t)wave * kWaveBytes;
    sp = reinterpret_cast<float*>(base);
    sr = sp + kSlab;
    B = reinterpret_cast<float2*>(base + 2 * kSlab * sizeof(float));
  }
  static __device__ void block_init(char* lds) {
    float2* t = reinterpret_cast<float2*>(lds);
    for (int m = threadIdx.x; m < N; m += blockDim.x) t[m] = kTw500[m];
  }

  // slices of a task: side f in groups of <= 3 sub-windows, then side o
  static __device__ __forceinline__ int n_groups(int nwin) { return (nwin + 2) / 3; }

  __device__ __forceinline__ void slice_of(const RowTask& t, int g, int hop, int& a, int& ns, bool& fwd) const {
    const int gf = n_groups(t.nwin_f);
    fwd = g < gf;
    const int gg = fwd ? g : g - gf;
    const int nw = fwd ? t.nwin_f : t.nwin_o;
    ns = min(3, nw - 3 * gg);
    a = (fwd ? t.a_f : t.a_o) + 3 * gg * hop;
  }

  // asynchronous global -> LDS copy of span samples of both channels (lane-linear destination)
  __device__ __forceinline__ void dma(const RowTask& t, int a, int span) {
#pragma unroll 1
    for (int m = 0; m < (span + 63) / 64; ++m) {
      const int n = min(64 * m + lane, span - 1);
      __builtin_amdgcn_global_load_lds((glb_void_t*)(t.piv + a + n), (lds_void_t*)(sp + 64 * m), 4, 0, 0);
      __builtin_amdgcn_global_load_lds((glb_void_t*)(t.rcv + a + n), (lds_void_t*)(sr + 64 * m), 4, 0, 0);
    }
  }
  __device__ __forceinline__ void dma_slice(const RowTask& t, int g, int w, int hop) {
    int a, ns;
    bool fwd;
    slice_of(t, g, hop, a, ns, fwd);
    dma(t, a, (ns - 1) * hop + w);
  }

  // stage 1 for ns sub-windows at slab offsets s * hop (radix-20 butterflies, 2 rounds); returns the
  // mask of sub-windows whose pivot and receiver slices both hold a non-zero sample
  __device__ __forceinline__ uint32_t stage1(int ns, int hop, float2* out) const {
    uint32_t live = 0;
#pragma unroll 1
    for (int r = 0; r < 2; ++r) {
      const int tt = lane + 64 * r;
      const int s = tt / 25, i = tt - 25 * (tt / 25);
      uint32_t bp = 0, br = 0;
      if (s < ns) {
        const float* pp = sp + s * hop + i;
        const float* rr = sr + s * hop + i;
        // DFT20 over t = 5 n1 + n2 of z[i + 25 t], output q = k1 + 4 k2, streamed per n2 column
        float2 y[4][5];
#pragma unroll
        for (int n2 = 0; n2 < 5; ++n2) {
          float2 v[4];
#pragma unroll
          for (int n1 = 0; n1 < 4; ++n1) {
            v[n1] = make_float2(pp[25 * (5 * n1 + n2)], rr[25 * (5 * n1 + n2)]);
            bp |= nzbits(v[n1].x);
            br |= nzbits(v[n1].y);
          }
          Dft<4>::run(v);
#pragma unroll
          for (int k1 = 0; k1 < 4; ++k1) y[k1][n2] = (n2 * k1 == 0) ? v[k1] : cmul(v[k1], tw20(n2 * k1));
        }
        float2* o = out + kBuf * s + 21 * i;
#pragma unroll
        for (int k1 = 0; k1 < 4; ++k1) {
          float2 u[5] = {y[k1][0], y[k1][1], y[k1][2], y[k1][3], y[k1][4]};
          Dft<5>::run(u);
#pragma unroll
          for (int k2 = 0; k2 < 5; ++k2) o[k1 + 4 * k2] = u[k2];
        }
      }
      // lanes of sub-window s in this round: tt in [25 s, 25 s + 25)
      const uint64_t mp = __ballot(bp != 0), mr = __ballot(br != 0);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int lo = max(25 * q - 64 * r, 0), hi = min(25 * q + 25 - 64 * r, 64);
        if (lo < hi) {
          const uint64_t rng = (hi - lo == 64 ? ~0ull : ((1ull << (hi - lo)) - 1)) << lo;
          if ((mp & rng) && (mr & rng)) live |= 1u << q;
        }
      }
    }
    return live;
  }

  // stage 2 in place on ns buffers (radix-25 butterflies with W500 twiddles, 1 round)
  __device__ __forceinline__ void stage2(int ns, float2* buf) const {
    const int s = lane / 20, k = lane - 20 * (lane / 20);
    if (s < ns) {
      float2* b = buf + kBuf * s + k;
      // DFT25 over t = 5 n1 + n2 of x[t] = X1[k + 20 t] * W500^(t k), output q = k1 + 5 k2,
      // streamed one n2 column at a time to bound the live registers
      float2 y[5][5];
#pragma unroll
      for (int n2 = 0; n2 < 5; ++n2) {
        float2 v[5];
#pragma unroll
        for (int n1 = 0; n1 < 5; ++n1) {
          const int t = 5 * n1 + n2;
          v[n1] = t == 0 ? b[0] : cmul(b[21 * t], tw[t * k]);
        }
        Dft<5>::run(v);
#pragma unroll
        for (int k1 = 0; k1 < 5; ++k1) y[k1][n2] = (n2 * k1 == 0) ? v[k1] : cmul(v[k1], tw25(n2 * k1));
      }
#pragma unroll
      for (int k1 = 0; k1 < 5; ++k1) {
        float2 u[5] = {y[k1][0], y[k1][1], y[k1][2], y[k1][3], y[k1][4]};
        Dft<5>::run(u);
#pragma unroll
        for (int k2 = 0; k2 < 5; ++k2) b[21 * (k1 + 5 * k2)] = u[k2];
      }
    }
  }

  __device__ __forceinline__ void extract(int ns, uint32_t live, float2 (&C)[NH]) const {
#pragma unroll 1
    for (int s = 0; s < ns; ++s) {
      if (!((live >> s) & 1u)) continue;
      const float2* b = B + kBuf * s;
#pragma unroll
      for (int j = 0; j < NH; ++j) {
        const int f = lane + 64 * j;
        if (f <= N / 2) accumulate_cross(b[pad500(f)], b[pad500(f == 0 ? 0 : N - f)], C[j]);
      }
    }
  }

  __device__ void spectra(const RowTask& t, const RowTask& nt, bool has_next, int w, int hop, float2 (&Cf)[NH],
                          float2 (&Co)[NH]) {
#pragma unroll
    for (int j = 0; j < NH; ++j) {
      Cf[j] = make_float2(0.f, 0.f);
      Co[j] = make_float2(0.f, 0.f);
    }
    const int ng = n_groups(t.nwin_f) + n_groups(t.nwin_o);
    bool next_issued = false;
    live_f = live_o = false;
    if (!pref && ng > 0) dma_slice(t, 0, w, hop);
    pref = false;
    for (int g = 0; g < ng; ++g) {
      int a, ns;
      bool fwd;
      slice_of(t, g, hop, a, ns, fwd);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      wave_sync();
      const uint32_t lm = stage1(ns, hop, B);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      wave_sync();
      // the slab is free: start the next slice's copy under stage 2 / extraction / inverse FFT
      if (g + 1 < ng) {
        dma_slice(t, g + 1, w, hop);
      } else if (has_next && (n_groups(nt.nwin_f) + n_groups(nt.nwin_o)) > 0) {
        dma_slice(nt, 0, w, hop);
        next_issued = true;
      }
      stage2(ns, B);
      wave_sync();
      if (fwd) {
        extract(ns, lm, Cf);
        live_f |= lm != 0;
      } else {
        extract(ns, lm, Co);
        live_o |= lm != 0;
      }
      wave_sync();
    }
    if (!next_issued && has_next && (n_groups(nt.nwin_f) + n_groups(nt.nwin_o)) > 0) {
      dma_slice(nt, 0, w, hop);
      next_issued = true;
    }
    pref = next_issued;
  }

  // inverse transform of W = Cf + i Co through conj(FFT(conj(W))): natural input in B[0, 500),
  // stage 1 -> buffer 1 (padded), stage 2 in place
  static __device__ __forceinline__ int bin(int lane, int j) {
    const int f = lane + 64 * j;
    return f <= N / 2 ? f : -1;
  }
  static __device__ __forceinline__ int slot(int n) { return n; }

  __device__ const float2* inverse(const float2 (&Cf)[NH], const float2 (&Co)[NH]) {
    store_conj_hermitian<Eng500>(B, Cf, Co, lane);
    wave_sync();
    if (lane < 25) {
      float2 x[20];
#pragma unroll
      for (int t = 0; t < 20; ++t) x[t] = B[lane + 25 * t];
      dft20(x);
      float2* o = B + kBuf + 21 * lane;
#pragma unroll
      for (int q = 0; q < 20; ++q) o[q] = x[q];
    }
    wave_sync();
    stage2(1, B + kBuf);
    wave_sync();
    return B + kBuf;
  }

  __device__ const float2* correlate(const RowTask& t, const RowTask& nt, bool has_next, int w, int hop) {
    float2 Cf[NH], Co[NH];
    spectra(t, nt, has_next, w, hop, Cf, Co);
    return inverse(Cf, Co);
  }

  __device__ float2 twiddle(int m) const { return tw[m]; }

  __device__ float2 c(const float2* Y, int k, int) const {
    const float2 v = Y[pad500(k)];
    return make_float2(v.x, -v.y);
  }
};


// EngP500: N = w = 500 with TWO sub-windows of the row task per transform pass (lanes 0-31 carry
// transform 0, lanes 32-63 transform 1) and one LDS round trip fewer than EngF500:
//   500 = 20 x 5 x 5, n = n2 + 25 n1, f = k1 + 20 j1 + 100 j2
//   stage 1  lane n2 < 25 of its half: the 20 samples x[n2 + 25 n1] straight from global memory,
//            a radix-20 (4 x 5, compile-time twiddles) in registers, x W500^(n2 k1) by recurrence,
//            20 LDS writes                                      (25 of 32 lanes busy)
//   stage 2  200 radix-5 butterflies (k1, m2) over m1, x W25^(m2 j1), written back IN PLACE
//            (the butterfly's five slots), 4 rounds
//   stage 3  the last radix-5 (k1, j1) over m2: bins b + 100 j2 of butterfly b = k1 + 20 j1 --
//            EngF500's last-stage layout, so the half-spectrum slots, partner pairing and the
//            cross-spectrum accumulation are EngF500's (lane l <= 50: butterflies l and 100 - l)
// Per transform the LDS traffic is 500 writes + 500 reads fewer than EngF500's three round trips;
// each transform owns one in-place buffer of 27 x 20 slots (pos = 27 k1 + n2: conflict-free stage-1
// stores, <= 1.6-way reads).
#ifndef DVH_P500_S2UNROLL
#define DVH_P500_S2UNROLL 0
#endif
#ifndef DVH_P500_NOPF
#define DVH_P500_NOPF 0
#endif
#ifndef DVH_P500_PAD
#define DVH_P500_PAD 27
#endif
struct EngP500 : EngF500 {
  static constexpr int S = DVH_P500_PAD;
  static constexpr int kBuf = 19 * S + 25;                      // slots per transform buffer
  static constexpr size_t kWaveBytes = sizeof(float2) * 2 * kBuf;  // two in-place buffers
  float2* buf1;

  __device__ EngP500(char* lds, int wave, int lane_) : EngF500(lds, wave, lane_) {
    bufA = reinterpret_cast<float2*>(lds + kBlockBytes + (size_t)wave * kWaveBytes);
    bufB = bufA + kBuf;
    buf1 = bufB;
  }
  static __device__ __forceinline__ int pos(int n2, int k1) { return S * k1 + n2; }

  // W20^m, m <= 12 (the q r products of the radix-20): (cos, -sin)(2 pi m / 20)
  static __device__ __forceinline__ float2 w20(int m) {
    constexpr float c[13] = {1.f, 0.951056516f, 0.809016994f, 0.587785252f, 0.309016994f, 0.f, -0.309016994f,
                             -0.587785252f, -0.809016994f, -0.951056516f, -1.f, -0.951056516f, -0.809016994f};
    constexpr float n[13] = {0.f, -0.309016994f, -0.587785252f, -0.809016994f, -0.951056516f, -1.f, -0.951056516f,
                             -0.809016994f, -0.587785252f, -0.309016994f, 0.f, 0.309016994f, 0.587785252f};
    return make_float2(c[m], n[m]);
  }

  // the pair's samples: lane half h -> sub-window starting at a_h, n2 = lane & 31 < 25
  __device__ __forceinline__ void load2(const RowTask& t, int a0, int a1, bool two, float (&zp)[20],
                                        float (&zr)[20]) const {
    const int h = lane >> 5, n2 = lane & 31;
    const bool ok = n2 < 25 && (h == 0 || two);
    const int a = (h ? a1 : a0) + n2;
#pragma unroll
    for (int n1 = 0; n1 < 20; ++n1) {
      zp[n1] = ok ? t.piv[a + 25 * n1] : 0.f;
      zr[n1] = ok ? t.rcv[a + 25 * n1] : 0.f;
    }
  }

  __device__ __forceinline__ void stage1(const float (&zp)[20], const float (&zr)[20], bool two) const {
    const int h = lane >> 5, n2 = lane & 31;
    if (n2 < 25 && (h == 0 || two)) {
      float2 A[20];  // A[r + 4 s]
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        float2 a[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) a[p] = make_float2(zp[5 * p + q], zr[5 * p + q]);
        Dft<4>::run(a);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = q * r;
          float2 v = a[r];
          if (m == 5) v = mul_mi(v);
          else if (m == 10) v = make_float2(-v.x, -v.y);
          else if (m != 0) v = cmul(v, w20(m));
          A[r + 4 * q] = v;  // D[q][r], parked in A until the radix-5 pass
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // in place: A[r + 4 s] <- radix-5 over q of A[r + 4 q]
        float2 e[5];
#pragma unroll
        for (int q = 0; q < 5; ++q) e[q] = A[r + 4 * q];
        Dft<5>::run(e);
#pragma unroll
        for (int s2 = 0; s2 < 5; ++s2) A[r + 4 * s2] = e[s2];
      }
      float2* buf = h ? buf1 : bufA;
      const float2 w1 = tw[n2];
      float2 w = w1;
      buf[pos(n2, 0)] = A[0];
#pragma unroll
      for (int k1 = 1; k1 < 20; ++k1) {
        buf[pos(n2, k1)] = cmul(A[k1], w);
        if (k1 < 19) w = cmul(w, w1);
      }
    }
  }

  // stage 2 over both transforms: task T = 64 r + lane < 100 (1 + two): (k1, m2) = (u % 20, u / 20)
  __device__ __forceinline__ void stage2(bool two) const {
    const int nt = two ? 200 : 100;
    auto round = [&](int r) {
      const int T = 64 * r + lane;
      if (T < nt) {
        const int f = T >= 100, u = T - 100 * f;
        const int k1 = u % 20, m2 = u / 20;
        float2* buf = f ? buf1 : bufA;
        float2 x[5];
#pragma unroll
        for (int m1 = 0; m1 < 5; ++m1) x[m1] = buf[pos(m2 + 5 * m1, k1)];
        Dft<5>::run(x);
        const float2 w1 = tw[20 * m2];  // W25^m2
        float2 w = w1;
#pragma unroll
        for (int j1 = 1; j1 < 5; ++j1) {
          x[j1] = cmul(x[j1], w);
          if (j1 < 4) w = cmul(w, w1);
        }
#pragma unroll
        for (int j1 = 0; j1 < 5; ++j1) buf[pos(m2 + 5 * j1, k1)] = x[j1];
      }
    };
#if DVH_P500_S2UNROLL
#pragma unroll
#else
#pragma unroll 1
#endif
    for (int r = 0; r < 4; ++r) round(r);
  }

  // last radix-5 of butterfly b (k1 = b % 20, j1 = b / 20): X[b + 100 j2]
  __device__ __forceinline__ void last_p(const float2* buf, int b, float2 (&x)[5]) const {
    const int k1 = b % 20, j1 = b / 20;
#pragma unroll
    for (int m2 = 0; m2 < 5; ++m2) x[m2] = buf[pos(5 * j1 + m2, k1)];
    Dft<5>::run(x);
  }

  // stage 3 of transform buf into the half-spectrum slots (EngF500::finish_with's pairing)
  template <class F>
  __device__ __forceinline__ void finish_p(const float2* buf, F&& acc) const {
    if (lane <= 50) {
      float2 XA[5], XB[5];
      last_p(buf, lane, XA);
      const bool pair = lane >= 1 && lane <= 49;
      last_p(buf, pair ? 100 - lane : lane, XB);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const float2 p0 = XA[(5 - j) % 5], p50 = XA[4 - j], pb = XB[4 - j];
        float2 pa;
        pa.x = lane == 0 ? p0.x : (lane == 50 ? p50.x : pb.x);
        pa.y = lane == 0 ? p0.y : (lane == 50 ? p50.y : pb.y);
        acc(j, XA[j], pa);
      }
      if (pair) {
#pragma unroll
        for (int q = 0; q < 2; ++q) acc(3 + q, XB[q], XA[4 - q]);
      }
    }
  }

  __device__ void spectra(const RowTask& t, const RowTask&, bool, int, int hop, float2 (&Cf)[NH], float2 (&Co)[NH]) {
    const int nq = t.nwin_f + t.nwin_o;
    float zp[20], zr[20];
#pragma unroll
    for (int j = 0; j < NH; ++j) {
      Cf[j] = make_float2(0.f, 0.f);
      Co[j] = make_float2(0.f, 0.f);
    }
    live_f = live_o = false;
    auto start = [&](int q) { return q < t.nwin_f ? t.a_f + q * hop : t.a_o + (q - t.nwin_f) * hop; };
    if (nq > 0) load2(t, start(0), nq > 1 ? start(1) : 0, nq > 1, zp, zr);
    for (int q = 0; q < nq; q += 2) {
      const bool two = q + 1 < nq;
      uint32_t bp = 0, br = 0;
#pragma unroll
      for (int j = 0; j < 20; ++j) {
        bp |= nzbits(zp[j]);
        br |= nzbits(zr[j]);
      }
      const uint64_t mp = __ballot(bp != 0), mr = __ballot(br != 0);
      const bool live0 = (mp & 0xffffffffull) && (mr & 0xffffffffull);
      const bool live1 = two && (mp >> 32) && (mr >> 32);
      if (live0 || live1) stage1(zp, zr, two);
#if !DVH_P500_NOPF
      if (q + 2 < nq) load2(t, start(q + 2), q + 3 < nq ? start(q + 3) : 0, q + 3 < nq, zp, zr);
#endif
      if (!(live0 || live1)) continue;  // exactly zero in the reference
      wave_sync();
      stage2(two);
      wave_sync();
      if (live0) {
        if (q < t.nwin_f) {
          live_f = true;
          finish_p(bufA, [&](int j, float2 a, float2 b) { accumulate_cross(a, b, Cf[j]); });
        } else {
          live_o = true;
          finish_p(bufA, [&](int j, float2 a, float2 b) { accumulate_cross(a, b, Co[j]); });
        }
      }
      if (live1) {
        if (q + 1 < t.nwin_f) {
          live_f = true;
          finish_p(buf1, [&](int j, float2 a, float2 b) { accumulate_cross(a, b, Cf[j]); });
        } else {
          live_o = true;
          finish_p(buf1, [&](int j, float2 a, float2 b) { accumulate_cross(a, b, Co[j]); });
        }
      }
      wave_sync();
#if DVH_P500_NOPF
      if (q + 2 < nq) load2(t, start(q + 2), q + 3 < nq ? start(q + 3) : 0, q + 3 < nq, zp, zr);
#endif
    }
  }

  __device__ const float2* correlate(const RowTask& t, const RowTask& nt, bool has_next, int w, int hop) {
    float2 Cf[NH], Co[NH];
    spectra(t, nt, has_next, w, hop, Cf, Co);
    return inverse(Cf, Co);
  }
};


/* EngF500 register-twiddle fragment (DVH_TW_REG):
  bool live_f, live_o;
#if DVH_TW_REG
  // this lane's twiddle powers of stages 2, 3 (two rounds each) and of its last-stage butterflies
  // k = lane and 100 - lane, read once from the table: the lane -> butterfly map is the same for
  // every transform of the wave, so the per-butterfly power recurrences disappear
  float2 w2[2][4], w3[2][4], wA[4], wB[4];
#endif

  __device__ EngF500(char* lds, int wave, int lane_) : lane(lane_), live_f(false), live_o(false) {
    tw = reinterpret_cast<float2*>(lds);
    bufA = reinterpret_cast<float2*>(lds + kBlockBytes + (size_t)wave * kWaveBytes);
    bufB = bufA + N;
#if DVH_TW_REG
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = lane + 64 * r, k2 = i % 4, k3 = i % 20;
#pragma unroll
      for (int t = 1; t < 5; ++t) {
        w2[r][t - 1] = tw[(t * k2 * 25) % N];
        w3[r][t - 1] = tw[(t * k3 * 5) % N];
      }
    }
    const int kb = (lane >= 1 && lane <= 49) ? 100 - lane : lane;
#pragma unroll
    for (int t = 1; t < 5; ++t) {
      wA[t - 1] = tw[(t * lane) % N];
      wB[t - 1] = tw[(t * kb) % N];
    }
#endif
  }

#if DVH_TW_REG
  // radix-5 Stockham stage of span Ls with this lane's register twiddles w[round][t - 1]
  template <int Ls>
  __device__ __forceinline__ void stage5(const float2* __restrict__ in, float2* __restrict__ out,
                                         const float2 (&w)[2][4]) const {
    constexpr int R = 5, NB = N / R;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = lane + 64 * r;
      if (i < NB) {
        const int k = i % Ls;
        float2 a[R];
#pragma unroll
        for (int t = 0; t < R; ++t) a[t] = lds_ld(in, i + t * NB);
#pragma unroll
        for (int t = 1; t < R; ++t) a[t] = cmul(a[t], w[r][t - 1]);
        Dft<R>::run(a);
        const int base = (i - k) * R + k;
#pragma unroll
        for (int q = 0; q < R; ++q) out[base + q * Ls] = a[q];
      }
    }
  }
  __device__ __forceinline__ void last_bfly_reg(const float2* src, int k, const float2 (&w)[4], float2 (&x)[5]) const {
#pragma unroll
    for (int t = 0; t < 5; ++t) x[t] = lds_ld(src, k + 100 * t);
#pragma unroll
    for (int t = 1; t < 5; ++t) x[t] = cmul(x[t], w[t - 1]);
    Dft<5>::run(x);
  }
#endif
*/

}  // namespace dvh
