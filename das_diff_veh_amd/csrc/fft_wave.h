// Wave-resident Stockham FFT for gfx950 (CDNA4, wave64).
//
// One 64-lane wave owns one complex transform of length N held in two LDS buffers (ping-pong);
// stages are radix 2/3/4/5 with compile-time plans, so every loop bound and index stride folds.
// Forward transform X[f] = sum_n x[n] exp(-2*pi*i*f*n/N); the inverse is obtained by the caller
// through conj(FFT(conj(.))).  Twiddles exp(-2*pi*i*m/N) live in a block-shared LDS table.
//
// Stage (radix R, span Ls): butterfly i in [0, N/R), k = i % Ls, inputs in[i + t*N/R],
// twiddle exp(-2*pi*i*t*k/(Ls*R)) = tw[t*k*N/(Ls*R)], R-point DFT, outputs out[(i-k)*R + k + q*Ls].
// After the last stage the result is in natural order (self-sorting).
#pragma once
#include <hip/hip_runtime.h>

// One LDS complex read (the compiler pairs neighbouring ones into ds_read2_b64; single reads measured slower on the
// stack kernels despite the LDS cycles they save: their address arithmetic costs more).
__device__ __forceinline__ float2 lds_ld(const float2* p, int idx) { return p[idx]; }

namespace dvh {

// Complex arithmetic as plain f32 ops (packed v_pk_*_f32 forms measured no faster on gfx950).
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
// -i * a and +i * a
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }
__device__ __forceinline__ float2 mul_pi(float2 a) { return make_float2(-a.y, a.x); }
// m + (-i) u = (m.x + u.y, m.y - u.x) and m + i u = (m.x - u.y, m.y + u.x)
__device__ __forceinline__ float2 add_mi(float2 m, float2 u) { return cadd(m, mul_mi(u)); }
__device__ __forceinline__ float2 add_pi(float2 m, float2 u) { return cadd(m, mul_pi(u)); }

// Orders this wave's LDS accesses across lanes (a single wave executes LDS ops in order; the
// fences stop the compiler from moving loads/stores across the stage boundary).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int R> struct Dft;

template <> struct Dft<2> {
  static __device__ __forceinline__ void run(float2 (&a)[2]) {
    const float2 t = a[1];
    a[1] = csub(a[0], t);
    a[0] = cadd(a[0], t);
  }
};

template <> struct Dft<3> {
  static __device__ __forceinline__ void run(float2 (&a)[3]) {
    constexpr float c = -0.5f, s = 0.86602540378443864676f;
    const float2 t = cadd(a[1], a[2]);
    const float2 d = csub(a[1], a[2]);
    const float2 m = make_float2(a[0].x + c * t.x, a[0].y + c * t.y);
    const float2 u = cscale(d, s);
    a[0] = cadd(a[0], t);
    a[1] = add_mi(m, u);
    a[2] = add_pi(m, u);
  }
};

template <> struct Dft<4> {
  static __device__ __forceinline__ void run(float2 (&a)[4]) {
    const float2 s02 = cadd(a[0], a[2]), d02 = csub(a[0], a[2]);
    const float2 s13 = cadd(a[1], a[3]), d13 = csub(a[1], a[3]);
    a[0] = cadd(s02, s13);
    a[2] = csub(s02, s13);
    a[1] = add_mi(d02, d13);
    a[3] = add_pi(d02, d13);
  }
};

template <> struct Dft<5> {
  static __device__ __forceinline__ void run(float2 (&a)[5]) {
    constexpr float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
    constexpr float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
    const float2 t1 = cadd(a[1], a[4]), t2 = cadd(a[2], a[3]);
    const float2 t3 = csub(a[1], a[4]), t4 = csub(a[2], a[3]);
    const float2 m1 = make_float2(a[0].x + c1 * t1.x + c2 * t2.x, a[0].y + c1 * t1.y + c2 * t2.y);
    const float2 m2 = make_float2(a[0].x + c2 * t1.x + c1 * t2.x, a[0].y + c2 * t1.y + c1 * t2.y);
    const float2 u1 = make_float2(s1 * t3.x + s2 * t4.x, s1 * t3.y + s2 * t4.y);
    const float2 u2 = make_float2(s2 * t3.x - s1 * t4.x, s2 * t3.y - s1 * t4.y);
    a[0] = cadd(a[0], cadd(t1, t2));
    a[1] = add_mi(m1, u1);
    a[4] = add_pi(m1, u1);
    a[2] = add_mi(m2, u2);
    a[3] = add_pi(m2, u2);
  }
};

// 16-point DFT in registers, natural order in and out (4 x 4: radix-4 DFTs over t2 of a[t1 + 4 t2], twiddles
// W16^(t1 q2), radix-4 DFTs over t1 into a[q2 + 4 q1]).  HALF: only a[0..7] are non-zero (a zero-padded input).
template <bool HALF = false>
__device__ __forceinline__ void dft16(float2 (&a)[16]) {
  constexpr float c8 = 0.92387953251128675613f, s8 = 0.38268343236508977173f, r2 = 0.70710678118654752440f;
  float2 y[4][4];
#pragma unroll
  for (int t1 = 0; t1 < 4; ++t1) {
    float2 c[4];
    if (HALF) {  // DFT4 of (a, b, 0, 0)
      const float2 u = a[t1], v = a[t1 + 4];
      c[0] = cadd(u, v);
      c[1] = add_mi(u, v);
      c[2] = csub(u, v);
      c[3] = add_pi(u, v);
    } else {
      c[0] = a[t1];
      c[1] = a[t1 + 4];
      c[2] = a[t1 + 8];
      c[3] = a[t1 + 12];
      Dft<4>::run(c);
    }
#pragma unroll
    for (int q2 = 0; q2 < 4; ++q2) y[t1][q2] = c[q2];
  }
  // W16^m, m = t1 q2: 1 (c8, -s8), 2 (r2, -r2), 3 (s8, -c8), 4 (-i), 6 (-r2, -r2), 9 (-c8, s8)
  y[1][1] = cmul(y[1][1], make_float2(c8, -s8));
  y[1][2] = cmul(y[1][2], make_float2(r2, -r2));
  y[1][3] = cmul(y[1][3], make_float2(s8, -c8));
  y[2][1] = cmul(y[2][1], make_float2(r2, -r2));
  y[2][2] = mul_mi(y[2][2]);
  y[2][3] = cmul(y[2][3], make_float2(-r2, -r2));
  y[3][1] = cmul(y[3][1], make_float2(s8, -c8));
  y[3][2] = cmul(y[3][2], make_float2(-r2, -r2));
  y[3][3] = cmul(y[3][3], make_float2(-c8, s8));
#pragma unroll
  for (int q2 = 0; q2 < 4; ++q2) {
    float2 c[4] = {y[0][q2], y[1][q2], y[2][q2], y[3][q2]};
    Dft<4>::run(c);
#pragma unroll
    for (int q1 = 0; q1 < 4; ++q1) a[q2 + 4 * q1] = c[q1];
  }
}

// a[t] *= w^t, t = 1..15, from w^1, w^4, w^8 (table reads: every power within three roundings of the table's)
__device__ __forceinline__ void twiddle16(float2 (&a)[16], float2 w1, float2 w4, float2 w8) {
  const float2 w2 = cmul(w1, w1), w3 = cmul(w2, w1);
  const float2 lo[4] = {make_float2(1.f, 0.f), w1, w2, w3};
#pragma unroll
  for (int t = 1; t < 16; ++t) {
    const int h = t >> 2, l = t & 3;
    float2 w = h == 0 ? lo[l] : (h == 1 ? w4 : (h == 2 ? w8 : cmul(w8, w4)));
    if (h > 0 && l > 0) w = cmul(w, lo[l]);
    a[t] = cmul(a[t], w);
  }
}

template <int N, int Ls, int R>
__device__ __forceinline__ void stockham_stage(const float2* __restrict__ in, float2* __restrict__ out,
                                               const float2* __restrict__ tw, int lane) {
  constexpr int NB = N / R;
  constexpr int TWS = N / (Ls * R);
  static_assert(N % (Ls * R) == 0, "plan does not divide N");
  auto round = [&](int i0) {
    const int i = i0 + lane;
    if (NB % 64 == 0 || i < NB) {
      const int k = i % Ls;
      float2 a[R];
#pragma unroll
      for (int t = 0; t < R; ++t) a[t] = lds_ld(in, i + t * NB);
      if (Ls > 1) {
        // one table read per butterfly, powers by recurrence (LDS reads are the scarcer resource; per-power table
        // reads measured 8 % slower)
        const float2 w1 = tw[k * TWS];
        float2 wt = w1;
#pragma unroll
        for (int t = 1; t < R; ++t) {
          a[t] = cmul(a[t], wt);
          if (t + 1 < R) wt = cmul(wt, w1);
        }
      }
      Dft<R>::run(a);
      const int base = (i - k) * R + k;
#pragma unroll
      for (int q = 0; q < R; ++q) out[base + q * Ls] = a[q];
    }
  };
  // Short radix <= 5 stages (<= 2 rounds of 64 butterflies) are unrolled so that the second round's LDS reads
  // overlap the first round's arithmetic (measured -8 % on the N = 500 stack kernel); long ones stay
  // rolled (code size, registers).
  if constexpr (NB <= 128 && R <= 5) {
#pragma unroll
    for (int i0 = 0; i0 < NB; i0 += 64) round(i0);
  } else {
#pragma unroll 1
    for (int i0 = 0; i0 < NB; i0 += 64) round(i0);
  }
}

template <int N, int Ls, int... Rs> struct Stockham;

template <int N, int Ls> struct Stockham<N, Ls> {
  static_assert(Ls == N, "radix plan must multiply to N");
  static __device__ __forceinline__ float2* run(float2* in, float2*, const float2*, int) { return in; }
};

template <int N, int Ls, int R, int... Rs> struct Stockham<N, Ls, R, Rs...> {
  static __device__ __forceinline__ float2* run(float2* in, float2* out, const float2* tw, int lane) {
    stockham_stage<N, Ls, R>(in, out, tw, lane);
    wave_sync();
    return Stockham<N, Ls * R, Rs...>::run(out, in, tw, lane);
  }
};

// Plans used by the library.  N is the transform length; PAD means the correlation is computed as a
// zero-padded linear correlation (N >= 2w - 1) and folded back to the circular one in the epilogue.
template <int N> struct FftPlan;
template <> struct FftPlan<250> { using T = Stockham<250, 1, 2, 5, 5, 5>; };
template <> struct FftPlan<500> { using T = Stockham<500, 1, 4, 5, 5, 5>; };
template <> struct FftPlan<1000> { using T = Stockham<1000, 1, 4, 2, 5, 5, 5>; };
template <> struct FftPlan<512> { using T = Stockham<512, 1, 4, 4, 4, 4, 2>; };
template <> struct FftPlan<1024> { using T = Stockham<1024, 1, 4, 4, 4, 4, 4>; };
template <> struct FftPlan<2048> { using T = Stockham<2048, 1, 4, 4, 4, 4, 4, 2>; };

// Block-cooperative twiddle table tw[m] = exp(-2*pi*i*m/N), computed in double then rounded.
template <int N>
__device__ __forceinline__ void init_twiddles(float2* tw) {
  for (int m = threadIdx.x; m < N; m += blockDim.x) {
    double s, c;
    sincospi(2.0 * (double)m / (double)N, &s, &c);
    tw[m] = make_float2((float)c, (float)(-s));
  }
}

}  // namespace dvh
