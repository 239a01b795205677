// Dispersion (f-v) image on MI355X (gfx950): map_fv of the reference, batched over gathers.
//
// Replaces fk (modules/utils.py:236-248) + map_fv (:457-475) + Dispersion (:383-426):
//   FK = |fftshift(fft2(data, s=[nk, nf]))| sampled bilinearly at (k = f / v, f) with the queries
//   clamped to the grid (interp2d(kind='linear') == FITPACK degree-1 spline), stored as float32,
//   then savgol_filter(25, 4, axis=0, mode='interp') along frequency, output [Nvel, Nfreq].
// Only the FK bins the queries touch are computed, as two GEMMs on the float64 MFMA pipe
// (v_mfma_f64_16x16x4_f64): |FK| then tracks the reference's float64 fft2 to ~1e-13, so the
// float32 f-v map (and its argmax pick) comes out as the reference's for exact inputs.
//   1. time DFT   D[r, q]  = sum_t data[r, t] * exp(-2 pi i nu_q t / nf)      (r = gather x channel)
//      real GEMM  [B*nch x nt] . [nt x 2*n_fb]  (cos | -sin float64 twiddles prepared on the host)
//   2. channel contraction  Z[m, q] = sum_x exp(-2 pi i kappa_m x / nk) D[x, q]  per gather,
//      complex GEMM as the real block GEMM [[Er, -Ei], [Ei, Er]] . [Dr; Di], then |Z| -> FK grid
//      (optionally accumulated per class slot with a weight: the f-v image is linear in |FK|)
//   3. f-v sampling: bilinear (FITPACK basis, double) -> float32 -> Savitzky-Golay operator (double)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <stdlib.h>

#include "dvh_common.h"
#include "dvh.h"

namespace dvh {

typedef double doublex4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

// v_mfma_f64_16x16x4_f64 lane maps: A[i = l & 15][k = l >> 4], B[k = l >> 4][j = l & 15],
// D[row = (l >> 4) + 4 r][col = l & 15] for r in [0, 4).
__device__ __forceinline__ doublex4 mfma_f64(double a, double b, doublex4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------------------------
// 1. time-DFT GEMM: C[r, n] = scale[r] * sum_k A[r, k] W[k, n]   (float64 MFMA, fp32 data)
// One wave per 32 x 32 output tile and K slice (split-K): the problem is small (tens of gather rows
// x a few hundred bins), so K is split to put hundreds of waves on the chip; the slices are summed
// with float64 atomics into C (zeroed by the launcher).
constexpr int kGT = 32;

__global__ __launch_bounds__(64) void tdft_gemm_kernel(const float* __restrict__ data, int64_t b_stride,
                                                        int64_t ch_stride, int32_t nch, int32_t M, int32_t K,
                                                        const double* __restrict__ W, int32_t N,
                                                        const float* __restrict__ row_scale, int32_t kslice,
                                                        double* __restrict__ C) {
  const int lane = threadIdx.x;
  const int m0 = blockIdx.y * kGT, n0 = blockIdx.x * kGT;
  const int k0 = blockIdx.z * kslice, k1 = min(K, k0 + kslice);
  const float* rowp[2];
  bool rok[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int r = m0 + f * 16 + (lane & 15);
    rok[f] = r < M;
    const int rr = rok[f] ? r : 0;
    rowp[f] = data + (int64_t)(rr / nch) * b_stride + (int64_t)(rr % nch) * ch_stride;
  }
  doublex4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = doublex4{0.0, 0.0, 0.0, 0.0};
  // kTU k-steps of 4 per round: all of the round's operand loads are issued before its MFMAs, so
  // their latency overlaps (one k-step at a time left the wave waiting on every load)
  constexpr int kTU = 4;
  for (int k = k0; k < k1; k += 4 * kTU) {
    double a[kTU][2], b[kTU][2];
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      const int kk = k + 4 * u + (lane >> 4);
      const bool kok = kk < k1;
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        a[u][f] = (kok && rok[f]) ? (double)rowp[f][kk] : 0.0;
        const int c = n0 + f * 16 + (lane & 15);
        b[u][f] = (kok && c < N) ? W[(int64_t)kk * N + c] : 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < kTU; ++u)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma_f64(a[u][i], b[u][j], acc[i][j]);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + i * 16 + (lane >> 4) + 4 * r;
        const int col = n0 + j * 16 + (lane & 15);
        if (row < M && col < N)
          atomicAdd(C + (int64_t)row * N + col, acc[i][j][r] * (row_scale ? (double)row_scale[row] : 1.0));
      }
}

// 1b. The same GEMM with the twiddle operand staged in LDS and reused across the rows of a block:
// a block (4 waves) owns 64 rows x kTdNT 16-column tiles; each wave 16 rows x all kTdNT tiles, so one A
// operand (the gather samples, float4 loads: lane (i, q) holds rows i, k = k0 + 8 q + s for the chunk's
// 8 k-steps s -- the same k permutation on both operands) feeds kTdNT MFMAs.  The block stages the
// twiddle chunk W[k0 .. k0 + 32)[c0 .. c0 + 16 kTdNT) by LDS-DMA (16 B per lane) into a double buffer,
// the next chunk's while this one is multiplied; chunk row 8 q + s sits in LDS row 4 s + q, so the four
// lane groups of one B-operand read hit rows next to each other (other bank halves), not 8 rows apart
// (the same banks; measured the same, 96-101 us either way).  No split-K: the tile is stored, not
// accumulated.  512 gathers of 25 x 500: 176 -> 96 us against the split-K kernel (DVH_TDFT_ROWS=0).
constexpr int kTdNT = 7;   // 16-column tiles per block (112 columns)
constexpr int kTdKC = 32;  // k per chunk
constexpr int kTdRows = 64;
// Small problems (a few class stacks: configs[1]'s six class images make a handful of blocks of the form above, each
// a chain of 32 chunk round trips, 56 us) split K over G wave groups of one block instead: group g multiplies the chunks
// kc = g (mod G), the groups' sums are added in group order through LDS (deterministic, no atomics); 2 tiles per
// block keep the 16-wave block within 128 VGPRs (4 tiles spilled 14).  DVH_TDFT_ROWS=2: never split (A/B).
constexpr int kTdNTs = 2, kTdGs = 4;

__host__ __device__ constexpr size_t tdft_rows_lds(int NT, int G) {
  // the groups' staging buffers, or (after the loop) their partial sums, whichever is larger
  return sizeof(double) * (size_t)G * ((size_t)2 * kTdKC * NT * 16 > (size_t)4 * NT * 4 * 64
                                           ? (size_t)2 * kTdKC * NT * 16
                                           : (size_t)4 * NT * 4 * 64);
}

template <int NT, int G>
__global__ __launch_bounds__(256 * G) void tdft_rows_kernel(const float* __restrict__ data, int64_t b_stride,
                                                            int64_t ch_stride, int32_t nch, int32_t M, int32_t K,
                                                            const double* __restrict__ W, int32_t N,
                                                            const float* __restrict__ row_scale, double* __restrict__ C) {
  extern __shared__ __attribute__((aligned(16))) double wsm_all[];  // per group [2][kTdKC][NT * 16]
  constexpr int NC = NT * 16, CH = kTdKC * NC;
  const int tid = threadIdx.x, lane = tid & 63, wave = (tid >> 6) & 3, grp = G > 1 ? (tid >> 8) : 0;
  double* wsm = wsm_all + (size_t)grp * 2 * CH;
  const int m0 = blockIdx.x * kTdRows + wave * 16, c0 = blockIdx.y * NC;
  const int li = lane & 15, q = lane >> 4;
  const int row = m0 + li;
  const bool rok = row < M;
  const float* rowp = data + (rok ? (int64_t)(row / nch) * b_stride + (int64_t)(row % nch) * ch_stride : 0);
  const bool vec4 = ((b_stride | ch_stride) & 3) == 0 && (reinterpret_cast<uintptr_t>(data) & 15) == 0;
  // LDS-DMA of twiddle chunk kc into buffer buf: doubles e = r * NC + c (linear), 2 per lane per piece
  const int n_chunk = (K + kTdKC - 1) / kTdKC;
  const int n_step = (n_chunk + G - 1) / G;  // every group runs n_step steps (the barriers), idle past n_chunk
  auto stage = [&](int kc, int buf) {
    if (kc >= n_chunk) return;
    for (int p = wave; p < CH / 128; p += 4) {
      const int e = p * 128 + 2 * lane;
      const int rho = e / NC, c = e - rho * NC;
      const int r = 8 * (rho & 3) + (rho >> 2);  // LDS row rho = 4 s + q holds chunk row k = 8 q + s
      const int kr = min(kc * kTdKC + r, K - 1), cc = min(c0 + c, N - 2);
      __builtin_amdgcn_global_load_lds((gbl_void*)(W + (int64_t)kr * N + cc), (lds_void*)(wsm + buf * CH + p * 128), 16,
                                       0, 0);
    }
  };
  // A operand of chunk kc: a[s] = data[row][k0 + 8 q + s] (0 past K or M)
  auto load_a = [&](int kc, double (&a)[8]) {
    const int kb = kc * kTdKC + 8 * q;
    if (vec4 && kb + 8 <= K && rok) {
      const float4 u = *reinterpret_cast<const float4*>(rowp + kb);
      const float4 v = *reinterpret_cast<const float4*>(rowp + kb + 4);
      a[0] = u.x; a[1] = u.y; a[2] = u.z; a[3] = u.w; a[4] = v.x; a[5] = v.y; a[6] = v.z; a[7] = v.w;
    } else {
#pragma unroll
      for (int s = 0; s < 8; ++s) a[s] = (rok && kb + s < K) ? (double)rowp[kb + s] : 0.0;
    }
  };
  doublex4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = doublex4{0.0, 0.0, 0.0, 0.0};
  double a[8];
  stage(grp, 0);
  load_a(grp, a);
  for (int st = 0; st < n_step; ++st) {
    const int kc = grp + G * st, kn = kc + G;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this chunk's twiddles have landed (and a)
    __syncthreads();  // ... for every wave; the other buffer's last readers are done
    double an[8];
    if (kn < n_chunk) {
      stage(kn, (st + 1) & 1);
      load_a(kn, an);
    }
    if (kc < n_chunk) {
      // rows beyond K in a partial chunk multiply a = 0 with finite (clamped) twiddles
      const double* Wc = wsm + (st & 1) * CH;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma_f64(a[s], Wc[(4 * s + q) * NC + t * 16 + li], acc[t]);
      }
    }
    if (kn < n_chunk) {
#pragma unroll
      for (int s = 0; s < 8; ++s) a[s] = an[s];
    }
  }
  if constexpr (G > 1) {  // group sums in group order: red[g][wave][t][r][lane]
    __syncthreads();       // every group's last chunk is read
    double* red = wsm_all;
    if (grp > 0) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[(((size_t)grp * 4 + wave) * NT + t) * 256 + r * 64 + lane] = acc[t][r];
    }
    __syncthreads();
    if (grp > 0) return;
#pragma unroll
    for (int g = 1; g < G; ++g)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[t][r] += red[(((size_t)g * 4 + wave) * NT + t) * 256 + r * 64 + lane];
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = c0 + t * 16 + li;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = m0 + q + 4 * r;
      if (rr < M && col < N) C[(int64_t)rr * N + col] = acc[t][r] * (row_scale ? (double)row_scale[rr] : 1.0);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// 2. channel contraction + magnitude (float64 MFMA).  A (host table, global/L2) is [2*MT][K2],
// K2 = 2*nch rounded up to a multiple of 4: rows [0, MT) give Re Z, rows [MT, 2MT) give Im Z.
// One block = (gather b, 32 f-bins).
constexpr int kFN = 32;

__global__ __launch_bounds__(256) void fk_contract_kernel(const double* __restrict__ D, int32_t nch, int32_t n_fb,
                                                           const double* __restrict__ Atab, int32_t MT, int32_t K2,
                                                           int32_t n_kb, double* __restrict__ FK,
                                                           const int32_t* __restrict__ slot,
                                                           const float* __restrict__ weight, int32_t n_slot) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int M2 = 2 * MT;
  double* Bs = sm;                      // [K2][kFN + 1]
  double* Cs = Bs + K2 * (kFN + 1);     // [M2][kFN + 1]
  const int b = blockIdx.y, q0 = blockIdx.x * kFN;
  const double* Db = D + (int64_t)b * nch * 2 * n_fb;
  for (int e = threadIdx.x; e < K2 * kFN; e += 256) {
    const int kk = e / kFN, n = e % kFN;
    const int q = q0 + n;
    double v = 0.0;
    if (q < n_fb && kk < 2 * nch) {
      const int x = kk < nch ? kk : kk - nch;
      v = Db[(int64_t)x * 2 * n_fb + 2 * q + (kk < nch ? 0 : 1)];
    }
    Bs[kk * (kFN + 1) + n] = v;
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n_mt = M2 / 16, n_nt = kFN / 16;
  for (int t = wave; t < n_mt * n_nt; t += 4) {
    const int mt = t / n_nt, nt = t % n_nt;
    doublex4 acc = {0.0, 0.0, 0.0, 0.0};
    const double* arow = Atab + (int64_t)(mt * 16 + (lane & 15)) * K2;
    for (int kk = 0; kk < K2; kk += 4) {
      const double a = arow[kk + (lane >> 4)];
      const double bb = Bs[(kk + (lane >> 4)) * (kFN + 1) + nt * 16 + (lane & 15)];
      acc = mfma_f64(a, bb, acc);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = mt * 16 + (lane >> 4) + 4 * r;
      Cs[row * (kFN + 1) + nt * 16 + (lane & 15)] = acc[r];
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < n_kb * kFN; e += 256) {
    const int m = e / kFN, n = e % kFN, q = q0 + n;
    if (q >= n_fb) continue;
    const double mag = hypot(Cs[m * (kFN + 1) + n], Cs[(MT + m) * (kFN + 1) + n]);
    if (slot) {
      const int sl = slot[b];
      if (sl >= 0 && sl < n_slot)  // the host rejects such slots; never write outside FK
        atomicAdd(FK + ((int64_t)sl * n_kb + m) * n_fb + q, mag * (double)weight[b]);
    } else {
      FK[((int64_t)b * n_kb + m) * n_fb + q] = mag;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// 3. f-v sampling + Savitzky-Golay.  One block = (gather b, 16 velocity rows), all frequencies.
constexpr int kVC = 4;        // velocities per block: 750 blocks for one set of 3 images of 1000 x 242
constexpr int kVS = kVC + 1;  // LDS row stride: the f-consecutive FIR reads hit distinct banks

__global__ __launch_bounds__(256) void fv_kernel(const double* __restrict__ FK, int32_t n_kb, int32_t n_fb,
                                                  const double* __restrict__ kgrid, double kmin, double kmax,
                                                  const double* __restrict__ kq, int32_t nF, int32_t nV,
                                                  const int32_t* __restrict__ fj, const double* __restrict__ fw,
                                                  const double* __restrict__ sg, int32_t sgl,
                                                  float* __restrict__ fv) {
  extern __shared__ __attribute__((aligned(16))) float raw[];  // [nF][kVS]
  const int b = blockIdx.y, v0 = blockIdx.x * kVC;
  const double* F = FK + (int64_t)b * n_kb * n_fb;
  const double k0 = kgrid[0], inv_dk = 1.0 / (kgrid[1] - kgrid[0]);
  for (int e = threadIdx.x; e < nF * kVC; e += blockDim.x) {
    const int f = e / kVC, iv = e % kVC, v = v0 + iv;
    float val = 0.f;
    if (v < nV) {
      double q = kq[(int64_t)f * nV + v];
      q = q < kmin ? kmin : (q > kmax ? kmax : q);  // fpbisp clamps to [t_b, t_e]
      int m = (int)floor((q - k0) * inv_dk);
      m = m < 0 ? 0 : (m > n_kb - 2 ? n_kb - 2 : m);
      while (m < n_kb - 2 && q >= kgrid[m + 1]) ++m;
      while (m > 0 && q < kgrid[m]) --m;
      const double klo = kgrid[m], khi = kgrid[m + 1];
      const double fx = 1.0 / (khi - klo);
      const double hx0 = fx * (khi - q), hx1 = fx * (q - klo);  // fpbspl, degree 1
      const int j = fj[f];
      const double hy0 = fw[2 * f], hy1 = fw[2 * f + 1];
      const double z00 = F[m * n_fb + j], z01 = F[m * n_fb + j + 1];
      const double z10 = F[(m + 1) * n_fb + j], z11 = F[(m + 1) * n_fb + j + 1];
      val = (float)(z00 * hx0 * hy0 + z01 * hx0 * hy1 + z10 * hx1 * hy0 + z11 * hx1 * hy1);
    }
    raw[f * kVS + iv] = val;
  }
  __syncthreads();
  const int half = sgl / 2;
  const double* h = sg;                        // interior taps, h[t] multiplies x[f - half + t]
  const double* el = sg + sgl;                 // [half][sgl] left edge (fit to x[0:sgl])
  const double* er = el + half * sgl;          // [half][sgl] right edge (fit to x[nF-sgl:nF])
  for (int e = threadIdx.x; e < nF * kVC; e += blockDim.x) {
    const int iv = e / nF, f = e % nF, v = v0 + iv;
    if (v >= nV) continue;
    double acc = 0.0;
    if (f < half) {
      for (int t = 0; t < sgl; ++t) acc += el[f * sgl + t] * (double)raw[t * kVS + iv];
    } else if (f >= nF - half) {
      const int r = f - (nF - half);
      for (int t = 0; t < sgl; ++t) acc += er[r * sgl + t] * (double)raw[(nF - sgl + t) * kVS + iv];
    } else {
      for (int t = 0; t < sgl; ++t) acc += h[t] * (double)raw[(f - half + t) * kVS + iv];
    }
    fv[((int64_t)b * nV + v) * nF + f] = (float)acc;
  }
}

// 3b. Batched f-v sampling (many images of one plan): one 1024-thread block = (VC velocities, all
// frequencies) x G consecutive images.  The bilinear weights depend on (f, v) only, so each thread
// computes them ONCE (frequency f = tid % nF, velocities 4 g .. 4 g + 3 of the chunk, g = tid / nF)
// and keeps them in registers across the G images.  Per image: the image's FK grid is staged in LDS
// (n_kb x n_fb doubles), the float32 samples go to an LDS row per velocity padded by kSgPad zeros on
// both sides, and the Savitzky-Golay pass gives every thread 4 consecutive outputs of one velocity
// (28 inputs read as 7 x 16 B, 25 taps each in double, the same tap order as fv_kernel).  Bound:
// float64 FMA issue (25 per output) and the 4 B/output HBM write.
constexpr int kFvThreads = 1024;
constexpr int kFvVT = 4;   // velocities per thread in the sampling phase
constexpr int kFvPre = 4;  // FK doubles prefetched per thread: grids up to 4 x 1024 bins
constexpr int kSgPad = 12; // zero pad per side of an LDS row (the fast path needs sgl = 2 * kSgPad + 1)

// Workgroup barrier for LDS hand-offs only.  __syncthreads() also orders global memory (a
// workgroup-scope release: s_waitcnt vmcnt(0)), which would stall every image on the previous
// image's f-v stores; the fv stores are never read back by the block.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ int fv_row_stride(int nF) { return ((nF + 3) & ~3) + 2 * kSgPad; }

__global__ __launch_bounds__(kFvThreads) void fv_batch_kernel(
    const double* __restrict__ FK, int32_t B, int32_t G, int32_t n_kb, int32_t n_fb,
    const double* __restrict__ kgrid, double kmin, double kmax, const double* __restrict__ kq, int32_t nF,
    int32_t nV, int32_t n_grp, const int32_t* __restrict__ fj, const double* __restrict__ fw,
    const double* __restrict__ sg, int32_t sgl, float* __restrict__ fv) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nfk = n_kb * n_fb;
  const int nfk2 = (nfk + 1) & ~1;
  double* fks = smem;                                                // 2 x [n_kb][n_fb] (double buffer)
  const int VC = kFvVT * n_grp, S = fv_row_stride(nF);
  double* sgs = smem + 2 * nfk2;                                     // Savitzky-Golay taps + edge fits
  float* raw = reinterpret_cast<float*>(sgs + ((sgl * sgl + 1) & ~1));  // [VC][S], x[f] at kSgPad + f
  const int v0 = blockIdx.x * VC, tid = threadIdx.x;

  // sampling ownership and weights (fv_kernel's expressions, computed once)
  const int g = tid / nF, f = tid - g * nF;
  const bool own = g < n_grp;
  int base[kFvVT];
  double hx0[kFvVT], hx1[kFvVT], hy0 = 0.0, hy1 = 0.0;
  {
    const double k0 = kgrid[0], inv_dk = 1.0 / (kgrid[1] - kgrid[0]);
    const int j = own ? fj[f] : 0;
    if (own) {
      hy0 = fw[2 * f];
      hy1 = fw[2 * f + 1];
    }
#pragma unroll
    for (int i = 0; i < kFvVT; ++i) {
      const int v = v0 + kFvVT * g + i;
      base[i] = -1;
      hx0[i] = hx1[i] = 0.0;
      if (own && v < nV) {
        double q = kq[(int64_t)f * nV + v];
        q = q < kmin ? kmin : (q > kmax ? kmax : q);
        int m = (int)floor((q - k0) * inv_dk);
        m = m < 0 ? 0 : (m > n_kb - 2 ? n_kb - 2 : m);
        while (m < n_kb - 2 && q >= kgrid[m + 1]) ++m;
        while (m > 0 && q < kgrid[m]) --m;
        const double klo = kgrid[m], khi = kgrid[m + 1];
        const double fx = 1.0 / (khi - klo);
        hx0[i] = fx * (khi - q);
        hx1[i] = fx * (q - klo);
        base[i] = m * n_fb + j;
      }
    }
  }
  // zero pads (never written afterwards)
  for (int e = tid; e < VC * S; e += kFvThreads) {
    const int c = e % S;
    if (c < kSgPad || c >= kSgPad + nF) raw[e] = 0.f;
  }
  const int half = sgl / 2;
  for (int e = tid; e < sgl * sgl; e += kFvThreads) sgs[e] = sg[e];  // sgl + 2 * half * sgl = sgl^2 entries
  const double* h = sgs;
  const double* el = sgs + sgl;
  const double* er = el + half * sgl;
  const int nb4 = (nF + 3) >> 2;
  const bool fast_taps = (sgl == 2 * kSgPad + 1);
  // FK grids are software-pipelined: image it + 1's grid is loaded into registers (kFvPre per
  // thread) while image it is sampled, and stored to the other LDS buffer before its filter pass
  const int b0 = blockIdx.y * G;
  const int n_img = min(G, B - b0);
  double pre[kFvPre];
#pragma unroll
  for (int k = 0; k < kFvPre; ++k) {
    const int e = tid + k * kFvThreads;
    if (e < nfk) fks[e] = FK[(int64_t)b0 * nfk + e];
  }
  for (int it = 0; it < n_img; ++it) {
    const int b = b0 + it;
    const double* fk_cur = fks + (it & 1) * nfk2;
    lds_barrier();  // fk_cur stored, raw free
    const bool more = it + 1 < n_img;
    if (more) {
#pragma unroll
      for (int k = 0; k < kFvPre; ++k) {
        const int e = min(tid + k * kFvThreads, nfk - 1);  // unconditional load: no register zeroing
        pre[k] = FK[(int64_t)(b + 1) * nfk + e];
      }
    }
    if (own) {
#pragma unroll
      for (int i = 0; i < kFvVT; ++i) {
        if (base[i] < 0) continue;
        const int m = base[i];
        const double z00 = fk_cur[m], z01 = fk_cur[m + 1], z10 = fk_cur[m + n_fb], z11 = fk_cur[m + n_fb + 1];
        raw[(kFvVT * g + i) * S + kSgPad + f] =
            (float)(z00 * hx0[i] * hy0 + z01 * hx0[i] * hy1 + z10 * hx1[i] * hy0 + z11 * hx1[i] * hy1);
      }
    }
    if (more) {  // next image's grid -> the other LDS buffer (last read in the previous image's sampling)
      double* fk_next = fks + ((it + 1) & 1) * nfk2;
#pragma unroll
      for (int k = 0; k < kFvPre; ++k) {
        const int e = tid + k * kFvThreads;
        if (e < nfk) fk_next[e] = pre[k];
      }
    }
    lds_barrier();
    for (int task = tid; task < VC * nb4; task += kFvThreads) {
      const int r = task / nb4, f0 = (task - r * nb4) * 4, v = v0 + r;
      if (v >= nV) continue;
      const float* row = raw + r * S + kSgPad;  // row[x] = sample at frequency x (zero outside [0, nF))
      double acc[4] = {0.0, 0.0, 0.0, 0.0};
      if (fast_taps && f0 >= half && f0 + 3 < nF - half) {
        float x[28];
#pragma unroll
        for (int q = 0; q < 7; ++q) {
          const float4 t4 = *reinterpret_cast<const float4*>(row + f0 - kSgPad + 4 * q);
          x[4 * q] = t4.x; x[4 * q + 1] = t4.y; x[4 * q + 2] = t4.z; x[4 * q + 3] = t4.w;
        }
#pragma unroll
        for (int t = 0; t < 2 * kSgPad + 1; ++t) {
          const double ht = sg[t];  // uniform: scalar loads, SGPR operands
#pragma unroll
          for (int o = 0; o < 4; ++o) acc[o] += ht * (double)x[o + t];
        }
      } else if (fast_taps) {
        // edge block: the edge fits read x[0, 25) or x[nF - 25, nF) -- loaded once, all loops
        // unrolled so the LDS reads are batched (a rolled loop here stalls the whole block at the
        // next barrier: one dependent LDS round trip per tap)
        constexpr int L = 2 * kSgPad + 1;
        const float* src = f0 < half ? row : row + nF - L;
        float y[L];
#pragma unroll
        for (int t = 0; t < L; ++t) y[t] = src[t];
#pragma unroll
        for (int o = 0; o < 4; ++o) {
          const int ff = f0 + o;
          if (ff >= nF) break;
          double a = 0.0;
          if (ff < half || ff >= nF - half) {
            const double* c = ff < half ? el + ff * L : er + (ff - (nF - half)) * L;
#pragma unroll
            for (int t = 0; t < L; ++t) a += c[t] * (double)y[t];
          } else {
#pragma unroll
            for (int t = 0; t < L; ++t) a += sg[t] * (double)row[ff - half + t];
          }
          acc[o] = a;
        }
      } else {
#pragma unroll
        for (int o = 0; o < 4; ++o) {
          const int ff = f0 + o;
          if (ff >= nF) break;
          double a = 0.0;
          if (ff < half) {
            for (int t = 0; t < sgl; ++t) a += el[ff * sgl + t] * (double)row[t];
          } else if (ff >= nF - half) {
            const int rr = ff - (nF - half);
            for (int t = 0; t < sgl; ++t) a += er[rr * sgl + t] * (double)row[nF - sgl + t];
          } else {
            for (int t = 0; t < sgl; ++t) a += h[t] * (double)row[ff - half + t];
          }
          acc[o] = a;
        }
      }
      float* out = fv + ((int64_t)b * nV + v) * nF + f0;
      if ((nF & 3) == 0) {
        *reinterpret_cast<float4*>(out) = make_float4((float)acc[0], (float)acc[1], (float)acc[2], (float)acc[3]);
      } else {
#pragma unroll
        for (int o = 0; o < 4; ++o)
          if (f0 + o < nF) out[o] = (float)acc[o];
      }
    }
  }
}

// 3c. Frequency-tiled f-v sampling: one 256-thread block = (a tile of TO output frequencies, 4
// velocities) x G images, so that several independent blocks share a CU (the 1 024-thread
// fv_batch_kernel leaves the SIMDs idle at every barrier).  The block samples the tile's
// frequencies plus a kSgPad halo on each side (clamped to the record; the last tile keeps at least
// the 25 samples the right-edge fit reads), so the Savitzky-Golay pass of its outputs is local.
// Only the FK columns the tile's frequencies touch are staged per image.
constexpr int kTileThreads = 256;
constexpr int kTileVT = 4;  // velocities per fv_tile block (8: more outputs per barrier pair, more registers)

// kCells: instead of every FK row of the columns the tile touches, the block stages only the cells its
// bilinear stencils read (host tables of DispPlan.cell_tables, per (velocity chunk, tile) ct: the cells'
// FK offsets, column-major, and per (frequency, velocity) the compact indices b0 of (m, j) and b1 of
// (m, j + 1) and the FITPACK interval m) -- a few rows per column instead of all n_kb.
template <int VT, bool kCells>
__global__ __launch_bounds__(kTileThreads) void fv_tile_kernel(
    const double* __restrict__ FK, int32_t B, int32_t G, int32_t n_kb, int32_t n_fb,
    const double* __restrict__ kgrid, double kmin, double kmax, const double* __restrict__ kq, int32_t nF,
    int32_t nV, int32_t TO, const int32_t* __restrict__ fj, const double* __restrict__ fw,
    const double* __restrict__ sg, int32_t sgl, float* __restrict__ fv, const int32_t* __restrict__ cell_off,
    const int32_t* __restrict__ n_cell, int32_t max_cell, const int4* __restrict__ qidx) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int S = 2 * kSgPad + kTileThreads + 4;  // row stride (floats), multiple of 4
  const int tid = threadIdx.x;
  const int f_lo = blockIdx.x * TO, f_hi = min(nF, f_lo + TO);
  const int half = sgl / 2;
  const int s0 = max(0, f_lo - kSgPad);
  const int s1 = min(nF, max(f_hi + kSgPad, sgl));
  const int v0 = blockIdx.y * VT;
  const int f = s0 + tid;
  const bool own = f < s1;
  const int ct = blockIdx.y * gridDim.x + blockIdx.x;  // (velocity chunk, tile) of the cell tables
  int jlo = 0, ncol = 0, nsub = 0;
  if constexpr (kCells) {
    nsub = n_cell[ct];
  } else {
    __shared__ int jr[2];
    if (tid == 0) {
      jr[0] = 1 << 30;
      jr[1] = -1;
    }
    __syncthreads();
    if (own) {
      atomicMin(&jr[0], fj[f]);
      atomicMax(&jr[1], fj[f]);
    }
    __syncthreads();
    jlo = jr[0];
    ncol = jr[1] + 2 - jr[0];  // columns jlo .. jhi + 1
    nsub = n_kb * ncol;
  }
  double* fks = smem;  // [n_kb][ncol], or the compact cells
  double* sgs = smem + (((kCells ? max_cell : n_kb * n_fb) + 1) & ~1);  // taps + edge fits
  float* raw = reinterpret_cast<float*>(sgs + ((sgl * sgl + 1) & ~1));  // [VT][S]
  for (int e = tid; e < sgl * sgl; e += kTileThreads) sgs[e] = sg[e];
  for (int e = tid; e < VT * S; e += kTileThreads) raw[e] = 0.f;
  const double* h = sgs;
  const double* el = sgs + sgl;
  const double* er = el + half * sgl;

  int base[VT], base1[VT];
  double hx0[VT], hx1[VT], hy0 = 0.0, hy1 = 0.0;
  {
    const double k0 = kgrid[0], inv_dk = 1.0 / (kgrid[1] - kgrid[0]);
    const int j = own && !kCells ? fj[f] - jlo : 0;
    if (own) {
      hy0 = fw[2 * f];
      hy1 = fw[2 * f + 1];
    }
#pragma unroll
    for (int i = 0; i < VT; ++i) {
      const int v = v0 + i;
      base[i] = -1;
      hx0[i] = hx1[i] = 0.0;
      if (own && v < nV) {
        double q = kq[(int64_t)f * nV + v];
        q = q < kmin ? kmin : (q > kmax ? kmax : q);
        int m;
        if constexpr (kCells) {
          const int4 ix = qidx[((int64_t)ct * kTileThreads + tid) * VT + i];
          m = ix.z;
          base[i] = ix.x;
          base1[i] = ix.y;
        } else {
          m = (int)floor((q - k0) * inv_dk);
          m = m < 0 ? 0 : (m > n_kb - 2 ? n_kb - 2 : m);
          while (m < n_kb - 2 && q >= kgrid[m + 1]) ++m;
          while (m > 0 && q < kgrid[m]) --m;
          base[i] = m * ncol + j;
          base1[i] = base[i] + 1;
        }
        const double klo = kgrid[m], khi = kgrid[m + 1];
        const double fx = 1.0 / (khi - klo);
        hx0[i] = fx * (khi - q);
        hx1[i] = fx * (q - klo);
      }
    }
  }
  const int nb4 = (f_hi - f_lo + 3) >> 2;
  const bool fast_taps = (sgl == 2 * kSgPad + 1);
  const int b0 = blockIdx.z * G;
  const int n_img = min(G, B - b0);
  // the sub-grid element -> FK offset map is the same for every image: computed once
  constexpr int kStage = 3;  // elements per thread held as offsets (sub-grids up to 768 bins)
  int goff[kStage];
#pragma unroll
  for (int q = 0; q < kStage; ++q) {
    const int e = tid + q * kTileThreads;
    if constexpr (kCells) {
      goff[q] = e < nsub ? cell_off[(int64_t)ct * max_cell + e] : -1;
    } else {
      const int m = e / ncol;
      goff[q] = e < nsub ? m * n_fb + (e - m * ncol) : -1;
    }
  }
  // filter tasks (velocity row, 4 outputs): tid and, for VT = 8, tid + kTileThreads
  constexpr int kTasks = (VT * 64 + kTileThreads - 1) / kTileThreads;  // task slots per thread (nb4 <= 64)
  // Two barriers per image: the next image's FK sub-grid is staged into fks while this image is
  // filtered (fks is free once every thread has sampled), and its first kStage elements come from
  // registers loaded one image earlier, so the FK fetch latency is not exposed between barriers.
  const int64_t img_stride = (int64_t)n_kb * n_fb;
  double pre[kStage];
  auto stage_img = [&](int it_s) {  // pre (image it_s) -> fks; the rest of the sub-grid from global
    const double* F = FK + (int64_t)(b0 + it_s) * img_stride + jlo;
#pragma unroll
    for (int q = 0; q < kStage; ++q)
      if (goff[q] >= 0) fks[tid + q * kTileThreads] = pre[q];
    for (int e = tid + kStage * kTileThreads; e < nsub; e += kTileThreads) {
      if constexpr (kCells) {
        fks[e] = F[cell_off[(int64_t)ct * max_cell + e]];
      } else {
        const int m = e / ncol, c = e - m * ncol;
        fks[e] = F[m * n_fb + c];
      }
    }
  };
  auto load_pre = [&](int it_l) {
    const double* F = FK + (int64_t)(b0 + it_l) * img_stride + jlo;
#pragma unroll
    for (int q = 0; q < kStage; ++q)
      if (goff[q] >= 0) pre[q] = F[goff[q]];
  };
  if (n_img > 0) {
    load_pre(0);
    stage_img(0);
    if (n_img > 1) load_pre(1);
  }
  for (int it = 0; it < n_img; ++it) {
    const int b = b0 + it;
    lds_barrier();  // fks holds image it; the previous image's filter is done with raw
    if (own) {
#pragma unroll
      for (int i = 0; i < VT; ++i) {
        if (base[i] < 0) continue;
        // (m, j), (m, j + 1), (m + 1, j), (m + 1, j + 1): row-major sub-grid, or compact column-major cells
        const int m = base[i], m1 = base1[i];
        const double z00 = fks[m], z01 = kCells ? fks[m1] : fks[m + 1];
        const double z10 = kCells ? fks[m + 1] : fks[m + ncol], z11 = kCells ? fks[m1 + 1] : fks[m + ncol + 1];
        raw[i * S + kSgPad + tid] =
            (float)(z00 * hx0[i] * hy0 + z01 * hx0[i] * hy1 + z10 * hx1[i] * hy0 + z11 * hx1[i] * hy1);
      }
    }
    lds_barrier();  // raw holds image it; fks is free
    if (it + 1 < n_img) {
      stage_img(it + 1);
      if (it + 2 < n_img) load_pre(it + 2);
    }
    // VT * nb4 filter tasks over the block's threads (TO + 2 kSgPad <= kTileThreads)
#pragma unroll
    for (int ts = 0; ts < kTasks; ++ts) {
      const int task = tid + ts * kTileThreads;
      const int t_r = task / nb4, t_f0 = f_lo + (task - t_r * nb4) * 4;
      if (!(task < VT * nb4 && v0 + t_r < nV)) continue;
      const int r = t_r, f0 = t_f0, v = v0 + r;
      const float* row = raw + r * S + kSgPad - s0;  // row[x] = sample at frequency x
      double acc[4] = {0.0, 0.0, 0.0, 0.0};
      if (fast_taps && f0 >= half && f0 + 3 < nF - half && f0 + 3 < f_hi) {
        float x[28];
#pragma unroll
        for (int q = 0; q < 7; ++q) {
          const float4 t4 = *reinterpret_cast<const float4*>(row + f0 - kSgPad + 4 * q);
          x[4 * q] = t4.x; x[4 * q + 1] = t4.y; x[4 * q + 2] = t4.z; x[4 * q + 3] = t4.w;
        }
#pragma unroll
        for (int t = 0; t < 2 * kSgPad + 1; ++t) {
          const double ht = sg[t];
#pragma unroll
          for (int o = 0; o < 4; ++o) acc[o] += ht * (double)x[o + t];
        }
      } else if (fast_taps) {  // edge (or partial) block, unrolled as in fv_batch_kernel
        constexpr int L = 2 * kSgPad + 1;
        const float* src = f0 < half ? row : row + nF - L;
        float y[L];
#pragma unroll
        for (int t = 0; t < L; ++t) y[t] = src[t];
#pragma unroll
        for (int o = 0; o < 4; ++o) {
          const int ff = f0 + o;
          if (ff >= f_hi) break;
          double a = 0.0;
          if (ff < half || ff >= nF - half) {
            const double* c = ff < half ? el + ff * L : er + (ff - (nF - half)) * L;
#pragma unroll
            for (int t = 0; t < L; ++t) a += c[t] * (double)y[t];
          } else {
#pragma unroll
            for (int t = 0; t < L; ++t) a += sg[t] * (double)row[ff - half + t];
          }
          acc[o] = a;
        }
      } else {
#pragma unroll
        for (int o = 0; o < 4; ++o) {
          const int ff = f0 + o;
          if (ff >= f_hi) break;
          double a = 0.0;
          if (ff < half) {
            for (int t = 0; t < sgl; ++t) a += el[ff * sgl + t] * (double)row[t];
          } else if (ff >= nF - half) {
            const int rr = ff - (nF - half);
            for (int t = 0; t < sgl; ++t) a += er[rr * sgl + t] * (double)row[nF - sgl + t];
          } else {
            for (int t = 0; t < sgl; ++t) a += h[t] * (double)row[ff - half + t];
          }
          acc[o] = a;
        }
      }
      float* out = fv + ((int64_t)b * nV + v) * nF + f0;
      if ((nF & 3) == 0 && f0 + 3 < f_hi) {
        *reinterpret_cast<float4*>(out) = make_float4((float)acc[0], (float)acc[1], (float)acc[2], (float)acc[3]);
      } else {
#pragma unroll
        for (int o = 0; o < 4; ++o)
          if (f0 + o < f_hi) out[o] = (float)acc[o];
      }
    }
  }
}

// 3d. f-v sampling with the Savitzky-Golay filter on the matrix pipe.  The filter is a banded Toeplitz
// operator along frequency, so a (16 velocities x 16 frequencies) output tile is one float64 MFMA GEMM
//   out[v][f0 + j] = sum_{k < 40} x[v][f0 - 12 + k] * H[k][j],   H[k][j] = sg[k - j] (0 <= k - j < 25)
// with the samples x as the A operand (A[i = v][k] on lane (v, k & 3)) and the band as B: 10 K-steps of
// v_mfma_f64_16x16x4_f64 per tile (40 / 25 of the filter's FMAs, on the MFMA pipe, beside the VALU that
// samples).  A wave owns 16 velocities of GI images (GI independent accumulation chains) and walks the
// frequency axis tile by tile; tile t + 1 shares 24 of its 40 inputs with tile t, so each lane keeps its
// samples in a register ring per image (step g = frequency 4 g - 12 + (lane >> 4), slot g & 15) and
// samples 4 new ones per tile: their table loads one tile ahead, their arithmetic during the tile before
// the MFMAs that consume them.  The first tile (left polynomial fit rows f < 12) and a last tile at
// f0 = nF - 16 (right fit) take their B operands from the operator in LDS; the regular tiles write rows
// f < nF - 16 only.  The block (4 waves, 64 velocities) stages the GI images' compact FK grids in LDS
// with LDS-DMA (global_load_lds_dword, no VGPRs).
// Sampling per (f, v) is fv_kernel's arithmetic with the image-independent parts from plan tables
// (DispPlan.mfma_tables), loaded once per sample for the GI images: the FITPACK weights hx[f][v] =
// {fx (khi - q), fx (q - klo)} of the clamped query and the cell offset cb[f][v] = m * n_fb + fj[f],
// bit-identical to what the other kernels compute.  (Forming the weights in the kernel from the query and
// LDS tables of the k grid and fw measured slower: 1 207 vs 704 us for one image per wave, the LDS
// bandwidth of the extra reads.)  Two images per wave (GI = 2) measured 673 vs 724 us for one.
constexpr int kMfGI = 2;   // images per wave in lock step
constexpr int kMfWpe = 2;  // waves per SIMD the kernel is register-budgeted for
constexpr int kMfV = 16;      // velocities per wave
constexpr int kMfWaves = 4;   // waves per block

__device__ __forceinline__ double sg_coef(const double* sgs, int nF, int f, int xi) {
  constexpr int L = 2 * kSgPad + 1, half = kSgPad;
  int t;
  const double* c;
  if (f < half) {  // left fit: x[0, L)
    t = xi;
    c = sgs + L + f * L;
  } else if (f >= nF - half) {  // right fit: x[nF - L, nF)
    t = xi - (nF - L);
    c = sgs + L + half * L + (f - (nF - half)) * L;
  } else {
    t = xi - f + half;
    c = sgs;
  }
  return (t >= 0 && t < L) ? c[t] : 0.0;
}

// LDS bytes of fv_mfma_kernel<GI>
__host__ __device__ inline size_t fv_mfma_lds(int GI, int nfk) {
  const int nbuf = (nfk + 31) & ~31;
  constexpr int L = 2 * kSgPad + 1;
  return sizeof(double) * ((size_t)GI * nbuf + (size_t)L * L + 64);
}

template <int GI>
__global__ __launch_bounds__(kMfWaves * 64) __attribute__((amdgpu_waves_per_eu(kMfWpe, kMfWpe))) void fv_mfma_kernel(
    const double* __restrict__ FK, int32_t B, int32_t G, int32_t n_kb, int32_t n_fb, const double2* __restrict__ hx,
    const int32_t* __restrict__ cb, int32_t nF, int32_t nV, const double2* __restrict__ fw, const double* __restrict__ sg,
    float* __restrict__ fv, int32_t n_vb, int32_t xcd_map) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int L = 2 * kSgPad + 1;
  const int nfk = n_kb * n_fb;
  const int nbuf = ((nfk + 31) & ~31);  // doubles of an FK buffer: whole 256-byte LDS-DMA pieces
  double* fks = smem;                   // [GI][nbuf]
  double* sgs = smem + GI * nbuf;       // taps + edge fits (L * L)
  double* bpad = sgs + L * L;           // [64]: taps at 16 .. 40, zeros around (the interior band)
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // the lane index formed afresh where it is used (mbcnt of an opaque zero: no value kept live, or spilled,
  // across the image loop)
  auto lane_now = []() {
    unsigned z = 0;
    asm volatile("" : "+v"(z));
    return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, z));
  };
  // block -> (velocity block, image group); XCD-aware when the velocity blocks split evenly over the 8
  // XCDs (blocks are dealt round robin): every block of a velocity block then runs on one XCD and its
  // (f, v) table slice stays in that XCD's L2
  int vb, ig;
  {
    const int L0 = blockIdx.x;
    if (xcd_map) {
      const int per = n_vb >> 3, x = L0 & 7, k = L0 >> 3;
      vb = x + 8 * (k % per);
      ig = k / per;
    } else {
      vb = L0 % n_vb;
      ig = L0 / n_vb;
    }
  }
  const int b0 = ig * G, n_img = min(G, B - b0);
  const int vw = vb * (kMfWaves * kMfV) + wave * kMfV;  // the wave's first velocity (uniform)

  // LDS-DMA of image `img`'s FK grid into buffer `buf` (256-byte pieces dealt over the waves; lanes past
  // the grid re-read its last dword, landing in the buffer's pad)
  const int n_piece = (2 * nfk + 63) >> 6;
  auto stage = [&](int img, int buf) {
    const float* src = reinterpret_cast<const float*>(FK + (int64_t)img * nfk);
    const int lane = lane_now();
    for (int p = wave; p < n_piece; p += kMfWaves) {
      const int e = min(p * 64 + lane, 2 * nfk - 1);
      __builtin_amdgcn_global_load_lds((gbl_void*)(src + e), (lds_void*)(fks + buf * nbuf + p * 32), 4, 0, 0);
    }
  };
  for (int e = tid; e < L * L; e += kMfWaves * 64) sgs[e] = sg[e];
  for (int e = tid; e < 64; e += kMfWaves * 64) bpad[e] = (e >= 16 && e < 16 + L) ? sg[e - 16] : 0.0;
  const int t_reg = (nF - kMfV + kMfV - 1) / kMfV;  // regular tiles: rows [16 t, min(16 t + 16, nF - 16))

  for (int it = 0; it < n_img; it += GI) {
    const int ng = min(GI, n_img - it);  // images of this pass (a lone last image runs as a pair with itself)
    // the previous pass's reads are done (first barrier), the DMA has landed (vmcnt, second barrier)
    __syncthreads();
#pragma unroll
    for (int g = 0; g < GI; ++g) stage(b0 + it + min(g, ng - 1), g);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // the lane indices and sizes are laundered per pass: the first and last tiles' samples, band values
    // and store addresses do not depend on the images, and hoisting them out of the image loop would hold
    // ~200 registers; recomputing them is a few VALU per tile
    int li_, kk_, nF_, nV_, va_, vc_, fl_, boff;
    bool vok_;
    auto launder = [&]() {  // also before the last tile: no common subexpression with tile 0 lives across the loop
      const int ln = lane_now();
      li_ = ln & 15;
      kk_ = ln >> 4;
      nF_ = nF;
      nV_ = nV;
      asm volatile("" : "+v"(li_), "+v"(kk_), "+s"(nF_), "+s"(nV_));
      boff = 16 + kk_ - li_;  // interior band B[k][j] of K-step s = bpad[boff + 4 s] = sg[4 s + k - j]
      va_ = vw + li_;
      vok_ = va_ < nV_;
      vc_ = min(va_, nV_ - 1);
      fl_ = nF_ - kMfV;  // the last tile's first row
    };
    launder();
    // one sample of this lane for the GI images, branch-free (indices clamped, values zeroed outside the
    // grid): x[va_][f] rounded to float32 as map_fv's interp2d output.  Two stages for the regular
    // tiles: the table loads (tload) one tile before the weights, corners and arithmetic (tfinish).
    struct Pend {
      double2 w;
      int base, fc;
      bool in;
    };
    auto tload = [&](int f) -> Pend {
      Pend p;
      p.in = vok_ && f >= 0 && f < nF_;
      p.fc = min(max(f, 0), nF_ - 1);
      const int qi = p.fc * nV_ + vc_;
      p.w = hx[qi];
      p.base = cb[qi];
      return p;
    };
    auto tfinish = [&](const Pend& p, double* xo) {
      const double2 y = fw[p.fc];  // per frequency: 16 lanes share it (an LDS copy measured slower: the
                                   // corner reads already load the LDS, 700 vs 673 us)
      // the corner pairs are merged into ds_read2_b64 (8 LDS cycles against 2 + 2 for single reads, but
      // four opaque single reads measured slower: 743-751 vs 731 us)
      const int i00 = p.base, i01 = p.base + 1, i10 = p.base + n_fb, i11 = p.base + n_fb + 1;
#pragma unroll
      for (int g = 0; g < GI; ++g) {
        const double* F = fks + g * nbuf;
        const double z00 = F[i00], z01 = F[i01], z10 = F[i10], z11 = F[i11];
        const double val = (double)(float)(z00 * p.w.x * y.x + z01 * p.w.x * y.y + z10 * p.w.y * y.x +
                                           z11 * p.w.y * y.y);
        xo[g] = p.in ? val : 0.0;
      }
    };
    auto sample = [&](int f, double* xo) { tfinish(tload(f), xo); };
    auto store = [&](const doublex4* acc, int f0, int f_end) {
      const int f = f0 + li_;
      if (f >= f_end) return;
#pragma unroll
      for (int g = 0; g < GI; ++g) {
        if (g >= ng) break;
        float* out_b = fv + (int64_t)(b0 + it + g) * nV_ * nF_;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int v = vw + kk_ + 4 * r;
          if (v < nV_) out_b[(int64_t)v * nF_ + f] = (float)acc[g][r];
        }
      }
    };
    // rings of samples: step g (frequency 4 g - 12 + kk) in slot g & 15; steps 4 t + 10 .. 4 t + 13 (tile
    // t + 1's new ones) are finished during tile t from table loads issued during tile t - 1
    double x[16][GI];
#pragma unroll
    for (int g = 0; g < GI; ++g) x[0][g] = x[1][g] = 0.0;  // frequencies < -4
#pragma unroll
    for (int s = 2; s < 14; ++s) {  // in groups of 4 loads in flight: the next group's addresses wait on
      sample(4 * s - 12 + kk_, x[s]);  // this group's samples (an opaque dependency the compiler keeps)
      if (s % 4 == 1) asm volatile("" : "+v"(kk_) : "v"(x[s - 3][0]), "v"(x[s - 2][0]), "v"(x[s - 1][0]), "v"(x[s][0]));
    }
#pragma unroll
    for (int s = 10; s < 14; ++s)  // every image's tile-1 samples finished here, not deferred past tile 0
#pragma unroll
      for (int g = 0; g < GI; ++g) asm volatile("" : "+v"(x[s][g]));
    Pend pd[4];  // table loads of steps 14 .. 17 (tile 2's new ones), in flight during tiles 0 and 1
#pragma unroll
    for (int i = 0; i < 4; ++i) pd[i] = tload(4 * (14 + i) - 12 + kk_);
    {  // tile 0: left-fit rows, B operands from the fit matrices in LDS
      doublex4 acc[GI];
#pragma unroll
      for (int g = 0; g < GI; ++g) acc[g] = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < 10; ++s) {
        const double bs = sg_coef(sgs, nF_, li_, 4 * s - 12 + kk_);
#pragma unroll
        for (int g = 0; g < GI; ++g) acc[g] = mfma_f64(x[s][g], bs, acc[g]);
      }
      store(acc, 0, min(kMfV, fl_));
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(pd[i].base));  // corner reads not hoisted above tile 0
    // regular tiles t = 1 .. t_reg - 1, four per iteration so that the ring slots are static.  Tile t
    // consumes steps 4 t .. 4 t + 9; during it, steps 4 t + 10 .. 4 t + 13 are finished from pd (loaded
    // during tile t - 1) and steps 4 t + 14 .. 4 t + 17 are loaded into pd.
    for (int t0 = 1; t0 < t_reg; t0 += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = t0 + u;
        if (t >= t_reg) break;
        Pend nx[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) nx[i] = tload(16 * t + 44 + 4 * i + kk_);
        // steps 4 t + 10 + i -> slot (4 (u + 1) + 10 + i) & 15  (t = t0 + u, t0 = 1 mod 4)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          tfinish(pd[i], x[(4 * (u + 1) + 10 + i) & 15]);
        }
        doublex4 acc[GI];
#pragma unroll
        for (int g = 0; g < GI; ++g) acc[g] = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < 10; ++s) {
          const double bs = bpad[boff + 4 * s];
#pragma unroll
          for (int g = 0; g < GI; ++g) {
            acc[g] = mfma_f64(x[(4 * (u + 1) + s) & 15][g], bs, acc[g]);
          }
        }
        store(acc, kMfV * t, fl_);
#pragma unroll
        for (int i = 0; i < 4; ++i) pd[i] = nx[i];
        // one tile per scheduling region, its samples finished in it
        asm volatile("" ::"v"(x[(4 * (u + 1) + 10) & 15][0]), "v"(x[(4 * (u + 1) + 11) & 15][0]),
                     "v"(x[(4 * (u + 1) + 12) & 15][0]), "v"(x[(4 * (u + 1) + 13) & 15][0]));
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    launder();
    {  // last tile: rows nF - 16 .. nF - 1 (right fit), fresh samples in two groups of 5
      doublex4 acc[GI];
#pragma unroll
      for (int g = 0; g < GI; ++g) acc[g] = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < 10; ++s) {
        const int xi = fl_ - 12 + 4 * s + kk_;
        double xs[GI];
        sample(xi, xs);
        const double bs = sg_coef(sgs, nF_, fl_ + li_, xi);
#pragma unroll
        for (int g = 0; g < GI; ++g) acc[g] = mfma_f64(xs[g], bs, acc[g]);
        if (s == 4) asm volatile("" : "+v"(kk_) : "v"(xs[0]));
      }
      store(acc, fl_, nF_);
    }
  }
}

// per-row L1 norms -> 1 / ||row||_1 (map_fv norm=True: data / norm(data, ord=1, axis=-1))
__global__ __launch_bounds__(256) void row_l1_kernel(const float* __restrict__ data, int64_t b_stride,
                                                      int64_t ch_stride, int32_t nch, int32_t nt,
                                                      float* __restrict__ inv_l1) {
  const int r = blockIdx.x;
  const int b = r / nch, x = r % nch;
  const float* row = data + (int64_t)b * b_stride + (int64_t)x * ch_stride;
  double s = 0.0;
  for (int t = threadIdx.x; t < nt; t += blockDim.x) s += fabs((double)row[t]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  __shared__ double part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) inv_l1[r] = (float)(1.0 / (part[0] + part[1] + part[2] + part[3]));
}

static int last_launch() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_error(-3, hipGetErrorString(e));
}

}  // namespace dvh

using namespace dvh;

DVH_API int dvh_disp_row_l1(const float* data, int64_t b_stride, int64_t ch_stride, int32_t B, int32_t nch,
                            int32_t nt, float* inv_l1, void* stream) {
  if (!data || !inv_l1) return set_error(-2, "null pointer argument");
  if (B * nch <= 0) return 0;
  hipLaunchKernelGGL(row_l1_kernel, dim3(B * nch), dim3(256), 0, (hipStream_t)stream, data, b_stride, ch_stride, nch,
                     nt, inv_l1);
  return last_launch();
}

DVH_API int dvh_disp_tdft(const float* data, int64_t b_stride, int64_t ch_stride, int32_t B, int32_t nch,
                          int32_t nt, const double* wt, int32_t n_fb, const float* row_scale, double* D,
                          void* stream) {
  if (!data || !wt || !D) return set_error(-2, "null pointer argument");
  const int M = B * nch, N = 2 * n_fb;
  if (M <= 0 || N <= 0) return 0;
  static const int rows_env = getenv("DVH_TDFT_ROWS") ? atoi(getenv("DVH_TDFT_ROWS")) : 1;
  if (rows_env && (reinterpret_cast<uintptr_t>(wt) & 15) == 0) {  // N = 2 n_fb is even: 16-byte twiddle pieces
    const int64_t blocks = (int64_t)((M + kTdRows - 1) / kTdRows) * ((N + kTdNT * 16 - 1) / (kTdNT * 16));
    // fewer blocks than a quarter of the CUs: the K-split form (16 waves per block)
    const bool split = blocks * 4 < cu_count() && rows_env != 2;
    const void* fn = split ? (const void*)tdft_rows_kernel<kTdNTs, kTdGs> : (const void*)tdft_rows_kernel<kTdNT, 1>;
    const int NT = split ? kTdNTs : kTdNT, G = split ? kTdGs : 1;
    const size_t lds = tdft_rows_lds(NT, G);
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return set_error(-3, hipGetErrorString(e));
    dim3 grid((M + kTdRows - 1) / kTdRows, (N + NT * 16 - 1) / (NT * 16));
    void* args[] = {(void*)&data, &b_stride, &ch_stride, &nch, (void*)&M, &nt, (void*)&wt, (void*)&N, (void*)&row_scale, &D};
    e = hipLaunchKernel(fn, grid, dim3(256 * G), args, lds, (hipStream_t)stream);
    return e == hipSuccess ? 0 : set_error(-3, hipGetErrorString(e));
  }
  hipError_t e = hipMemsetAsync(D, 0, sizeof(double) * (size_t)M * N, (hipStream_t)stream);
  if (e != hipSuccess) return set_error(-3, hipGetErrorString(e));
  const int tiles = ((M + kGT - 1) / kGT) * ((N + kGT - 1) / kGT);
  // enough K slices for ~1024 waves, at least 64 samples each (more slices measured no faster on
  // 512 gathers: 4 096 / 8 192-wave targets 187 / 188 us vs 167)
  int splits = (1024 + tiles - 1) / tiles;
  int kslice = (nt + splits - 1) / splits;
  kslice = kslice < 64 ? 64 : ((kslice + 3) / 4) * 4;
  splits = (nt + kslice - 1) / kslice;
  dim3 grid((N + kGT - 1) / kGT, (M + kGT - 1) / kGT, splits);
  hipLaunchKernelGGL(tdft_gemm_kernel, grid, dim3(64), 0, (hipStream_t)stream, data, b_stride, ch_stride, nch, M, nt,
                     wt, N, row_scale, kslice, D);
  return last_launch();
}

DVH_API int dvh_disp_fk(const double* D, int32_t B, int32_t nch, int32_t n_fb, const double* atab, int32_t MT,
                        int32_t K2, int32_t n_kb, double* FK, const int32_t* slot, const float* weight,
                        int32_t n_slot, void* stream) {
  if (!D || !atab || !FK) return set_error(-2, "null pointer argument");
  if ((slot == nullptr) != (weight == nullptr)) return set_error(-2, "slot and weight go together");
  if (slot && n_slot <= 0) return set_error(-2, "slot accumulation needs n_slot > 0");
  if (MT % 16 || n_kb > MT || K2 < 2 * nch || K2 % 4) return set_error(-2, "invalid contraction table shape");
  if (B <= 0 || n_fb <= 0) return 0;
  const size_t lds = sizeof(double) * ((size_t)K2 * (kFN + 1) + (size_t)2 * MT * (kFN + 1));
  if (lds > 160 * 1024) return set_error(-4, "too many channels / wavenumbers for one block");
  hipError_t e = hipFuncSetAttribute((const void*)fk_contract_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return set_error(-3, hipGetErrorString(e));
  dim3 grid((n_fb + kFN - 1) / kFN, B);
  hipLaunchKernelGGL(fk_contract_kernel, grid, dim3(256), lds, (hipStream_t)stream, D, nch, n_fb, atab, MT, K2, n_kb,
                     FK, slot, weight, n_slot);
  return last_launch();
}

DVH_API int dvh_disp_fv(const double* FK, int32_t B, int32_t n_kb, int32_t n_fb, const double* kgrid, double kmin,
                        double kmax, const double* kq, int32_t nF, int32_t nV, const int32_t* fj, const double* fw,
                        const double* sg, int32_t sgl, float* fv, void* stream) {
  if (!FK || !kgrid || !kq || !fj || !fw || !sg || !fv) return set_error(-2, "null pointer argument");
  if (n_kb < 2 || n_fb < 2) return set_error(-2, "FK grid needs at least 2 x 2 bins");
  if (sgl % 2 == 0 || sgl > nF) return set_error(-4, "savgol window must be odd and <= number of frequencies");
  if (B <= 0 || nV <= 0) return 0;
  // batched kernel: weights computed once per (f, v) and reused over G images of the block
  // frequency-tiled kernel: tiles of TO outputs (multiple of 4, ~200), the last one >= kSgPad + 1
  {
    const int nt = (nF + 199) / 200;
    int TO = (nF + nt - 1) / nt;
    TO = (TO + 3) & ~3;
    const int last = nF - (nt - 1) * TO;
    int mode = 1;  // the frequency-tiled kernel where it pays (below)
    if (const char* ev = getenv("DVH_FV_TILE")) mode = atoi(ev);  // A/B: 0 = batched / per-image, 2 = always tiled
    const size_t lds_t = sizeof(double) * (size_t)(((size_t)n_kb * n_fb + 1) & ~(size_t)1) +
                         sizeof(double) * (size_t)((sgl * sgl + 1) & ~1) +
                         sizeof(float) * (size_t)kTileVT * (2 * kSgPad + kTileThreads + 4);
    // large batches of long frequency axes only: on few images (the bench's 3 class stacks of
    // 1 000 x 242) the per-image kernel measured faster (1.100 vs 1.125 ms per bench step), and with
    // tiles under 160 outputs (nF = 242: 2 x 124) half the block idles -- the batched kernel packs
    // 4 velocity groups there (sliding bench 16.2 vs 17.6 ms per step)
    const int64_t work = (int64_t)B * nt * ((nV + kFvVT - 1) / kFvVT);  // in 4-velocity units
    if (mode && ((work >= 8192 && TO >= 160) || mode > 1) && last >= kSgPad + 1 && TO + 2 * kSgPad <= kTileThreads &&
        nF >= sgl && lds_t <= 64 * 1024) {
      constexpr int VT = kTileVT;
      hipError_t e = hipFuncSetAttribute((const void*)fv_tile_kernel<VT, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)lds_t);
      if (e != hipSuccess) return set_error(-3, hipGetErrorString(e));
      const int nvc = (nV + VT - 1) / VT;
      const int64_t pairs = (int64_t)nt * nvc;
      int G = (int)((pairs * B + 8191) / 8192);  // ~8 k blocks, at most 64 images each
      G = G < 1 ? 1 : (G > 64 ? 64 : G);
      if (const char* ev = getenv("DVH_FV_TG")) G = atoi(ev) > 0 ? atoi(ev) : G;
      dim3 grid(nt, nvc, (B + G - 1) / G);
      hipLaunchKernelGGL((fv_tile_kernel<VT, false>), grid, dim3(kTileThreads), lds_t, (hipStream_t)stream, FK, B, G,
                         n_kb, n_fb, kgrid, kmin, kmax, kq, nF, nV, TO, fj, fw, sg, sgl, fv, nullptr, nullptr, 0,
                         nullptr);
      return last_launch();
    }
  }
  int n_grp = nF <= kFvThreads ? kFvThreads / nF : 0;
  n_grp = n_grp > 8 ? 8 : n_grp;
  if (n_grp > 0) {
    const int VC = kFvVT * n_grp;
    const size_t lds_b = 2 * sizeof(double) * (size_t)(((size_t)n_kb * n_fb + 1) & ~(size_t)1) +
                         sizeof(double) * (size_t)((sgl * sgl + 1) & ~1) + sizeof(float) * (size_t)VC * (((nF + 3) & ~3) + 2 * kSgPad);
    if ((int64_t)n_kb * n_fb <= (int64_t)kFvPre * kFvThreads && lds_b <= 150 * 1024) {
      hipError_t e = hipFuncSetAttribute((const void*)fv_batch_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)lds_b);
      if (e != hipSuccess) return set_error(-3, hipGetErrorString(e));
      const int nvc = (nV + VC - 1) / VC;
      // images per block: enough blocks to fill the chip (>= ~2048), at most 16 images each
      // images per block: 1 024 blocks (4 per CU) amortise the per-block weights best (measured
      // G = 64 > 16 > 4 on 512 images of 512 x 1000); below ~1 024 (v-chunk, image) pairs the
      // per-image kernel's 256-thread blocks fill the chip better
      int G = (int)(((int64_t)B * nvc + 1023) / 1024);
      G = G < 1 ? 1 : (G > 64 ? 64 : G);
      if ((int64_t)B * nvc < 1024) G = 0;
      if (const char* ev = getenv("DVH_FV_G")) G = atoi(ev);  // A/B: images per block (0: per-image kernel)
      if (G > 0) {
      dim3 grid(nvc, (B + G - 1) / G);
      hipLaunchKernelGGL(fv_batch_kernel, grid, dim3(kFvThreads), lds_b, (hipStream_t)stream, FK, B, G, n_kb, n_fb,
                         kgrid, kmin, kmax, kq, nF, nV, n_grp, fj, fw, sg, sgl, fv);
      return last_launch();
      }
    }
  }
  const size_t lds = sizeof(float) * (size_t)nF * kVS;
  if (lds > 160 * 1024) return set_error(-4, "too many frequencies for one block");
  hipError_t e = hipFuncSetAttribute((const void*)fv_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return set_error(-3, hipGetErrorString(e));
  dim3 grid((nV + kVC - 1) / kVC, B);
  hipLaunchKernelGGL(fv_kernel, grid, dim3(256), lds, (hipStream_t)stream, FK, n_kb, n_fb, kgrid, kmin, kmax, kq, nF,
                     nV, fj, fw, sg, sgl, fv);
  return last_launch();
}

DVH_API int dvh_disp_fv_cells(const double* FK, int32_t B, int32_t n_kb, int32_t n_fb, const double* kgrid, double kmin,
                              double kmax, const double* kq, int32_t nF, int32_t nV, const double* fw, const double* sg,
                              int32_t sgl, int32_t TO, int32_t n_tile, int32_t VT, int32_t max_cell,
                              const int32_t* cell_off, const int32_t* n_cell, const int32_t* qidx, float* fv,
                              void* stream) {
  if (!FK || !kgrid || !kq || !fw || !sg || !fv || !cell_off || !n_cell || !qidx)
    return set_error(-2, "null pointer argument");
  if (n_kb < 2 || n_fb < 2) return set_error(-2, "FK grid needs at least 2 x 2 bins");
  if (sgl != 2 * kSgPad + 1 && (sgl % 2 == 0 || sgl > nF)) return set_error(-4, "savgol window must be odd and <= nF");
  if (VT != kFvVT) return set_error(-4, "cell tables are built for 4 velocities per block");
  if (TO <= 0 || TO % 4 || n_tile <= 0 || (int64_t)(n_tile - 1) * TO >= nF || (int64_t)n_tile * TO < nF)
    return set_error(-2, "tile width / count do not cover the frequencies");
  if (max_cell <= 0 || max_cell > 8192) return set_error(-4, "cell table wider than 8192 cells");
  for (int t = 0; t < n_tile; ++t) {  // every tile's sampled span (with its halo) fits the block
    const int f_lo = t * TO, f_hi = nF < f_lo + TO ? nF : f_lo + TO;
    const int s0 = f_lo - kSgPad > 0 ? f_lo - kSgPad : 0;
    const int s1 = nF < (f_hi + kSgPad > sgl ? f_hi + kSgPad : sgl) ? nF : (f_hi + kSgPad > sgl ? f_hi + kSgPad : sgl);
    if (s1 - s0 > kTileThreads || (f_hi - f_lo + 3) / 4 > 64) return set_error(-4, "tile wider than the block");
    if (t == n_tile - 1 && f_hi - f_lo < kSgPad + 1 && n_tile > 1) return set_error(-4, "last tile too narrow");
  }
  if (B <= 0 || nV <= 0) return 0;
  const size_t lds = sizeof(double) * (size_t)((max_cell + 1) & ~1) + sizeof(double) * (size_t)((sgl * sgl + 1) & ~1) +
                     sizeof(float) * (size_t)kFvVT * (2 * kSgPad + kTileThreads + 4);
  hipError_t e = hipFuncSetAttribute((const void*)fv_tile_kernel<kFvVT, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return set_error(-3, hipGetErrorString(e));
  const int nvc = (nV + kFvVT - 1) / kFvVT;
  const int64_t pairs = (int64_t)n_tile * nvc;
  int G = (int)((pairs * B + 8191) / 8192);  // ~8 k blocks, at most 64 images each
  G = G < 1 ? 1 : (G > 64 ? 64 : G);
  if (const char* ev = getenv("DVH_FV_TG")) G = atoi(ev) > 0 ? atoi(ev) : G;
  dim3 grid(n_tile, nvc, (B + G - 1) / G);
  hipLaunchKernelGGL((fv_tile_kernel<kFvVT, true>), grid, dim3(kTileThreads), lds, (hipStream_t)stream, FK, B, G, n_kb,
                     n_fb, kgrid, kmin, kmax, kq, nF, nV, TO, (const int32_t*)nullptr, fw, sg, sgl, fv, cell_off, n_cell,
                     max_cell, (const int4*)qidx);
  return last_launch();
}

DVH_API int dvh_disp_fv_mfma(const double* FK, int32_t B, int32_t n_kb, int32_t n_fb, const double* hx,
                             const int32_t* cb, int32_t nF, int32_t nV, const double* fw, const double* sg, int32_t sgl,
                             int32_t G, float* fv, void* stream) {
  if (!FK || !hx || !cb || !fw || !sg || !fv) return set_error(-2, "null pointer argument");
  if (n_kb < 2 || n_fb < 2) return set_error(-2, "FK grid needs at least 2 x 2 bins");
  if (sgl != 2 * kSgPad + 1) return set_error(-4, "the MFMA f-v kernel is built for savgol window 25");
  if (nF < 2 * kMfV) return set_error(-4, "the MFMA f-v kernel needs at least 32 frequencies");
  if ((int64_t)n_kb * n_fb > 8192) return set_error(-4, "FK grid larger than 8192 bins");
  if ((int64_t)nF * nV > 0x7fffffff) return set_error(-4, "f-v grid larger than 2^31 points");
  if (B <= 0 || nV <= 0) return 0;
  constexpr int GI = kMfGI;
  const size_t lds = fv_mfma_lds(GI, n_kb * n_fb);
  hipError_t e = hipFuncSetAttribute((const void*)fv_mfma_kernel<GI>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return set_error(-3, hipGetErrorString(e));
  const int n_vb = (nV + kMfWaves * kMfV - 1) / (kMfWaves * kMfV);
  if (G <= 0) {  // ~2 k blocks, at most 16 images each, a multiple of GI
    G = (int)(((int64_t)n_vb * B) / 2048);
    G = G < GI ? GI : (G > 16 ? 16 : G);
  }
  G = (G + GI - 1) / GI * GI;
  const int n_ig = (B + G - 1) / G;
  const int xcd_map = (n_vb % 8 == 0) ? 1 : 0;
  const int64_t n_blk = (int64_t)n_vb * n_ig;
  if (n_blk > 0x7fffffff) return set_error(-4, "grid too large");
  hipLaunchKernelGGL(fv_mfma_kernel<GI>, dim3((unsigned)n_blk), dim3(kMfWaves * 64), lds, (hipStream_t)stream, FK, B, G,
                     n_kb, n_fb, (const double2*)hx, cb, nF, nV, (const double2*)fw, sg, fv, n_vb, xcd_map);
  return last_launch();
}
