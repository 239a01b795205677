// Per-pass windowing, taper and bandpass on MI355X (gfx950).
//
//   dvh_sosfiltfilt  bandpass_data (modules/utils.py:179-189): scipy.signal.sosfiltfilt(sos, x, axis=1)
//                    = odd extension by padlen, sosfilt with zi * x_ext[0], reverse, sosfilt with
//                    zi * y[-1], reverse, trim.  Float64 recursion, time-parallel over blocks of each
//                    trace (zero-state block filters + a state scan + re-filter, below).
//   dvh_mute_traj    SurfaceWaveWindow.mute_along_traj (apis/data_classes.py:49-72): column t is
//                    multiplied by a tukey taper placed along the vehicle trajectory (host tables).
//   dvh_mute_time    SurfaceWaveWindow.mute_along_time (apis/data_classes.py:100-104).
//   dvh_trace_cleanup  the rest of TimeLapseImaging._preprocessing_for_surface_waves
//                    (apis/timeLapseImaging.py:51-71) after the bandpass: find_noise_idx /
//                    impute_noisy_trace (modules/utils.py:316-329) for empty traces (L2 norm below
//                    the threshold) then noisy traces (max above it), then the per-trace L2 norm.
// Data may be float32 (dtype 0) or float64 (dtype 1), modified in place.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>

#include <algorithm>

#include "dvh_common.h"
#include "dvh.h"

namespace dvh {

constexpr int kMaxSec = 16;

// orders one wave's LDS stores and loads (a single-wave block: the fence keeps the compiler from moving them)
__device__ __forceinline__ void wave_barrier_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------------------------------------
// sosfiltfilt, time-parallel.  The cascade of n_sec transposed-direct-form-II sections (scipy's sosfilt:
// o = b0 v + z0; z0 = b1 v - a1 o + z1; z1 = b2 v - a2 o) is linear in its 2 n_sec states, so a sequence
// u[0, n_ext) cut into blocks of L samples is filtered block-parallel in three phases:
//   A  every block except the last is filtered from ZERO state (block 0 from the true initial state
//      zi * u[0]), keeping only its end state e_k;
//   B  per row, the true end states follow by a scan over the blocks, s_k = e_k + M s_{k-1} with
//      M = A^L the zero-input state transition of L samples (sos_transition_kernel forms it on the
//      device with the filter's own arithmetic);
//   C  every block is filtered again from its true start state s_{k-1} and writes its outputs.
// sosfiltfilt = the forward pass over the odd extension ext(x) (zi * ext[0]), then the backward pass over
// the reversed forward output y (zi * y[-1]), trimmed by padlen.  One lane per (row, block): n_rows x n_ext
// / L lanes instead of n_rows (a 1 024-trace record filled 16 of the chip's 1 024 SIMDs with one lane per
// trace).  The poles of the order-10 band (1.2 Hz at fs = 250 Hz) sit about 1e-2 inside the unit circle,
// so M is a contraction and the scan is well conditioned.
template <int NS>
struct SosCoef {
  double b0[NS], b1[NS], b2[NS], a1[NS], a2[NS];
  __device__ __forceinline__ void load(const double* __restrict__ sos) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      b0[s] = sos[6 * s];
      b1[s] = sos[6 * s + 1];
      b2[s] = sos[6 * s + 2];
      a1[s] = sos[6 * s + 4];
      a2[s] = sos[6 * s + 5];
    }
  }
  // one sample through the cascade (scipy's sosfilt expressions)
  __device__ __forceinline__ double step(double (&z0)[NS], double (&z1)[NS], double v) const {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const double o = b0[s] * v + z0[s];
      z0[s] = b1[s] * v - a1[s] * o + z1[s];
      z1[s] = b2[s] * v - a2[s] * o;
      v = o;
    }
    return v;
  }
};

// The filtered sequence u of a row: the odd extension of x (forward pass) or the reversed forward output.
template <typename T, bool BWD>
struct SosInput {
  const T* row;      // forward: the row of x
  const double* y;   // backward: the row's forward output [n_ext]
  int64_t n_t, n_ext, padlen;
  double x0, xn;
  __device__ __forceinline__ double operator()(int64_t i) const {
    if (BWD) return y[n_ext - 1 - i];
    if (i < padlen) return 2.0 * x0 - (double)row[padlen - i];
    const int64_t j = i - padlen;
    if (j < n_t) return (double)row[j];
    return 2.0 * xn - (double)row[n_t - 2 - (j - n_t)];
  }
};

struct SosGeom {
  int64_t n_rows, row_stride;
  int32_t n_t, padlen, L, nb;
  int64_t n_ext;
};

template <typename T, bool BWD>
__device__ __forceinline__ SosInput<T, BWD> sos_input(const T* x, const double* y, const SosGeom& G, int64_t r) {
  SosInput<T, BWD> u;
  u.row = x + r * G.row_stride;
  u.y = y + r * G.n_ext;
  u.n_t = G.n_t;
  u.n_ext = G.n_ext;
  u.padlen = G.padlen;
  if (!BWD) {
    u.x0 = (double)u.row[0];
    u.xn = (double)u.row[G.n_t - 1];
  } else {
    u.x0 = u.xn = 0.0;
  }
  return u;
}

// M[j][m] (row-major, 2 NS states ordered z0[0], z1[0], z0[1], ...): the state after L zero-input samples
// from the unit state e_m.  One wave, lane m < 2 NS.
template <int NS>
__global__ __launch_bounds__(64) void sos_transition_kernel(const double* __restrict__ sos, int32_t L,
                                                             double* __restrict__ M) {
  constexpr int NST = 2 * NS;
  const int m = threadIdx.x;
  if (m >= NST) return;
  SosCoef<NS> c;
  c.load(sos);
  double z0[NS], z1[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    z0[s] = (2 * s == m) ? 1.0 : 0.0;
    z1[s] = (2 * s + 1 == m) ? 1.0 : 0.0;
  }
  for (int i = 0; i < L; ++i) c.step(z0, z1, 0.0);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    M[(2 * s) * NST + m] = z0[s];
    M[(2 * s + 1) * NST + m] = z1[s];
  }
}

// Phases A (OUT = false: end states of blocks k < nb - 1 into S) and C (OUT = true: filter from the true start
// state S[k - 1] and write the outputs: y[i] forward, the trimmed row backward).  One wave per 64 consecutive
// lanes g = r * nb + k.  A lane's block is a run of L samples at its own address, so direct per-lane loads
// would touch 64 cache lines per instruction; instead the wave moves its 64 runs in chunks of kSosCh samples
// through an LDS tile: cooperative loads (16 lanes per run: each instruction reads 4 contiguous runs of 16
// samples), the recursion on the lane's own tile row, and (phase C) the outputs written back into the same
// tile slots and stored cooperatively, again 16 contiguous samples per 16 lanes.
constexpr int kSosCh = 16;           // samples per chunk (L is a multiple of 32)
constexpr int kSosLd = kSosCh + 1;   // tile row stride in doubles: conflict-free own-row reads
template <typename T, int NS, bool BWD, bool OUT>
__global__ __launch_bounds__(64) void sos_block_kernel(T* __restrict__ x, double* __restrict__ y, SosGeom G,
                                                        const double* __restrict__ sos, const double* __restrict__ zi,
                                                        double* __restrict__ S) {
  constexpr int NST = 2 * NS;
  __shared__ double tile[64 * kSosLd];
  const int lane = threadIdx.x;
  const int64_t n_lanes = G.n_rows * G.nb;
  const int64_t g0 = (int64_t)blockIdx.x * 64;
  const int64_t g = g0 + lane;
  const bool act = g < n_lanes && (OUT || (g % G.nb) != G.nb - 1);  // phase A: no end state of the last block
  const int64_t r = act ? g / G.nb : 0;
  const int k = act ? (int)(g - r * G.nb) : 0;
  const int64_t i0 = (int64_t)k * G.L, i1 = act ? min(i0 + G.L, G.n_ext) : i0;
  // this lane's part of the cooperative moves: runs s = 4 m + (lane >> 4), samples e = lane & 15 of a chunk
  const int e = lane & 15;
  SosCoef<NS> c;
  c.load(sos);
  double z0[NS], z1[NS];
  double* Sr = S + g * NST;  // S[r][k]
  if (act && k == 0) {
    const SosInput<T, BWD> u = sos_input<T, BWD>(x, y, G, r);
    const double u0 = u(0);
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      z0[q] = zi[2 * q] * u0;
      z1[q] = zi[2 * q + 1] * u0;
    }
  } else if (act && OUT) {
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      z0[q] = Sr[-NST + 2 * q];
      z1[q] = Sr[-NST + 2 * q + 1];
    }
  } else {
#pragma unroll
    for (int q = 0; q < NS; ++q) z0[q] = z1[q] = 0.0;
  }
  // the longest run of the wave (every block but a row's last has L samples)
  int64_t n_chunks = 0;
  {
    const int64_t len = i1 - i0;
    int64_t mx = len;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (int64_t)__shfl_xor((long long)mx, o));
    n_chunks = (mx + kSosCh - 1) / kSosCh;
  }
  // run s = 4 m + (lane >> 4) of the wave is lane g0 + s: its (row, block) by stepping 4 lanes per m
  const int l4 = lane >> 4;
  const int64_t gl = g0 + l4;
  const int64_t r_l = gl / G.nb;
  const int k_l = (int)(gl - r_l * G.nb);
  // sample i of run (rs, ks): the sequence the pass filters (forward: the odd extension of x; backward: the
  // forward output reversed)
  auto in_at = [&](int64_t rs, int64_t i) -> double {
    if (BWD) return y[rs * G.n_ext + (G.n_ext - 1 - i)];
    const T* row = x + rs * G.row_stride;
    const int64_t j = i - G.padlen;
    if (j >= 0 && j < G.n_t) return (double)row[j];
    if (j < 0) return 2.0 * (double)row[0] - (double)row[-j];                    // i < padlen
    return 2.0 * (double)row[G.n_t - 1] - (double)row[2 * (G.n_t - 1) - j];     // past the end
  };
  // cooperative load of chunk ch into registers (this lane's 16 values: runs 4 m + l4, sample e)
  double pv[16];
  auto coop_load = [&](int64_t cbase) {
    int64_t rs = r_l;
    int ks = k_l;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      double v = 0.0;
      if (g0 + 4 * m + l4 < n_lanes) {
        const int64_t i = (int64_t)ks * G.L + cbase + e;
        if (i < min((int64_t)(ks + 1) * G.L, G.n_ext)) v = in_at(rs, i);
      }
      pv[m] = v;
      ks += 4;
      while (ks >= G.nb) {
        ks -= G.nb;
        ++rs;
      }
    }
  };
  if (n_chunks > 0) coop_load(0);
  for (int64_t ch = 0; ch < n_chunks; ++ch) {
    const int64_t cbase = ch * kSosCh;
#pragma unroll
    for (int m = 0; m < 16; ++m) tile[(4 * m + l4) * kSosLd + e] = pv[m];
    __syncthreads();
    if (ch + 1 < n_chunks) coop_load(cbase + kSosCh);  // the next chunk's loads in flight under this one's recursion
    const int64_t nn = min((int64_t)kSosCh, i1 - i0 - cbase);
    if (OUT) {
      for (int t = 0; t < nn; ++t) tile[lane * kSosLd + t] = c.step(z0, z1, tile[lane * kSosLd + t]);
    } else {
      for (int t = 0; t < nn; ++t) c.step(z0, z1, tile[lane * kSosLd + t]);
    }
    __syncthreads();
    if (OUT) {  // cooperative store of the outputs
      int64_t rs = r_l;
      int ks = k_l;
#pragma unroll 4
      for (int m = 0; m < 16; ++m) {
        const int sidx = 4 * m + l4;
        if (g0 + sidx < n_lanes) {
          const int64_t i = (int64_t)ks * G.L + cbase + e;
          if (i < min((int64_t)(ks + 1) * G.L, G.n_ext)) {
            const double v = tile[sidx * kSosLd + e];
            if (!BWD) {
              y[rs * G.n_ext + i] = v;
            } else {
              // reversed index i is sample n_ext - 1 - i of the extension; the row keeps [padlen, padlen + n_t)
              const int64_t j = G.n_ext - 1 - i - G.padlen;
              if (j >= 0 && j < G.n_t) x[rs * G.row_stride + j] = (T)v;
            }
          }
        }
        ks += 4;
        while (ks >= G.nb) {
          ks -= G.nb;
          ++rs;
        }
      }
      __syncthreads();
    }
  }
  if (!OUT && act) {
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      Sr[2 * q] = z0[q];
      Sr[2 * q + 1] = z1[q];
    }
  }
}

// Phase B: s_k = e_k + M s_{k-1} for k = 1 .. nb - 2 (s_0 = e_0 is already the true state).  Two rows per
// wave (lanes 0-31 / 32-63), lane j = state component j.  Each step's state goes through LDS: one 8-byte store
// per lane, then every lane reads the half's whole state with broadcast 16-byte reads (no per-element
// cross-lane shuffles on the step's critical path).
template <int NS>
__global__ __launch_bounds__(64) void sos_scan_kernel(SosGeom G, const double* __restrict__ M, double* __restrict__ S) {
  constexpr int NST = 2 * NS;
  __shared__ __attribute__((aligned(16))) double sv[2][32];
  const int half = threadIdx.x >> 5, j = threadIdx.x & 31;
  const int64_t r = 2 * (int64_t)blockIdx.x + half;
  const bool act = r < G.n_rows && j < NST;
  double m[NST];
#pragma unroll
  for (int i = 0; i < NST; ++i) m[i] = act ? M[j * NST + i] : 0.0;
  double* Sr = S + (act ? r : 0) * (int64_t)G.nb * NST;
  sv[half][j] = act ? Sr[j] : 0.0;
  // the zero-state end states e_k come from memory 8 steps at a time, the next 8 loaded under this group's
  // arithmetic (a load per step would put one memory latency on the critical path of every step)
  constexpr int PF = 8;
  const int kend = G.nb - 1;  // steps k = 1 .. nb - 2
  double cur[PF], nxt[PF];
#pragma unroll
  for (int t = 0; t < PF; ++t) cur[t] = (act && 1 + t < kend) ? Sr[(int64_t)(1 + t) * NST + j] : 0.0;
  for (int kb = 1; kb < kend; kb += PF) {
#pragma unroll
    for (int t = 0; t < PF; ++t) {
      const int k = kb + PF + t;
      nxt[t] = (act && k < kend) ? Sr[(int64_t)k * NST + j] : 0.0;
    }
#pragma unroll
    for (int t = 0; t < PF; ++t) {
      const int k = kb + t;
      if (k < kend) {
        wave_barrier_lds();
        const double2* v2 = reinterpret_cast<const double2*>(sv[half]);
        double x[NST];
#pragma unroll
        for (int i = 0; i < NST / 2; ++i) {
          const double2 u = v2[i];
          x[2 * i] = u.x;
          x[2 * i + 1] = u.y;
        }
        // M s in four partial sums (a 5-deep instead of a 20-deep chain of dependent FMAs per step)
        double pa[4] = {cur[t], 0.0, 0.0, 0.0};
#pragma unroll
        for (int i = 0; i < NST; ++i) pa[i & 3] += m[i] * x[i];
        const double acc = (pa[0] + pa[1]) + (pa[2] + pa[3]);
        if (act) Sr[(int64_t)k * NST + j] = acc;
        wave_barrier_lds();
        sv[half][j] = acc;
      }
    }
#pragma unroll
    for (int t = 0; t < PF; ++t) cur[t] = nxt[t];
  }
}

// ---------------------------------------------------------------------------------------------
// sosfiltfilt on the float64 matrix pipe (round 5).  With blocks of kSmL = 64 samples the phases A and C above are
// GEMMs whose operands are the block's samples and the filter's block operators, formed on the device from the
// filter's own recursion (sosm_mats_kernel):
//   h[t]       the cascade's impulse response (zero state, unit sample at step 0), t < L
//   Hm[t][m]   its output at step t from the unit state e_m and zero input
//   g[t][m]    its state after step t from the unit sample at step 0 (zero state)
//   M = A^L    the zero-input transition of L samples, Mzi = M zi, MQ = M^Q (the scan's group transition)
// A block of L samples u_0..u_{L-1} filtered from start state s gives
//   outputs   y_i = sum_{j <= i} h[i - j] u_j + sum_m Hm[i][m] s_m            (lower-triangular Toeplitz + L x 2NS)
//   end state s' = M s + sum_j g[L - 1 - j] u_j                                 (2NS x L)
// and the backward pass over the reversed forward output, in forward indexing i of the same block (backward
// blocks aligned with the forward ones; the partial last forward block is the first backward block):
//   outputs   v_i = sum_{i'' >= i} h[i'' - i] y_i'' + sum_m Hm[L - 1 - i][m] s_m  (upper-triangular Toeplitz)
//   end state s' = M s + sum_i g[i] y_i
// The products are v_mfma_f64_16x16x4_f64 tiles over 16 blocks (columns, 1 024 samples).  A tile's samples are moved
// by coalesced loads (issued one tile ahead, under the previous tile's MFMAs) into an LDS image [block][sample]
// (row stride 65 doubles: the B-operand reads are conflict-free), and its outputs leave through the same image by
// coalesced stores.  The GEMMs fed from the image take their k index in the order sample = 16 (l >> 4) + kk, those
// fed from accumulators (the backward end states) in the accumulator order sample = 4 kk + (l >> 4); the operator
// (A) values are read from small LDS tables (h zero-extended for the Toeplitz factors, Hm, g) by lane-constant
// offsets.  Launches:
//   sosm_mats   the operators (one wave per record)
//   sosm_fa     forward zero-state end states E_f (block 0 plus M zi x_ext[0]: its true end state)
//   sosm_scan   true forward end states (two-level, below)
//   sosm_fc     forward outputs y from the true start states, written once, and from the same accumulators the
//               backward zero-state end states E_b of every full block (the backward phase A, fused)
//   sosm_bf     the first backward block (the partial last forward block) by the recursion, one lane per row
//   sosm_scan   true backward end states
//   sosm_bc     backward outputs from the true start states, trimmed into the row
// The outputs equal the recursion's up to rounding (sums of <= 84 products per output instead of the cascade's chain;
// a float64 model of this scheme matches scipy.signal.sosfiltfilt to 1e-13); tests/test_prep_gpu.py holds them to
// scipy at 1e-10 (float64) / 2e-6 (float32).
constexpr int kSmL = 64;     // samples per block: four 16-row MFMA tiles
constexpr int kSmLd = 65;  // LDS image row stride (doubles), odd: the B-operand reads (column li, sample 4 kk + q),
                           // which the compiler pairs into ds_read2_b64 (16-lane groups, 32 banks), and the
                           // accumulator stores (ds_write_b64, 16-lane groups) of the 16 columns land on 16 distinct
                           // bank pairs (at 66 they fell on 8: 2-way conflicts; conflict cycles per LDS instruction
                           // fa / fc / bc 1.73 / 3.44 / 2.51 -> 0.23 / 0.22 / 0.15, profiles/r6_pmc_prep_sosm.json)
constexpr int kSmOcc = 3;  // sosm_fa / sosm_bc: waves per SIMD the registers are sized for (their LDS allows 3 blocks
                           // of 4 waves per CU; sosm_fc's 65 KB and 220 registers hold it at 2)
constexpr int kSmRows = 32;  // state rows of the MFMA tiles (2 NS <= 32)
typedef double doublex4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ doublex4_t mfma_f64x4(double a, double b, doublex4_t c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// offsets (doubles) of the filter operators in the MFMA path's table (the "plan")
template <int NS>
struct SosmMats {
  static constexpr int NST = 2 * NS;
  static constexpr int h = 0, Hm = kSmL, g = Hm + kSmL * NST, M = g + kSmL * NST, Mzi = M + NST * NST,
                       MQ = Mzi + NST, MQ16 = MQ + NST * NST, Qk = MQ16 + NST * NST, size = Qk + 2;
};
// + the key (Q, Q16) the group transitions MQ / MQ16 were formed for: a scan whose own Q differs (a plan built for
// another record length) uses a NaN transition, so that the mismatch shows in the output instead of a wrong filter
constexpr int64_t sosm_plan_doubles(int n_sec) {
  return kSmL + 2 * kSmL * (2 * n_sec) + 3 * (2 * n_sec) * (2 * n_sec) + 2 * n_sec + 2;
}
// M^Q from the plan for a scan of group length Q: NaN when the plan's key is another Q
template <int NS>
__device__ __forceinline__ double sosm_mq(const double* __restrict__ mats, bool q16, int32_t Q, int idx) {
  using O = SosmMats<NS>;
  const double v = mats[(q16 ? O::MQ16 : O::MQ) + idx];
  return mats[O::Qk + (q16 ? 1 : 0)] == (double)Q ? v : __builtin_nan("");
}

// Lanes e < NST: unit state e_e, zero input (Hm[:, e], M[:, e]); lane NST: zero state, unit sample (h, g).  Then
// Mzi = M zi, MQ = M^Q and MQ16 = M^Q16 by repeated products (threads (row, col) of the 20 x 20 result, LDS): the
// group transitions of the 8-group scans (sosm_scan_kernel, sosm_scanr_kernel) and the 16-group one (sosm_scanm).
template <int NS>
__global__ __launch_bounds__(512) void sosm_mats_kernel(const double* __restrict__ sos, const double* __restrict__ zi,
                                                        int32_t Q, int32_t Q16, double* __restrict__ mats) {
  using O = SosmMats<NS>;
  constexpr int NST = 2 * NS;
  __shared__ double P[NST * NST], R[NST * NST], M0[NST * NST];
  const int e = threadIdx.x;
  if (e <= NST) {
    SosCoef<NS> c;
    c.load(sos);
    double z0[NS], z1[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      z0[s] = (2 * s == e) ? 1.0 : 0.0;
      z1[s] = (2 * s + 1 == e) ? 1.0 : 0.0;
    }
    for (int t = 0; t < kSmL; ++t) {
      const double o = c.step(z0, z1, (e == NST && t == 0) ? 1.0 : 0.0);
      if (e == NST) {
        mats[O::h + t] = o;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          mats[O::g + t * NST + 2 * s] = z0[s];
          mats[O::g + t * NST + 2 * s + 1] = z1[s];
        }
      } else {
        mats[O::Hm + t * NST + e] = o;
      }
    }
    if (e < NST) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        P[(2 * s) * NST + e] = z0[s];
        P[(2 * s + 1) * NST + e] = z1[s];
      }
    }
  }
  __syncthreads();
  const int row = e / NST, col = e % NST;
  const bool act = e < NST * NST;
  if (act) {
    mats[O::M + e] = P[e];
    M0[e] = P[e];
  }
  if (e < NST) {
    double a = 0.0;
    for (int j = 0; j < NST; ++j) a += P[e * NST + j] * zi[j];
    mats[O::Mzi + e] = a;
  }
  // M^q by binary powering: R *= P when the bit is set, P = P P (P restarts from M)
  for (int pass = 0; pass < 2; ++pass) {
    __syncthreads();
    if (act) {
      P[e] = M0[e];
      R[e] = row == col ? 1.0 : 0.0;  // R = M^0
    }
    for (int q = pass == 0 ? Q : Q16; q > 0; q >>= 1) {
      __syncthreads();
      if (q & 1) {
        double a = 0.0;
        if (act)
          for (int j = 0; j < NST; ++j) a += R[row * NST + j] * P[j * NST + col];
        __syncthreads();
        if (act) R[e] = a;
        __syncthreads();
      }
      if (q > 1) {
        double a = 0.0;
        if (act)
          for (int j = 0; j < NST; ++j) a += P[row * NST + j] * P[j * NST + col];
        __syncthreads();
        if (act) P[e] = a;
      }
    }
    __syncthreads();
    if (act) mats[(pass == 0 ? O::MQ : O::MQ16) + e] = R[e];
  }
  if (e < 2) mats[O::Qk + e] = (double)(e == 0 ? Q : Q16);
}

// sample i of row r of the forward pass's sequence: the odd extension of x (0 past n_ext)
template <typename T>
__device__ __forceinline__ double sosm_ext(const T* __restrict__ x, const SosGeom& G, int64_t r, int64_t i) {
  if (r >= G.n_rows || i >= G.n_ext) return 0.0;  // padding columns of a record's last tile: nothing to read
  const T* row = x + r * G.row_stride;
  const int64_t j = i - G.padlen;
  if (j >= 0 && j < G.n_t) return (double)row[j];
  if (j < 0) return 2.0 * (double)row[0] - (double)row[-j];
  return 2.0 * (double)row[G.n_t - 1] - (double)row[2 * (G.n_t - 1) - j];
}

// Operator tables in LDS, laid out so that the lane-constant A-operand reads of a 32-lane group spread over the banks
// (k index = sample 4 kk + q, or state KS q + q'):
//   hq[q][64 + d] = h[d] (0 for d < 0) and hr[q][64 + d] = h[-d], one copy per lane group q at stride 145: the
//     Toeplitz factors T[i][j] = h[i - j] = hq[q][64 + i - j] and U[i][j] = h[j - i] = hr[q][64 + i - j]
//   hm[i][m] = Hm[i][m], stride 21;  ga[j][m] = g[L - 1 - j][m], stride 48;  gb[m][i] = g[i][m], stride 66
//   (rows m >= 2 NS zero)
constexpr int kHq = 145, kHmLd = 21, kGaLd = 33, kGbLd = kSmLd;
template <int NS>
__device__ __forceinline__ void sosm_tables(const double* __restrict__ mats, double* hq, double* hr, double* hm, double* ga,
                                            double* gb) {
  using O = SosmMats<NS>;
  constexpr int NST = 2 * NS;
  for (int v = threadIdx.x; v < 4 * kHq; v += blockDim.x) {
    const int d = v % kHq - kSmL;
    if (hq) hq[v] = (d >= 0 && d < kSmL) ? mats[O::h + d] : 0.0;
    if (hr) hr[v] = (d <= 0 && -d < kSmL) ? mats[O::h - d] : 0.0;
  }
  if (hm)
    for (int v = threadIdx.x; v < kSmL * kHmLd; v += blockDim.x) {
      const int i = v / kHmLd, m = v % kHmLd;
      hm[v] = m < NST ? mats[O::Hm + i * NST + m] : 0.0;
    }
  if (ga)
    for (int v = threadIdx.x; v < kSmL * kGaLd; v += blockDim.x) {
      const int j = v / kGaLd, m = v % kGaLd;
      ga[v] = m < NST ? mats[O::g + (kSmL - 1 - j) * NST + m] : 0.0;
    }
  if (gb)
    for (int v = threadIdx.x; v < kSmRows * kGbLd; v += blockDim.x) {
      const int m = v / kGbLd, i = v % kGbLd;
      gb[v] = (m < NST && i < kSmL) ? mats[O::g + i * NST + m] : 0.0;
    }
}

// A tile: 16 consecutive columns c0 .. c0 + 15 of an [n_rows][ncpr] column grid (block k of row r = column r ncpr + k;
// 32-bit: the host checks n_rows * nb < 2^31).  Its 1 024 samples in registers: lane l, step u holds sample l of
// column u (the LDS image [column][sample] is filled from these).
struct SosmTile {
  int c0, r0, k0;
  bool one_row;  // all 16 columns in row r0
};
__device__ __forceinline__ SosmTile sosm_tile(int tile, int n_rows, int ncpr) {
  SosmTile t;
  t.c0 = tile * 16;
  t.r0 = t.c0 / ncpr;
  t.k0 = t.c0 - t.r0 * ncpr;
  t.one_row = t.k0 + 16 <= ncpr && t.r0 < n_rows;
  return t;
}
// (row, block) of column u of a tile
__device__ __forceinline__ void sosm_col(const SosmTile& t, int u, int ncpr, int& r, int& k) {
  if (t.one_row) {
    r = t.r0;
    k = t.k0 + u;
  } else {
    const int c = t.c0 + u;
    r = c / ncpr;
    k = c - r * ncpr;
  }
}

// forward sequence (odd extension of x) of a tile's columns (blocks of the ext, ncpr = nb), in two halves so that the
// loads of the next tile stay in flight under this tile's MFMAs: sosm_fetch_x issues them into registers of x's own
// type (the samples each lane's sample index reflects to, plus the two reflection centres, x[0] of the last column's
// row and x[n_t - 1] of the first's), sosm_expand_x forms the extension from them when the tile is consumed.  (A
// conversion or sum right after a load makes the compiler wait for it there: the prefetch would be a plain load.)
__device__ __forceinline__ bool sosm_interior(const SosGeom& G, const SosmTile& t) {  // all 16 columns inside x's row
  const int64_t e0 = (int64_t)t.k0 * kSmL;
  return t.one_row && e0 >= G.padlen && e0 + 16 * kSmL <= G.padlen + G.n_t;
}
template <typename T>
struct SosmXRaw {
  T v[16];
  T xl, xr;
};
template <typename T>
__device__ __forceinline__ void sosm_fetch_x(const T* __restrict__ x, const SosGeom& G, const SosmTile& t, int lane,
                                             SosmXRaw<T>& raw) {
  const int nr = (int)G.n_rows;
  {
    int rl, kl;
    sosm_col(t, 15, G.nb, rl, kl);
    raw.xl = x[(int64_t)min(rl, nr - 1) * G.row_stride];
    raw.xr = x[(int64_t)min(t.r0, nr - 1) * G.row_stride + G.n_t - 1];
  }
  if (sosm_interior(G, t)) {  // one contiguous run of x
    const T* p = x + (int64_t)t.r0 * G.row_stride + ((int64_t)t.k0 * kSmL - G.padlen) + lane;
#pragma unroll
    for (int u = 0; u < 16; ++u) raw.v[u] = p[64 * u];
  } else {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      int r, k;
      sosm_col(t, u, G.nb, r, k);
      const int64_t j = (int64_t)k * kSmL + lane - G.padlen;
      int64_t src = j < 0 ? -j : (j < G.n_t ? j : 2 * ((int64_t)G.n_t - 1) - j);
      src = src < 0 ? 0 : (src >= G.n_t ? G.n_t - 1 : src);  // past the extension: any valid sample (unused)
      raw.v[u] = x[(int64_t)min(r, nr - 1) * G.row_stride + src];
    }
  }
}
// the tile's extension samples from its fetched raw values; a column whose reflection centre is not in the raw set
// (a tile over more than two rows: records of under 16 blocks) reads x directly
template <typename T>
__device__ __forceinline__ void sosm_expand_x(const T* __restrict__ x, const SosGeom& G, const SosmTile& t, int lane,
                                              const SosmXRaw<T>& raw, double (&v)[16]) {
  if (sosm_interior(G, t)) {
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = (double)raw.v[u];
  } else {
    int rl, kl;
    sosm_col(t, 15, G.nb, rl, kl);
    const double xl = (double)raw.xl, xr = (double)raw.xr;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      int r, k;
      sosm_col(t, u, G.nb, r, k);
      const int64_t i = (int64_t)k * kSmL + lane, j = i - G.padlen;
      const double a = (double)raw.v[u];
      double e = 0.0;  // padding columns (r >= n_rows) and samples past the extension are zero, and read nothing
      if (r < G.n_rows && i < G.n_ext) {
        if (j >= 0 && j < G.n_t)
          e = a;
        else if (j < 0)
          e = r == rl ? 2.0 * xl - a : sosm_ext(x, G, r, i);
        else
          e = r == t.r0 ? 2.0 * xr - a : sosm_ext(x, G, r, i);
      }
      v[u] = e;
    }
  }
}

// forward output y of a tile's columns (ncpr = nb - 1: blocks k < nb - 1 of each row, all full)
__device__ __forceinline__ void sosm_load_y(const double* __restrict__ y, const SosGeom& G, const SosmTile& t, int lane,
                                            double (&v)[16]) {
  if (t.one_row) {  // one contiguous run of the row's y (every column a full block)
    const double* p = y + (int64_t)t.r0 * G.n_ext + (int64_t)t.k0 * kSmL + lane;
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = p[64 * u];
    return;
  }
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    int r, k;
    sosm_col(t, u, G.nb - 1, r, k);
    v[u] = r < G.n_rows ? y[(int64_t)r * G.n_ext + (int64_t)k * kSmL + lane] : 0.0;
  }
}

// register samples -> the wave's LDS image [column][sample]
__device__ __forceinline__ void sosm_to_lds(double* img, int lane, const double (&v)[16]) {
#pragma unroll
  for (int u = 0; u < 16; ++u) img[u * kSmLd + lane] = v[u];
}

// accumulator rows (row i = 16 t + 4 rr + (l >> 4) of column l & 15) -> the LDS image
__device__ __forceinline__ void sosm_acc_to_lds(double* img, int lane, const doublex4_t (&acc)[4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) img[(lane & 15) * kSmLd + 16 * t + 4 * rr + (lane >> 4)] = acc[t][rr];
}

// state accumulators (rows m = 16 t + 4 rr + (l >> 4)) -> the LDS image as [column][sosm_stp(NST)]: an odd row
// stride, so that the 16 columns of a write land in 16 distinct bank pairs (at NST = 20 they fell on 4: 4-way
// conflicts); element (column, m) is read back at sosm_sv(v) for v = column NST + m
__host__ __device__ constexpr int sosm_stp(int nst) { return nst | 1; }
template <int NST>
__device__ __forceinline__ int sosm_sv(int v) { return (v / NST) * sosm_stp(NST) + v % NST; }
template <int NST>
__device__ __forceinline__ void sosm_states_out(double* img, int lane, const doublex4_t (&e)[2]) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int m = 16 * t + 4 * rr + (lane >> 4);
      if (m < NST) img[(lane & 15) * sosm_stp(NST) + m] = e[t][rr];
    }
}

// B operand of k-step kk (sample 4 kk + q of column li) and the Toeplitz A operands
#define SOSM_B(kk) bsrc[4 * (kk)]

// Forward phase A: E_f[c] = G u_block for k < nb - 1 (block 0: + M zi u_0, its true end state).
template <typename T, int NS>
__global__ __launch_bounds__(256, kSmOcc) void sosm_fa_kernel(const T* __restrict__ x, SosGeom G, const double* __restrict__ mats,
                                                      double* __restrict__ Sf) {
  using O = SosmMats<NS>;
  constexpr int NST = 2 * NS;
  __shared__ double ga[kSmL * kGaLd], imgs[4][16 * kSmLd];
  sosm_tables<NS>(mats, nullptr, nullptr, nullptr, ga, nullptr);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double* img = imgs[wave];
  const int q = lane >> 4, li = lane & 15;
  const int nr = (int)G.n_rows;
  const int n_tiles = (nr * G.nb + 15) / 16, stride = gridDim.x * 4;
  int tile = blockIdx.x * 4 + wave;
  // M zi rows m = 16 t + 4 rr + q of this lane (block 0's true end state adds M zi u_0)
  double mzi[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int m = 16 * t + 4 * rr + q;
      mzi[t][rr] = m < NST ? mats[O::Mzi + m] : 0.0;
    }
  SosmXRaw<T> raw;
  if (tile < n_tiles) sosm_fetch_x(x, G, sosm_tile(tile, nr, G.nb), lane, raw);
  for (; tile < n_tiles; tile += stride) {
    const SosmTile tl = sosm_tile(tile, nr, G.nb);
    {
      double v[16];
      sosm_expand_x(x, G, tl, lane, raw, v);
      wave_barrier_lds();
      sosm_to_lds(img, lane, v);
    }
    if (tile + stride < n_tiles) sosm_fetch_x(x, G, sosm_tile(tile + stride, nr, G.nb), lane, raw);  // next tile
    wave_barrier_lds();
    doublex4_t acc[2] = {doublex4_t{0.0, 0.0, 0.0, 0.0}, doublex4_t{0.0, 0.0, 0.0, 0.0}};
    const double* bsrc = img + li * kSmLd + q;               // B: sample 4 kk + q of column li
    const double* asrc = ga + q * kGaLd + li;  // A: G[16 t + li][4 kk + q] = ga[4 kk + q][16 t + li]
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const double b = SOSM_B(kk);
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = mfma_f64x4(asrc[4 * kk * kGaLd + 16 * t], b, acc[t]);
    }
    // block 0 of a row: its true end state M zi u_0 + E (u_0: the column's sample 0, in the image)
    int r, k;
    sosm_col(tl, li, G.nb, r, k);
    const double u0 = (k == 0 && r < nr) ? img[li * kSmLd] : 0.0;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) acc[t][rr] += u0 * mzi[t][rr];
    wave_barrier_lds();
    sosm_states_out<NST>(img, lane, acc);
    wave_barrier_lds();
    // 16 x NST states, element v = column * NST + m; only full blocks (k < nb - 1) keep an end state
    if (tl.one_row && tl.k0 + 16 <= G.nb - 1) {  // one contiguous run of Sf
      double* sp = Sf + ((int64_t)tl.r0 * G.nb + tl.k0) * NST;
#pragma unroll
      for (int u = 0; u < (16 * NST + 63) / 64; ++u) {
        const int v = lane + 64 * u;
        if (v < 16 * NST) sp[v] = img[sosm_sv<NST>(v)];
      }
    } else {
#pragma unroll
      for (int u = 0; u < (16 * NST + 63) / 64; ++u) {
        const int v = lane + 64 * u;
        if (v < 16 * NST) {
          int rc, kc;
          sosm_col(tl, v / NST, G.nb, rc, kc);
          if (rc < nr && kc < G.nb - 1) Sf[((int64_t)rc * G.nb + kc) * NST + v % NST] = img[sosm_sv<NST>(v)];
        }
      }
    }
  }
}

// Forward phase C + backward phase A: y = T u + Hm s (s: the true start state, zi u_0 for block 0), then
// E_b = Gb y from the accumulators, stored at the backward block index nb - 1 - k (full blocks only).
template <typename T, int NS>
__global__ __launch_bounds__(256) void sosm_fc_kernel(const T* __restrict__ x, SosGeom G, const double* __restrict__ mats,
                                                      const double* __restrict__ zi, const double* __restrict__ Sf,
                                                      double* __restrict__ y, double* __restrict__ Sb) {
  constexpr int NST = 2 * NS, KS = (NST + 3) / 4;
  __shared__ double hq[4 * kHq], hm[kSmL * kHmLd], gb[kSmRows * kGbLd], imgs[4][16 * kSmLd];
  sosm_tables<NS>(mats, hq, nullptr, hm, nullptr, gb);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double* img = imgs[wave];
  const int q = lane >> 4, li = lane & 15;
  const int nr = (int)G.n_rows;
  const int n_tiles = (nr * G.nb + 15) / 16, stride = gridDim.x * 4;
  int tile = blockIdx.x * 4 + wave;
  // the start state of column li, states m = KS q + q' (q' < KS) in this lane: contiguous in Sf (raw loads, block 0's
  // zi u_0 formed at use, u_0 from the image)
  auto load_s = [&](const SosmTile& t, double (&s)[KS]) {
    int r, k;
    sosm_col(t, li, G.nb, r, k);
    const double* sp = Sf + ((int64_t)min(r, nr - 1) * G.nb + max(k - 1, 0)) * NST;
#pragma unroll
    for (int qq = 0; qq < KS; ++qq) s[qq] = sp[min(KS * q + qq, NST - 1)];
  };
  double zim[KS];
#pragma unroll
  for (int qq = 0; qq < KS; ++qq) zim[qq] = KS * q + qq < NST ? zi[KS * q + qq] : 0.0;
  SosmXRaw<T> raw;
  double ns[KS];
  if (tile < n_tiles) {
    const SosmTile t0 = sosm_tile(tile, nr, G.nb);
    sosm_fetch_x(x, G, t0, lane, raw);
    load_s(t0, ns);
  }
  for (; tile < n_tiles; tile += stride) {
    const SosmTile tl = sosm_tile(tile, nr, G.nb);
    {
      double v[16];
      sosm_expand_x(x, G, tl, lane, raw, v);
      wave_barrier_lds();
      sosm_to_lds(img, lane, v);
    }
    double sv[KS];
    {
      int r, k;
      sosm_col(tl, li, G.nb, r, k);
      const bool ok = r < nr;
      wave_barrier_lds();
      const double u0 = img[li * kSmLd];
#pragma unroll
      for (int qq = 0; qq < KS; ++qq) {
        const bool real = ok && KS * q + qq < NST;
        sv[qq] = !real ? 0.0 : (k == 0 ? zim[qq] * u0 : ns[qq]);
      }
    }
    if (tile + stride < n_tiles) {  // the next tile's samples and start states, in flight under this tile's MFMAs
      const SosmTile tn = sosm_tile(tile + stride, nr, G.nb);
      sosm_fetch_x(x, G, tn, lane, raw);
      load_s(tn, ns);
    }
    wave_barrier_lds();
    doublex4_t acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = doublex4_t{0.0, 0.0, 0.0, 0.0};
    const double* bsrc = img + li * kSmLd + q;          // B: sample 4 kk + q of column li
    const double* tsrc = hq + q * kHq + kSmL + li - q;  // A: T[16 t + li][4 kk + q] = hq[q][64 + 16 t + li - 4 kk - q]
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const double b = SOSM_B(kk);
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (kk <= 4 * t + 3) acc[t] = mfma_f64x4(tsrc[16 * t - 4 * kk], b, acc[t]);  // the lower triangle's k-steps
    }
    const double* msrc = hm + li * kHmLd + KS * q;   // A: Hm[16 t + li][KS q + q']
#pragma unroll
    for (int qq = 0; qq < KS; ++qq)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = mfma_f64x4(msrc[16 * t * kHmLd + qq], sv[qq], acc[t]);
    // backward zero-state end state Gb y: y (rows = samples) as the B operand straight from the accumulators
    // (register rr of tile t is k-step 4 t + rr: sample 16 t + 4 rr + q)
    doublex4_t e[2] = {doublex4_t{0.0, 0.0, 0.0, 0.0}, doublex4_t{0.0, 0.0, 0.0, 0.0}};
    const double* gsrc = gb + li * kGbLd + q;        // A: gb[16 t' + li][4 kk + q]
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
#pragma unroll
      for (int t = 0; t < 2; ++t) e[t] = mfma_f64x4(gsrc[16 * t * kGbLd + 4 * kk], acc[kk >> 2][kk & 3], e[t]);
    // y through the image: coalesced row runs
    wave_barrier_lds();
    sosm_acc_to_lds(img, lane, acc);
    wave_barrier_lds();
    const bool full = tl.one_row && tl.k0 + 16 <= G.nb - 1;  // 16 full blocks of one row: plain runs
    if (full) {
      double* yp = y + (int64_t)tl.r0 * G.n_ext + (int64_t)tl.k0 * kSmL + lane;
#pragma unroll
      for (int u = 0; u < 16; ++u) yp[64 * u] = img[u * kSmLd + lane];
    } else {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        int r, k;
        sosm_col(tl, u, G.nb, r, k);
        const int64_t i = (int64_t)k * kSmL + lane;
        if (r < nr && i < G.n_ext) y[(int64_t)r * G.n_ext + i] = img[u * kSmLd + lane];
      }
    }
    // E_b of full blocks at backward index nb - 1 - k
    wave_barrier_lds();
    sosm_states_out<NST>(img, lane, e);
    wave_barrier_lds();
    if (full) {  // column c at backward index nb - 1 - k0 - c: descending runs of NST
      double* sp = Sb + ((int64_t)tl.r0 * G.nb + (G.nb - 1 - tl.k0)) * NST;
#pragma unroll
      for (int u = 0; u < (16 * NST + 63) / 64; ++u) {
        const int v = lane + 64 * u;
        if (v < 16 * NST) sp[v % NST - (v / NST) * NST] = img[sosm_sv<NST>(v)];
      }
    } else {
#pragma unroll
      for (int u = 0; u < (16 * NST + 63) / 64; ++u) {
        const int v = lane + 64 * u;
        if (v < 16 * NST) {
          int rc, kc;
          sosm_col(tl, v / NST, G.nb, rc, kc);
          if (rc < nr && kc < G.nb - 1) Sb[((int64_t)rc * G.nb + (G.nb - 1 - kc)) * NST + v % NST] = img[sosm_sv<NST>(v)];
        }
      }
    }
  }
}

// The first backward block (forward block nb - 1, P = n_ext - (nb - 1) L samples) by the recursion from zi y[-1],
// one lane per row: its outputs (trimmed) and the backward state after it (Sb[r][0]).  The block's samples are loaded
// 16 at a time ahead of the recursion that consumes them.
template <typename T, int NS>
__global__ __launch_bounds__(64) void sosm_bf_kernel(T* __restrict__ x, SosGeom G, const double* __restrict__ sos,
                                                     const double* __restrict__ zi, const double* __restrict__ y,
                                                     double* __restrict__ Sb) {
  constexpr int NST = 2 * NS;
  const int64_t r = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (r >= G.n_rows) return;
  SosCoef<NS> c;
  c.load(sos);
  const double* yr = y + r * G.n_ext;
  const double ul = yr[G.n_ext - 1];
  double z0[NS], z1[NS];
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    z0[q] = zi[2 * q] * ul;
    z1[q] = zi[2 * q + 1] * ul;
  }
  const int64_t start = (int64_t)(G.nb - 1) * kSmL;
  double cur[16];
  for (int64_t i0 = G.n_ext - 1; i0 >= start; i0 -= 16) {
#pragma unroll
    for (int t = 0; t < 16; ++t) cur[t] = i0 - t >= start ? yr[i0 - t] : 0.0;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int64_t i = i0 - t;
      if (i >= start) {
        const double v = c.step(z0, z1, cur[t]);
        const int64_t j = i - G.padlen;
        if (j >= 0 && j < G.n_t) x[r * G.row_stride + j] = (T)v;
      }
    }
  }
  double* sb = Sb + r * G.nb * NST;
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    sb[2 * q] = z0[q];
    sb[2 * q + 1] = z1[q];
  }
}

// Backward phase C for backward blocks k' >= 1 (forward blocks k = nb - 1 - k' < nb - 1, columns (r, k) of an
// [n_rows][nb - 1] grid): v = U y + Hrev s with s the true backward state before the block, trimmed into the row.
template <typename T, int NS>
__global__ __launch_bounds__(256, kSmOcc) void sosm_bc_kernel(T* __restrict__ x, SosGeom G, const double* __restrict__ mats,
                                                      const double* __restrict__ y, const double* __restrict__ Sb) {
  constexpr int NST = 2 * NS, KS = (NST + 3) / 4;
  __shared__ double hr[4 * kHq], hm[kSmL * kHmLd], imgs[4][16 * kSmLd];
  sosm_tables<NS>(mats, nullptr, hr, hm, nullptr, nullptr);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double* img = imgs[wave];
  const int q = lane >> 4, li = lane & 15;
  const int nr = (int)G.n_rows, nc = G.nb - 1;
  const int n_tiles = (nr * nc + 15) / 16, stride = gridDim.x * 4;
  int tile = blockIdx.x * 4 + wave;
  auto load_s = [&](const SosmTile& t, double (&s)[KS]) {  // backward state before block k: Sb[r][nb - 2 - k]
    int r, k;
    sosm_col(t, li, nc, r, k);
    const bool ok = r < nr;
    const double* sp = Sb + ((int64_t)r * G.nb + (G.nb - 2 - k)) * NST;
#pragma unroll
    for (int qq = 0; qq < KS; ++qq) {
      const int m = KS * q + qq;
      s[qq] = (ok && m < NST) ? sp[m] : 0.0;
    }
  };
  double ny[16], ns[KS];
  if (tile < n_tiles) {
    const SosmTile t0 = sosm_tile(tile, nr, nc);
    sosm_load_y(y, G, t0, lane, ny);
    load_s(t0, ns);
  }
  for (; tile < n_tiles; tile += stride) {
    const SosmTile tl = sosm_tile(tile, nr, nc);
    double sv[KS];
#pragma unroll
    for (int qq = 0; qq < KS; ++qq) sv[qq] = ns[qq];
    wave_barrier_lds();
    sosm_to_lds(img, lane, ny);
    if (tile + stride < n_tiles) {
      const SosmTile tn = sosm_tile(tile + stride, nr, nc);
      sosm_load_y(y, G, tn, lane, ny);
      load_s(tn, ns);
    }
    wave_barrier_lds();
    doublex4_t acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = doublex4_t{0.0, 0.0, 0.0, 0.0};
    const double* bsrc = img + li * kSmLd + q;          // B: sample 4 kk + q of column li
    const double* usrc = hr + q * kHq + kSmL + li - q;  // A: U[16 t + li][4 kk + q] = hr[q][64 + 16 t + li - 4 kk - q]
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const double b = SOSM_B(kk);
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (kk >= 4 * t) acc[t] = mfma_f64x4(usrc[16 * t - 4 * kk], b, acc[t]);  // the upper triangle's k-steps
    }
    const double* msrc = hm + (kSmL - 1 - li) * kHmLd + KS * q;  // A: Hm[L - 1 - (16 t + li)][KS q + q']
#pragma unroll
    for (int qq = 0; qq < KS; ++qq)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = mfma_f64x4(msrc[-16 * t * kHmLd + qq], sv[qq], acc[t]);
    wave_barrier_lds();
    sosm_acc_to_lds(img, lane, acc);
    wave_barrier_lds();
    // v at ext index k L + i -> x[j = k L + i - padlen] when 0 <= j < n_t
    const int64_t j0 = (int64_t)tl.k0 * kSmL - G.padlen;
    if (tl.one_row && j0 >= 0 && j0 + 16 * kSmL <= G.n_t) {  // one contiguous run of x
      T* xp = x + (int64_t)tl.r0 * G.row_stride + j0 + lane;
#pragma unroll
      for (int u = 0; u < 16; ++u) xp[64 * u] = (T)img[u * kSmLd + lane];
    } else {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        int r, k;
        sosm_col(tl, u, nc, r, k);
        const int64_t j = (int64_t)k * kSmL + lane - G.padlen;
        if (r < nr && j >= 0 && j < G.n_t) x[(int64_t)r * G.row_stride + j] = (T)img[u * kSmLd + lane];
      }
    }
  }
}
#undef SOSM_B

// The state scan S[k] = S[k] + M S[k - 1], k = 1 .. K - 1 (K = nb - 1 end states; S[0] already true; S[k] holds
// the zero-state end state E[k] on entry), two-level: one 256-thread block per row, 8 half-waves (lane j = state
// component j; every row's block resident at once on a 1 024-row record).  The steps are cut into NG <= 8 groups of Q
// (q covers k in [1 + q Q, 1 + (q + 1) Q)):
//   1  every group runs the scan from a zero start (group 0 from S[0]): Z[k] = E[k] + M Z[k - 1] (into S[k]);
//   2  the carries, in order: C_q = Z[last of q] + M^Q C_{q - 1} (C_0 = Z[last of 0], already true);
//   3  every group q >= 1 adds the carried part: D = M D from D = C_{q - 1}, S[k] = Z[k] + D.
// 2 Q + NG dependent steps instead of K - 1 (record of 1 024 x 60 s: 68 instead of 235; 16 half-waves per row gave 46
// steps but two rounds of blocks).  A step is one LDS round trip: the state and the step's own operand come from the
// LDS in one batch of reads (the 16 steps' operands of a batch are staged there from HBM at once), its result goes
// to the LDS slot and to HBM by stores nothing waits for.  (Operands held in registers instead left room for two
// reads in flight: five round trips per step, 43 us per scan.)
constexpr int kScanHW = 8, kScanPF = 16;
__host__ __device__ constexpr int sosm_scan_q(int nb) { return nb > 2 ? (nb - 2 + kScanHW - 1) / kScanHW : 1; }
// the 16-group scan on the matrix pipe (sosm_scanm_kernel): its group length, at most kScanMQ steps
constexpr int kScanMG = 16, kScanMQ = 16;
__host__ __device__ constexpr int sosm_scan_q16(int nb) { return nb > 2 ? (nb - 2 + kScanMG - 1) / kScanMG : 1; }

template <int NS>
__global__ __launch_bounds__(32 * kScanHW, 4) void sosm_scan_kernel(SosGeom G, const double* __restrict__ mats, int32_t Q,
                                                        double* __restrict__ S) {
  using O = SosmMats<NS>;
  constexpr int NST = 2 * NS;
  __shared__ __attribute__((aligned(16))) double sv[kScanHW][32];
  __shared__ double zb[kScanHW][kScanPF][NST];  // the batch's operands, then its results
  __shared__ double carry[kScanHW][NST], zlast[kScanHW][NST];
  const int hw = threadIdx.x >> 5, j = threadIdx.x & 31;
  const bool act = j < NST;
  const int jc = act ? j : 0;
  double* Sr = S + (int64_t)blockIdx.x * G.nb * NST;
  const int K = G.nb - 1;
  const int k0 = 1 + hw * Q, k1 = min(1 + (hw + 1) * Q, K);  // this half-wave's group [k0, k1)
  const int ng = K > 1 ? (K - 1 + Q - 1) / Q : 0;              // non-empty groups
  // add + sum_i A[i] x_i (row j of the matrix), x from the LDS slot: every read of the step issued together
  auto matvec = [&](const double* A, double add) {
    wave_barrier_lds();
    const double2* v2 = reinterpret_cast<const double2*>(sv[hw]);
    double2 u[NST / 2];
#pragma unroll
    for (int i = 0; i < NST / 2; ++i) u[i] = v2[i];
    double pa[4] = {add, 0.0, 0.0, 0.0};
#pragma unroll
    for (int i = 0; i < NST / 2; ++i) {
      pa[(2 * i) & 3] += A[2 * i] * u[i].x;
      pa[(2 * i + 1) & 3] += A[2 * i + 1] * u[i].y;
    }
    return (pa[0] + pa[1]) + (pa[2] + pa[3]);
  };
  auto put = [&](double v) {
    wave_barrier_lds();
    sv[hw][j] = v;
  };
  double m[NST];
#pragma unroll
  for (int i = 0; i < NST; ++i) {
    const double v = mats[O::M + jc * NST + i];
    m[i] = act ? v : 0.0;
  }
  // rows kb .. kb + 15 of this group into zb[hw] (zeros past the group; loads unconditional, clamped, so that the
  // compiler issues them together instead of one under each lane test)
  auto stage = [&](int kb) {
    double v[kScanPF];
#pragma unroll
    for (int t = 0; t < kScanPF; ++t) v[t] = Sr[(int64_t)min(kb + t, K - 1) * NST + jc];
#pragma unroll
    for (int t = 0; t < kScanPF; ++t)
      if (act) zb[hw][t][j] = kb + t < k1 ? v[t] : 0.0;
  };
  // level 1: zero-start scans of the groups (group 0 from the true S[0]); every half-wave runs Q steps rounded up to
  // whole batches (steps past the group compute on zeros or run on past its end, and store nothing)
  {
    const double s0 = Sr[jc];
    put((hw == 0 && act) ? s0 : 0.0);
  }
  double zl = 0.0;
  for (int kb = k0; kb < k0 + Q; kb += kScanPF) {
    stage(kb);
#pragma unroll
    for (int t = 0; t < kScanPF; ++t) {
      const double z = matvec(m, act ? zb[hw][t][j] : 0.0);
      zl = kb + t == k1 - 1 ? z : zl;  // the group's last Z, for the carries
      put(z);
      if (act) zb[hw][t][j] = z;
      if (act && kb + t < k1) Sr[(int64_t)(kb + t) * NST + j] = z;
    }
  }
  if (act) zlast[hw][j] = zl;
  __syncthreads();
  // level 2: carries by one half-wave (M^Q rows from HBM: six steps)
  if (hw == 0) {
    double mq[NST];
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const double v = sosm_mq<NS>(mats, false, Q, jc * NST + i);
      mq[i] = act ? v : 0.0;
    }
    double c = act ? zlast[0][j] : 0.0;
    if (act) carry[0][j] = c;
    for (int g = 1; g + 1 < ng; ++g) {
      put(c);
      c = matvec(mq, act ? zlast[g][j] : 0.0);
      if (act) carry[g][j] = c;
    }
  }
  __syncthreads();
  // level 3: the carried part of groups q >= 1 (Z from the LDS when the group fits one batch, else from HBM again)
  if (hw >= 1 && hw < ng) {
    double d = act ? carry[hw - 1][j] : 0.0;
    for (int kb = k0; kb < k1; kb += kScanPF) {
      if (Q > kScanPF) stage(kb);
#pragma unroll
      for (int t = 0; t < kScanPF; ++t) {
        put(d);
        d = matvec(m, 0.0);
        if (act && kb + t < k1) Sr[(int64_t)(kb + t) * NST + j] = zb[hw][t][j] + d;
      }
    }
  }
}

// The same scan with the row's states resident in the LDS (records of up to kScanCap / NST end states: 240 blocks of
// 64 samples at NS = 10, 61 s at 250 Hz): the row's E[0 .. K) come in by one coalesced batch of 16-byte loads, level 1
// turns them into Z in place, level 3 stores S = Z + D straight from there.  HBM sees each state read once and written
// once (the staged kernel above reads E, writes Z, reads Z again and writes S: twice the bytes, in bursts that no
// step overlaps).
constexpr int kScanCap = 4800;  // doubles: 37.5 KB, with the carries and the broadcast slots 40 KB (4 rows per CU)
template <int NS>
__global__ __launch_bounds__(32 * kScanHW, 4) void sosm_scanr_kernel(SosGeom G, const double* __restrict__ mats,
                                                                    int32_t Q, double* __restrict__ S) {
  using O = SosmMats<NS>;
  constexpr int NST = 2 * NS;
  __shared__ __attribute__((aligned(16))) double zf[kScanCap];
  __shared__ __attribute__((aligned(16))) double sv[kScanHW][NST + (NST & 1)];
  __shared__ double carry[kScanHW][NST];
  const int hw = threadIdx.x >> 5, j = threadIdx.x & 31;
  const bool act = j < NST;
  const int jc = act ? j : 0;
  double* Sr = S + (int64_t)blockIdx.x * G.nb * NST;
  const int K = G.nb - 1;
  const int k0 = 1 + hw * Q, k1 = min(1 + (hw + 1) * Q, K);  // this half-wave's group [k0, k1)
  const int ng = K > 1 ? (K - 1 + Q - 1) / Q : 0;              // non-empty groups
  double m[NST];
#pragma unroll
  for (int i = 0; i < NST; ++i) {
    const double v = mats[O::M + jc * NST + i];
    m[i] = act ? v : 0.0;
  }
  // E[0 .. K) -> zf: K NST doubles by LDS-DMA (16 bytes per lane, no registers: M stays in them)
  {
    const int n16 = K * NST / 2;  // NST even
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int c = 0; c * 32 * kScanHW < n16; ++c) {
      const int e0 = c * 32 * kScanHW + w * 64, e = e0 + lane;
      if (e < n16)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(Sr + 2 * e),
                                         (__attribute__((address_space(3))) void*)(zf + 2 * e0), 16, 0, 0);
    }
  }
  __syncthreads();
  // add + sum_i A[i] x_i, x = the NST doubles at xs (LDS, broadcast): every read of the step issued together
  auto matvec = [&](const double* A, const double* xs, double add) {
    const double2* v2 = reinterpret_cast<const double2*>(xs);
    double2 u[NST / 2];
#pragma unroll
    for (int i = 0; i < NST / 2; ++i) u[i] = v2[i];
    double pa[4] = {add, 0.0, 0.0, 0.0};
#pragma unroll
    for (int i = 0; i < NST / 2; ++i) {
      pa[(2 * i) & 3] += A[2 * i] * u[i].x;
      pa[(2 * i + 1) & 3] += A[2 * i + 1] * u[i].y;
    }
    return (pa[0] + pa[1]) + (pa[2] + pa[3]);
  };
  // level 1: Z[k] = E[k] + M Z[k - 1] in place (group 0 from the true S[0]; the others from zero: their first step
  // takes E alone, the product with the neighbouring group's row discarded)
#pragma unroll 1
  for (int k = k0; k < k1; ++k) {
    wave_barrier_lds();
    const double z = matvec(m, zf + (k - 1) * NST, zf[k * NST + jc]);
    const double e = zf[k * NST + jc];
    wave_barrier_lds();
    if (act) zf[k * NST + j] = (k == k0 && hw > 0) ? e : z;
  }
  __syncthreads();
  // level 2: the carries C_g (true state at the end of group g), in order, by one half-wave
  if (hw == 0) {
    double mq[NST];
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const double v = sosm_mq<NS>(mats, false, Q, jc * NST + i);
      mq[i] = act ? v : 0.0;
    }
    double c = act ? zf[(min(1 + Q, K) - 1) * NST + j] : 0.0;
    if (act) carry[0][j] = c;
#pragma unroll 1
    for (int g = 1; g + 1 < ng; ++g) {
      if (act) sv[0][j] = c;
      wave_barrier_lds();
      c = matvec(mq, sv[0], act ? zf[(min(1 + (g + 1) * Q, K) - 1) * NST + j] : 0.0);
      wave_barrier_lds();
      if (act) carry[g][j] = c;
    }
  }
  __syncthreads();
  // level 3: S[k] = Z[k] + M^(k - k0 + 1) C_(q - 1) for groups q >= 1, S[k] = Z[k] for group 0, stored to HBM (M
  // again from memory, L2-resident: holding it over level 2 beside M^Q would spill; the pointer is laundered so that
  // the compiler does not reuse the first loads' registers instead)
  const double* mats3 = mats;
  asm volatile("" : "+s"(mats3));
#pragma unroll
  for (int i = 0; i < NST; ++i) {
    const double v = mats3[O::M + jc * NST + i];
    m[i] = act ? v : 0.0;
  }
  double d = (hw >= 1 && hw < ng && act) ? carry[hw - 1][j] : 0.0;
#pragma unroll 1
  for (int k = k0; k < k1; ++k) {
    if (hw >= 1) {
      if (act) sv[hw][j] = d;
      wave_barrier_lds();
      d = matvec(m, sv[hw], 0.0);
      wave_barrier_lds();
    }
    if (act) Sr[(int64_t)k * NST + j] = zf[k * NST + j] + d;
  }
}

// The same scan on the float64 matrix pipe, one wave per row: its 16 groups of Q16 <= 16 blocks are the 16 columns
// of v_mfma_f64_16x16x4_f64 GEMMs, so a step of all 16 groups is M [NST x NST] times their states [NST x 16]: 2 row
// tiles x KS k-steps.  Lane l holds fragment kk of column c = l & 15, state row 4 kk + (l >> 4), which is at once the
// step's accumulator (tile kk / 4, register kk % 4) and the next step's B operand (k-step kk): the recurrence never
// leaves the registers (the LDS broadcast of the VALU scans was their bound).  Level 1 keeps every group's Z in
// registers (Q16 x KS doubles per lane), level 2 (the carries through M^Q16) runs on lanes 0 .. NST - 1 through the
// LDS, level 3 adds M^(s + 1) C to the registers' Z and stores S as it goes.  E is read once (all loads of a lane
// issued together at the start), S written once.  (Staging E and S through the LDS for whole-line transfers measured
// slower, 31.5 against 28.1 us: the stores no longer overlap the steps.)
template <int NS>
__global__ __launch_bounds__(64, 1) void sosm_scanm_kernel(SosGeom G, const double* __restrict__ mats, int32_t Q,
                                                          double* __restrict__ S) {
  using O = SosmMats<NS>;
  constexpr int NST = 2 * NS, KS = (NST + 3) / 4, TT = (NST + 15) / 16;
  __shared__ __attribute__((aligned(16))) double zl[kScanMG][NST + (NST & 1)];
  __shared__ __attribute__((aligned(16))) double carry[kScanMG][NST + (NST & 1)];
  __shared__ __attribute__((aligned(16))) double slot[NST + (NST & 1)];
  const int l = threadIdx.x, c = l & 15, q4 = l >> 4;
  double* Sr = S + (int64_t)blockIdx.x * G.nb * NST;
  const int K = G.nb - 1;
  const int k0 = 1 + c * Q, k1 = min(1 + (c + 1) * Q, K);  // group c = [k0, k1)
  const int len = max(k1 - k0, 0);
  const int ng = K > 1 ? (K - 1 + Q - 1) / Q : 0;
  // A operands: M[16 t + c][4 kk + q4] (zero outside NST x NST)
  double a[TT][KS];
#pragma unroll
  for (int t = 0; t < TT; ++t)
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int r = 16 * t + c, k = 4 * kk + q4;
      const double v = mats[O::M + min(r, NST - 1) * NST + min(k, NST - 1)];
      a[t][kk] = (r < NST && k < NST) ? v : 0.0;
    }
  // E of every step of the group, fragment kk = row 4 kk + q4 (rows past NST and steps past the group: any finite
  // value of the row, never used)
  double z[kScanMQ][KS];
#pragma unroll
  for (int st = 0; st < kScanMQ; ++st)
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int k = min(k0 + st, K - 1), r = min(4 * kk + q4, NST - 1);
      z[st][kk] = Sr[(int64_t)k * NST + r];
    }
  double b[KS];  // the state entering the step (B operand): S[0] for group 0, zero for the others
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    const double v = Sr[min(4 * kk + q4, NST - 1)];
    b[kk] = (c == 0 && 4 * kk + q4 < NST) ? v : 0.0;
  }
  auto step = [&](double (&v)[KS], const double* cin) {  // v = cin + M b (cin: KS fragments, or zero), b = v
    doublex4_t acc[TT];
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) acc[t][rr] = (cin && 4 * t + rr < KS) ? cin[4 * t + rr] : 0.0;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
#pragma unroll
      for (int t = 0; t < TT; ++t) acc[t] = mfma_f64x4(a[t][kk], b[kk], acc[t]);
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      v[kk] = acc[kk >> 2][kk & 3];
      b[kk] = v[kk];
    }
  };
  // level 1: Z in place of E
#pragma unroll
  for (int st = 0; st < kScanMQ; ++st)
    if (st < Q) step(z[st], z[st]);
  // the groups' last Z -> LDS
#pragma unroll
  for (int st = 0; st < kScanMQ; ++st)
    if (st == len - 1)
#pragma unroll
      for (int kk = 0; kk < KS; ++kk)
        if (4 * kk + q4 < NST) zl[c][4 * kk + q4] = z[st][kk];
  __syncthreads();
  // level 2: C_0 = Z_last(0), C_g = Z_last(g) + M^Q16 C_(g - 1), lanes j < NST
  if (l < NST) {
    double mq[NST];
#pragma unroll
    for (int i = 0; i < NST; ++i) mq[i] = sosm_mq<NS>(mats, true, Q, l * NST + i);
    double cv = zl[0][l];
    carry[0][l] = cv;
    for (int g = 1; g + 1 < ng; ++g) {
      slot[l] = cv;
      wave_barrier_lds();
      double acc = zl[g][l];
#pragma unroll
      for (int i = 0; i < NST; ++i) acc += mq[i] * slot[i];
      wave_barrier_lds();
      cv = acc;
      carry[g][l] = cv;
    }
  }
  __syncthreads();
  // level 3: D = M^(s + 1) C_(c - 1) (zero for group 0), S = Z + D
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    const int r = 4 * kk + q4;
    const double v = carry[c > 0 ? c - 1 : 0][min(r, NST - 1)];
    b[kk] = (c > 0 && c < ng && r < NST) ? v : 0.0;
  }
#pragma unroll
  for (int st = 0; st < kScanMQ; ++st) {
    if (st < Q) {
      double d[KS];
      step(d, nullptr);
      if (st < len)
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
          if (4 * kk + q4 < NST) Sr[(int64_t)(k0 + st) * NST + 4 * kk + q4] = z[st][kk] + d[kk];
    }
  }
}

template <int NS>
static void sosm_scan(const SosGeom& G, const double* plan, int Q, double* S, hipStream_t st) {
  if (G.nb <= 2) return;
  if (sosm_scan_q16(G.nb) <= kScanMQ)  // the matrix-pipe scan where its 16 groups of <= 16 blocks cover the row
    hipLaunchKernelGGL(sosm_scanm_kernel<NS>, dim3((unsigned)G.n_rows), dim3(64), 0, st, G, plan,
                       (int32_t)sosm_scan_q16(G.nb), S);
  else if ((int64_t)(G.nb - 1) * 2 * NS <= kScanCap)
    hipLaunchKernelGGL(sosm_scanr_kernel<NS>, dim3((unsigned)G.n_rows), dim3(32 * kScanHW), 0, st, G, plan, Q, S);
  else
    hipLaunchKernelGGL(sosm_scan_kernel<NS>, dim3((unsigned)G.n_rows), dim3(32 * kScanHW), 0, st, G, plan, Q, S);
}

static SosGeom sosm_geom(int64_t n_rows, int64_t row_stride, int32_t n_t, int32_t padlen) {
  SosGeom G;
  G.n_rows = n_rows;
  G.row_stride = row_stride;
  G.n_t = n_t;
  G.padlen = padlen;
  G.n_ext = (int64_t)n_t + 2 * padlen;
  G.L = kSmL;
  G.nb = (int32_t)((G.n_ext + kSmL - 1) / kSmL);
  return G;
}

// workspace of the MFMA path: y [n_rows][n_ext] + Sf, Sb [n_rows][nb][2 n_sec] + the plan (operator table), doubles
static int64_t sosm_workspace_doubles(const SosGeom& G, int n_sec) {
  const int64_t nst = 2 * n_sec;
  return ((G.n_rows * G.n_ext + 1) & ~1LL) + 2 * G.n_rows * G.nb * nst + sosm_plan_doubles(n_sec);  // Sf 16-byte aligned
}
// the MFMA path's column indices are 32-bit
static bool sosm_fits(const SosGeom& G) { return G.n_rows * (int64_t)G.nb < (1LL << 31) - 16; }

template <int NS>
static void sosm_plan(const double* sos, const double* zi, const SosGeom& G, double* plan, hipStream_t st) {
  hipLaunchKernelGGL(sosm_mats_kernel<NS>, dim3(1), dim3(512), 0, st, sos, zi, (int32_t)sosm_scan_q(G.nb),
                     (int32_t)sosm_scan_q16(G.nb), plan);
}

template <typename T, int NS>
static int sosm_run(T* x, const SosGeom& G, const double* sos, const double* zi, const double* plan, double* work,
                    hipStream_t st) {
  constexpr int NST = 2 * NS;
  double* y = work;
  double* Sf = y + ((G.n_rows * G.n_ext + 1) & ~1LL);  // 16-byte aligned (the scans' 16-byte loads)
  double* Sb = Sf + G.n_rows * G.nb * NST;
  const int Q = sosm_scan_q(G.nb);
  // persistent grids: the blocks that are resident at once (LDS and registers), each wave looping over tiles, so
  // that every block forms its operator tables once for many tiles
  const int64_t tiles = (G.n_rows * G.nb + 15) / 16;
  static unsigned res_fa = 0, res_fc = 0, res_bc = 0;
  auto resident = [](unsigned& cache, const void* fn) {
    if (!cache) {
      int n = 0, dev = 0, cus = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 256, 0) != hipSuccess || n <= 0) n = 1;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          cus <= 0)
        cus = 256;
      cache = (unsigned)(n * cus);
    }
    return cache;
  };
  auto grid_of = [](int64_t tiles_, unsigned res) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((tiles_ + 3) / 4, res)); };
  const unsigned gfa = grid_of(tiles, resident(res_fa, (const void*)sosm_fa_kernel<T, NS>));
  const unsigned gfc = grid_of(tiles, resident(res_fc, (const void*)sosm_fc_kernel<T, NS>));
  if (G.nb > 1) hipLaunchKernelGGL((sosm_fa_kernel<T, NS>), dim3(gfa), dim3(256), 0, st, (const T*)x, G, plan, Sf);
  sosm_scan<NS>(G, plan, Q, Sf, st);
  hipLaunchKernelGGL((sosm_fc_kernel<T, NS>), dim3(gfc), dim3(256), 0, st, (const T*)x, G, plan, zi,
                     (const double*)Sf, y, Sb);
  hipLaunchKernelGGL((sosm_bf_kernel<T, NS>), dim3((unsigned)((G.n_rows + 63) / 64)), dim3(64), 0, st, x, G, sos, zi,
                     (const double*)y, Sb);
  if (G.nb > 1) {
    sosm_scan<NS>(G, plan, Q, Sb, st);
    const int64_t tb = (G.n_rows * (G.nb - 1) + 15) / 16;
    const unsigned gbc = grid_of(tb, resident(res_bc, (const void*)sosm_bc_kernel<T, NS>));
    hipLaunchKernelGGL((sosm_bc_kernel<T, NS>), dim3(gbc), dim3(256), 0, st, x, G, plan, (const double*)y,
                       (const double*)Sb);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_error(-3, hipGetErrorString(e));
}

// plan == nullptr: formed into the workspace's tail first (dvh_sosfiltfilt); else the caller's (dvh_sosfiltfilt_planned)
template <typename T, int NS>
static int sosfiltfilt_mfma(T* x, const SosGeom& G, const double* sos, const double* zi, const double* plan, double* work,
                            hipStream_t st) {
  if (!plan) {
    double* p = work + ((G.n_rows * G.n_ext + 1) & ~1LL) + 2 * G.n_rows * G.nb * (2 * NS);
    sosm_plan<NS>(sos, zi, G, p, st);
    plan = p;
  }
  return sosm_run<T, NS>(x, G, sos, zi, plan, work, st);
}

// block length: enough (row, block) lanes for ~4 waves per SIMD, blocks of 32 .. 4096 samples
static int sos_block_len(int64_t n_rows, int64_t n_ext) {
  const int64_t target = 256LL * 4 * 4 * 64;
  int64_t L = (n_rows * n_ext + target - 1) / target;
  L = (L + 31) / 32 * 32;
  return (int)std::min<int64_t>(std::max<int64_t>(L, 32), 4096);
}

static SosGeom sos_geom(int64_t n_rows, int64_t row_stride, int32_t n_t, int32_t padlen) {
  SosGeom G;
  G.n_rows = n_rows;
  G.row_stride = row_stride;
  G.n_t = n_t;
  G.padlen = padlen;
  G.n_ext = (int64_t)n_t + 2 * padlen;
  G.L = sos_block_len(n_rows, G.n_ext);
  G.nb = (int32_t)((G.n_ext + G.L - 1) / G.L);
  return G;
}

// workspace: y [n_rows][n_ext] + S [n_rows][nb][2 n_sec] + M [2 n_sec]^2, doubles
static int64_t sos_workspace_doubles(const SosGeom& G, int n_sec) {
  const int64_t nst = 2 * n_sec;
  return G.n_rows * G.n_ext + G.n_rows * G.nb * nst + nst * nst;
}

template <typename T, int NS>
static int sosfiltfilt_blocks(T* x, const SosGeom& G, const double* sos, const double* zi, double* work,
                              hipStream_t st) {
  constexpr int NST = 2 * NS;
  double* y = work;
  double* S = y + G.n_rows * G.n_ext;
  double* M = S + G.n_rows * G.nb * NST;
  const int64_t lanes = G.n_rows * G.nb;
  const dim3 grid((unsigned)((lanes + 63) / 64)), scan_grid((unsigned)((G.n_rows + 1) / 2));
  hipLaunchKernelGGL(sos_transition_kernel<NS>, dim3(1), dim3(64), 0, st, sos, G.L, M);
  // forward pass over the odd extension -> y
  hipLaunchKernelGGL((sos_block_kernel<T, NS, false, false>), grid, dim3(64), 0, st, x, y, G, sos, zi, S);
  if (G.nb > 2) hipLaunchKernelGGL(sos_scan_kernel<NS>, scan_grid, dim3(64), 0, st, G, (const double*)M, S);
  hipLaunchKernelGGL((sos_block_kernel<T, NS, false, true>), grid, dim3(64), 0, st, x, y, G, sos, zi, S);
  // backward pass over reversed y -> the trimmed row
  hipLaunchKernelGGL((sos_block_kernel<T, NS, true, false>), grid, dim3(64), 0, st, x, y, G, sos, zi, S);
  if (G.nb > 2) hipLaunchKernelGGL(sos_scan_kernel<NS>, scan_grid, dim3(64), 0, st, G, (const double*)M, S);
  hipLaunchKernelGGL((sos_block_kernel<T, NS, true, true>), grid, dim3(64), 0, st, x, y, G, sos, zi, S);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_error(-3, hipGetErrorString(e));
}

// MFMA path (a plan given and the 32-bit column indices fit) or the VALU block recursion.  The block GEMMs add the
// contributions of states that grow like 1 / (1 - r) for the filter's largest pole radius r, so their rounding grows
// with it: relative error 1e-13 at r = 0.9956 (1.2-30 Hz at 250 Hz), 5e-10 at r = 0.99973 (0.08-1 Hz); callers
// plan the matrix form only for r <= DVH_SOS_MFMA_MAX_POLE (dvh_sos_pole_radius) and take the recursion otherwise.
template <typename T>
static int sosfiltfilt_dispatch(T* x, const SosGeom& Gm, const SosGeom& Gb, const double* sos, int n_sec, const double* zi,
                                const double* plan, double* work, hipStream_t st) {
  const bool mf = plan && sosm_fits(Gm);
  switch (n_sec) {
#define DVH_SOS_CASE(n) \
  case n: return mf ? sosfiltfilt_mfma<T, n>(x, Gm, sos, zi, plan, work, st) : sosfiltfilt_blocks<T, n>(x, Gb, sos, zi, work, st);
    DVH_SOS_CASE(1) DVH_SOS_CASE(2) DVH_SOS_CASE(3) DVH_SOS_CASE(4) DVH_SOS_CASE(5) DVH_SOS_CASE(6)
    DVH_SOS_CASE(7) DVH_SOS_CASE(8) DVH_SOS_CASE(9) DVH_SOS_CASE(10) DVH_SOS_CASE(11) DVH_SOS_CASE(12)
    DVH_SOS_CASE(13) DVH_SOS_CASE(14) DVH_SOS_CASE(15) DVH_SOS_CASE(16)
#undef DVH_SOS_CASE
    default: return set_error(-4, "unsupported number of second-order sections");
  }
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
  // 8 loads in flight per thread (one load per iteration left the block waiting out a memory latency per 256 samples:
  // a one-block impute round took 38 us)
  constexpr int U = 8;
  int t = threadIdx.x;
  for (; t + (U - 1) * kStatBlock < n_t; t += U * kStatBlock) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = row[t + u * kStatBlock];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double d = (double)v[u];
      s += d * d;
      m = nan_max(m, d);
    }
  }
  for (; t < n_t; t += kStatBlock) {
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
  constexpr int U = 8;
  int t = threadIdx.x;
  for (; t + (U - 1) * kStatBlock < n_t; t += U * kStatBlock) {
    T va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      va[u] = a[t + u * kStatBlock];
      vb[u] = b ? b[t + u * kStatBlock] : (T)0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) dst[t + u * kStatBlock] = b ? (T)(va[u] + vb[u]) : va[u];
  }
  for (; t < n_t; t += kStatBlock) dst[t] = b ? (T)(a[t] + b[t]) : a[t];
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

// the same with 16-byte accesses (rows 16-byte aligned): 4 floats or 2 doubles per lane
template <typename T>
__global__ __launch_bounds__(256) void row_normalize_vec_kernel(T* __restrict__ x, int64_t row_stride, int32_t n_t,
                                                                const double* __restrict__ stats) {
  constexpr int V = 16 / sizeof(T);
  using Vec = typename std::conditional<sizeof(T) == 4, float4, double2>::type;
  const int64_t r = blockIdx.y;
  const double nrm = sqrt(stats[2 * r]);
  T* row = x + r * row_stride;
  const int nv = n_t / V;
  Vec* rv = reinterpret_cast<Vec*>(row);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += gridDim.x * blockDim.x) {
    Vec v = rv[i];
    T* e = reinterpret_cast<T*>(&v);
#pragma unroll
    for (int k = 0; k < V; ++k) e[k] = (T)((double)e[k] / nrm);
    rv[i] = v;
  }
  for (int t = nv * V + blockIdx.x * blockDim.x + threadIdx.x; t < n_t; t += gridDim.x * blockDim.x)
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
  if (flags & 4) {
    constexpr int V = 16 / sizeof(T);
    if (reinterpret_cast<uintptr_t>(x) % 16 == 0 && row_stride % V == 0)
      hipLaunchKernelGGL(row_normalize_vec_kernel<T>, dim3((unsigned)((n_t / V + 255) / 256 + 1), (unsigned)n_rows),
                         dim3(256), 0, s, x, row_stride, n_t, stats);
    else
      hipLaunchKernelGGL(row_normalize_kernel<T>, dim3((unsigned)((n_t + 255) / 256), (unsigned)n_rows), dim3(256), 0,
                         s, x, row_stride, n_t, stats);
  }
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

DVH_API int64_t dvh_sosfiltfilt_workspace(int64_t n_rows, int32_t n_t, int32_t n_sec, int32_t padlen) {
  if (n_rows <= 0 || n_t <= 0 || n_sec <= 0 || n_sec > kMaxSec || padlen < 0) return 0;
  return 8 * std::max(sosm_workspace_doubles(sosm_geom(n_rows, n_t, n_t, padlen), n_sec),
                      sos_workspace_doubles(sos_geom(n_rows, n_t, n_t, padlen), n_sec));
}

DVH_API double dvh_sos_pole_radius(const double* sos, int32_t n_sec) {
  if (!sos || n_sec <= 0) return -1.0;
  double r = 0.0;
  for (int s = 0; s < n_sec; ++s) {
    const double a0 = sos[6 * s + 3], a1 = sos[6 * s + 4] / a0, a2 = sos[6 * s + 5] / a0;
    const double disc = a1 * a1 - 4.0 * a2;
    if (disc < 0.0) {
      r = std::max(r, std::sqrt(a2));
    } else {
      const double q = std::sqrt(disc);
      r = std::max(r, std::max(std::fabs(0.5 * (-a1 + q)), std::fabs(0.5 * (-a1 - q))));
    }
  }
  return r;
}

DVH_API int64_t dvh_sosfiltfilt_plan_bytes(int32_t n_sec) {
  if (n_sec <= 0 || n_sec > kMaxSec) return 0;
  return 8 * sosm_plan_doubles(n_sec);
}

DVH_API int dvh_sosfiltfilt_plan(const double* sos, int32_t n_sec, const double* zi, int32_t n_t, int32_t padlen,
                                 double* plan, void* stream) {
  if (!sos || !zi || !plan) return set_error(-2, "null pointer argument");
  if (n_sec <= 0 || n_sec > kMaxSec) return set_error(-4, "unsupported number of second-order sections");
  if (padlen < 0 || n_t < 2) return set_error(-2, "invalid padlen / length");
  const SosGeom G = sosm_geom(1, n_t, n_t, padlen);
  switch (n_sec) {
#define DVH_SOS_PLAN(n) \
  case n: sosm_plan<n>(sos, zi, G, plan, (hipStream_t)stream); break;
    DVH_SOS_PLAN(1) DVH_SOS_PLAN(2) DVH_SOS_PLAN(3) DVH_SOS_PLAN(4) DVH_SOS_PLAN(5) DVH_SOS_PLAN(6)
    DVH_SOS_PLAN(7) DVH_SOS_PLAN(8) DVH_SOS_PLAN(9) DVH_SOS_PLAN(10) DVH_SOS_PLAN(11) DVH_SOS_PLAN(12)
    DVH_SOS_PLAN(13) DVH_SOS_PLAN(14) DVH_SOS_PLAN(15) DVH_SOS_PLAN(16)
#undef DVH_SOS_PLAN
    default: break;
  }
  return last_launch();
}

DVH_API int dvh_sosfiltfilt(void* x, int32_t dtype, int64_t n_rows, int64_t row_stride, int32_t n_t,
                            const double* sos, int32_t n_sec, int32_t padlen, const double* zi, double* work,
                            void* stream) {
  if (!x || !sos || !zi || !work) return set_error(-2, "null pointer argument");
  if (reinterpret_cast<uintptr_t>(work) % 16) return set_error(-2, "work must be 16-byte aligned");
  if (n_sec <= 0 || n_sec > kMaxSec) return set_error(-4, "unsupported number of second-order sections");
  if (n_t <= padlen) return set_error(-4, "The length of the input vector x must be greater than padlen");
  if (padlen < 0 || n_t < 2) return set_error(-2, "invalid padlen / length");
  if (n_rows <= 0) return 0;
  const SosGeom Gm = sosm_geom(n_rows, row_stride, n_t, padlen), Gb = sos_geom(n_rows, row_stride, n_t, padlen);
  if (dtype == 0) return sosfiltfilt_dispatch<float>((float*)x, Gm, Gb, sos, n_sec, zi, nullptr, work, (hipStream_t)stream);
  if (dtype == 1) return sosfiltfilt_dispatch<double>((double*)x, Gm, Gb, sos, n_sec, zi, nullptr, work, (hipStream_t)stream);
  return set_error(-2, "dtype must be 0 (float32) or 1 (float64)");
}

DVH_API int dvh_sosfiltfilt_planned(void* x, int32_t dtype, int64_t n_rows, int64_t row_stride, int32_t n_t,
                                    const double* sos, int32_t n_sec, int32_t padlen, const double* zi, const double* plan,
                                    double* work, void* stream) {
  if (!x || !sos || !zi || !work) return set_error(-2, "null pointer argument");  // plan NULL: the recursion
  if (reinterpret_cast<uintptr_t>(work) % 16) return set_error(-2, "work must be 16-byte aligned");
  if (n_sec <= 0 || n_sec > kMaxSec) return set_error(-4, "unsupported number of second-order sections");
  if (n_t <= padlen) return set_error(-4, "The length of the input vector x must be greater than padlen");
  if (padlen < 0 || n_t < 2) return set_error(-2, "invalid padlen / length");
  if (n_rows <= 0) return 0;
  const SosGeom Gm = sosm_geom(n_rows, row_stride, n_t, padlen), Gb = sos_geom(n_rows, row_stride, n_t, padlen);
  if (dtype == 0) return sosfiltfilt_dispatch<float>((float*)x, Gm, Gb, sos, n_sec, zi, plan, work, (hipStream_t)stream);
  if (dtype == 1) return sosfiltfilt_dispatch<double>((double*)x, Gm, Gb, sos, n_sec, zi, plan, work, (hipStream_t)stream);
  return set_error(-2, "dtype must be 0 (float32) or 1 (float64)");
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
