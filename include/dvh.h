/*
 * libdvh — MI355X (gfx950) C-ABI for the vehicle-pass imaging hot path of NohPei/das_diff_veh.
 *
 * The reference is pure Python; its "FFI" for this path is the Python call surface of
 * apis/virtual_shot_gather.py, apis/dispersion_classes.py and modules/utils.py.  Each entry point
 * below replaces the reference function cited next to it; the Python mirror of the reference API in
 * das_diff_veh_amd/ binds them with ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - every pointer is DEVICE memory owned by the caller (e.g. a torch tensor); nothing is
 *     allocated inside;  `stream` is a hipStream_t (NULL = default stream); calls are
 *     stream-ordered, asynchronous and graph-capturable (no host synchronisation inside)
 *   - windows are float32, channel-major: sample (pass p, channel c, time t) is
 *     win[p * pass_stride + c * ch_stride + t]  (strides in elements)
 *   - return 0 on success; negative on error: -2 invalid argument, -3 HIP launch error,
 *     -4 unsupported size; dvh_last_error() describes the calling thread's last error
 */
#ifndef DVH_H
#define DVH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int dvh_abi_version(void);
const char* dvh_last_error(void);

/* Host function: `times` successive random.sample(range(lo, lo + n), k) draws of CPython's `random`
 * (bootstrap_disp's draws, apis/imaging_classes.py:8-48), bit for bit, from the Mersenne Twister state
 * random.getstate()[1] (624 words + index, uint32[625], updated in place for random.setstate()).
 * out: int64 [times][k] (host memory). */
int dvh_random_sample(uint32_t* state, int64_t lo, int64_t n, int32_t k, int32_t times, int64_t* out);

/* Host function: n blocks of nbytes, src[i] -> dst + i * nbytes (host memory, non-temporal stores): the packing
 * of the drop-in classes' NumPy windows (VirtualShotGathersFromWindows, apis/imaging_classes.py:91-126) into a
 * pinned staging buffer before their H2D copy.  Thread-safe; callers split the windows over threads. */
int dvh_host_gather(void* dst, const void* const* src, int64_t nbytes, int32_t n);

/* ---------------------------------------------------------------- virtual shot gathers
 * pass_tab [n_pass][2] = {row0 (= start_idx), pivot_idx};  gather row i is channel row0 + i.
 * seg_tab  [n_pass][R][2 sides][2] = {slice start, slice length} of the row's time slice on the
 *          forward (0) and other (1) side, exactly as the reference slices them
 *          (apis/virtual_shot_gather.py:111-126, 14-43, 152, 172).
 * w = int(wlen / dt), hop = int(w * 0.5) (modules/utils.py:255-256, 292-294).
 * flags: 1 include_other_side, 2 norm (row L2), 4 norm_amp (divide by the pivot row's max).
 */

/* FFT length used for correlation windows of w samples (0 if unsupported). */
int dvh_vsg_fft_length(int32_t w);

/* Per-pass time slices seg_tab[n_pass][R][2][2] derived on the device, float64, with the reference's
 * expressions (preprocessing_window apis/virtual_shot_gather.py:111-126: interp1d extrapolation of
 * the trajectory, pt = argmax(t >= f(pivot) +- delta_t); xcorr_two_traces_based_on_traj :24-35: the
 * per-row t_idx and Python-slice clamping) -- what das_diff_veh_amd.plan.pass_geometry computes on the
 * host, bit for bit.  Inputs per pass p (strides in elements, 0 = shared by every pass):
 *   x_axis[p * x_stride + c] channel positions, t_axis[p * t_stride + t] ascending sample times (n_t),
 *   trajectory trk_x / trk_t[p * trk_stride + k], k < trk_len[p], trk_x strictly ascending,
 *   pivot_x[p] the `pivot` argument, pass_tab[p] = {row0 = start_idx, pivot_idx} (from the spatial
 *   searches, which the host does once per channel axis).
 * flags bit 0: include_other_side.  status[p] = 1 when the trajectory has < 2 points or is not strictly
 * ascending (interp1d would raise / sort); that pass's rows get empty slices. */
int dvh_pass_geometry(const double* x_axis, int64_t x_stride, const double* t_axis, int64_t t_stride, int32_t n_t,
                      const double* trk_x, const double* trk_t, int64_t trk_stride, const int32_t* trk_len,
                      const double* pivot_x, const int32_t* pass_tab, int32_t n_pass, int32_t R, double delta_t,
                      int32_t nsamp, int32_t flags, int32_t* seg_tab, int32_t* status, void* stream);

/* ||window||_F^2 per pass (np.linalg.norm(window.data)**2, apis/virtual_shot_gather.py:125). */
int dvh_window_sumsq(const float* win, int64_t pass_stride, int64_t ch_stride, int32_t n_pass, int32_t n_ch,
                     int32_t n_t, double* out, void* stream);

/* Per-pass, per-side amplitude normalisation: scales[p][side] = 1 / amax(pivot row)
 * (post_processing_XCF, apis/virtual_shot_gather.py:137-138), or 1 / ||window||_F^2 when
 * neither norm nor norm_amp is set (win_sumsq from dvh_window_sumsq; required then, optional
 * otherwise).  When win_sumsq is given, a pass whose window is not finite or all zero gets NaN
 * scales: the reference's data / ||data||_F (:125) makes that whole gather NaN. */
int dvh_vsg_scales(const float* win, int64_t pass_stride, int64_t ch_stride, int32_t n_pass, const int32_t* pass_tab,
                   const int32_t* seg_tab, int32_t R, int32_t w, int32_t hop, int32_t flags, const double* win_sumsq,
                   float* scales, void* stream);

/* Per-pass gathers out[n_pass][R][w]: VirtualShotGather(window, include_other_side, ...).XCF_out
 * (apis/virtual_shot_gather.py:184-192 with construct_shot_gather[_other_side] :145-180,
 * XCORR_vshot / XCORR_two_traces modules/utils.py:253-314). */
int dvh_vsg_gathers(const float* win, int64_t pass_stride, int64_t ch_stride, int32_t n_pass, const int32_t* pass_tab,
                    const int32_t* seg_tab, int32_t R, int32_t w, int32_t hop, int32_t flags, const float* scales,
                    float* out, void* stream);

/* Class stacks, accumulated: stack[slot][R][w] += sum_{p in slot} weight[p] * gather_p.
 * With weight[p] = 1 / count[slot] this is sum(images) / len(images) per class
 * (ImagesFromWindows.get_images, apis/imaging_classes.py:106-107; VirtualShotGather.__add__ /
 * __truediv__ apis/virtual_shot_gather.py:195-210).  order[] lists passes grouped by slot;
 * chunk_tab [n_chunk][3] = {begin, end (into order), slot}.  spec_ws: see dvh_vsg_stack_workspace. */
int dvh_vsg_stack(const float* win, int64_t pass_stride, int64_t ch_stride, int32_t n_pass, const int32_t* pass_tab,
                  const int32_t* seg_tab, int32_t R, int32_t w, int32_t hop, int32_t flags, const float* scales,
                  const int32_t* order, const int32_t* chunk_tab, int32_t n_chunk, const float* weight, float* stack,
                  void* spec_ws, void* stream);

/* dvh_vsg_stack with the windows' validity decided in the same launch.  The reference divides every
 * window by ||data||_F (preprocessing_window, apis/virtual_shot_gather.py:125), so a NaN / inf
 * anywhere in a window [n_ch][n_t], or an all-zero window, makes that pass's gather -- and the mean of
 * its class -- NaN.  This entry reads every sample of every pass's window once, alongside the
 * correlations (at w = 500 the validity scan leaves out the samples the correlations load, which check them
 * themselves), and sets stack[slot] to NaN for each slot (< n_slot) holding such a pass; the
 * scales must then come from dvh_vsg_scales WITHOUT win_sumsq.  Requires flags & (norm | norm_amp):
 * with neither, the scale itself is 1 / ||data||_F^2 (use dvh_window_sumsq).
 * Scan windows: with scan_tab == NULL window p is pass p (win + p * pass_stride, n_ch rows); a unit
 * launch (pass stride 0 over one flattened record, each (pass, pivot) unit a "pass") gives instead
 * n_scan windows of n_ch rows starting at record rows scan_tab[s], and unit_scan[p] = the window
 * whose validity unit p takes (a pass imaged at several pivots is read once).  work: device
 * workspace of (scan_tab ? n_scan : n_pass) + 2 uint32 (per-window max |x| bit pattern, two work
 * counters), zeroed inside. */
int dvh_vsg_stack_validated(const float* win, int64_t pass_stride, int64_t ch_stride, int32_t n_pass, int32_t n_ch,
                            int32_t n_t, const int32_t* pass_tab, const int32_t* seg_tab, int32_t R, int32_t w,
                            int32_t hop, int32_t flags, const float* scales, const int32_t* order,
                            const int32_t* chunk_tab, int32_t n_chunk, int32_t n_slot, const float* weight, float* stack,
                            const int32_t* scan_tab, int32_t n_scan, const int32_t* unit_scan, uint32_t* work,
                            void* spec_ws, void* stream);

/* Bytes of the spec_ws workspace dvh_vsg_stack / dvh_vsg_stack_validated take for n_pass passes at
 * window length w: the spectra of every pass's pivot slices that many rows share (w = 500: the shared
 * windows of both sides and the far rows' clamped windows, 24 KiB + 32 B per pass), which lets the
 * stack launch transform only receivers for those rows (EngF500::spectra_tab).  0 when w does not use
 * it; with spec_ws == NULL the stack entries run the per-sub-window engine instead. */
int64_t dvh_vsg_stack_workspace(int32_t n_pass, int32_t w);

/* ---------------------------------------------------------------- dispersion (map_fv)
 * Gathers data[B][nch][nt] (strides in elements).  Only the FK bins the (f, k = f / v) queries
 * touch are formed: n_fb frequency bins (twiddles wt[nt][2 * n_fb] = cos | -sin) and n_kb
 * wavenumber bins (atab [2 * MT][K2] float64 = [[Er, -Ei], [Ei, Er]], MT = 16 * ceil(n_kb / 16),
 * K2 = 2 * nch rounded up to a multiple of 4).  Replaces fk (modules/utils.py:236-248) and map_fv (:457-475). */

/* 1 / ||row||_1 per gather row (map_fv norm=True, modules/utils.py:461-464). */
int dvh_disp_row_l1(const float* data, int64_t b_stride, int64_t ch_stride, int32_t B, int32_t nch, int32_t nt,
                    float* inv_l1, void* stream);

/* Time DFT on the float64 MFMA pipe: D[B * nch][2 * n_fb] float64 (re, im interleaved), rows
 * scaled by row_scale (nullable).  wt[nt][2 * n_fb] float64. */
int dvh_disp_tdft(const float* data, int64_t b_stride, int64_t ch_stride, int32_t B, int32_t nch, int32_t nt,
                  const double* wt, int32_t n_fb, const float* row_scale, double* D, void* stream);

/* Channel contraction (complex GEMM on MFMA) + |.|: FK[B][n_kb][n_fb]; with slot/weight
 * (both non-NULL) FK[slot[b]] += weight[b] * |Z_b| instead (class mean of |FK|), FK holding n_slot
 * slots (a slot outside [0, n_slot) is never written; callers validate slots on the host). */
int dvh_disp_fk(const double* D, int32_t B, int32_t nch, int32_t n_fb, const double* atab, int32_t MT, int32_t K2,
                int32_t n_kb, double* FK, const int32_t* slot, const float* weight, int32_t n_slot, void* stream);

/* f-v sampling: fv[B][nV][nF] = savgol(float32(bilinear(FK; k = kq[f][v], f)))  with the
 * interp2d query order (kq sorted per frequency), FITPACK clamping to [kmin, kmax], the compact
 * k grid kgrid[n_kb], per-frequency lower bin fj[nF] and weights fw[nF][2], and the
 * Savitzky-Golay operator sg = {h[sgl], left[sgl/2][sgl], right[sgl/2][sgl]}. */
int dvh_disp_fv(const double* FK, int32_t B, int32_t n_kb, int32_t n_fb, const double* kgrid, double kmin,
                double kmax, const double* kq, int32_t nF, int32_t nV, const int32_t* fj, const double* fw,
                const double* sg, int32_t sgl, float* fv, void* stream);

/* dvh_disp_fv for large batches with the FK cells staged per block: 256-thread blocks of 4 velocities x a
 * frequency tile (TO outputs, n_tile tiles, 12-sample halos; one tile when nF <= 256), block ct =
 * chunk * n_tile + tile stages only the cells its bilinear stencils read: cell_off[ct][max_cell] (FK
 * offsets m * n_fb + j, column-major per column), n_cell[ct], and per (f, v) of the block
 * qidx[ct][256][4][4] int32 = {compact index of (m, j), of (m, j + 1), m, 0}, f = tile start - halo + thread.
 * Tables: das_diff_veh_amd.disp.DispPlan.cell_tables.  VT must be 4.  Same outputs as dvh_disp_fv. */
int dvh_disp_fv_cells(const double* FK, int32_t B, int32_t n_kb, int32_t n_fb, const double* kgrid, double kmin,
                      double kmax, const double* kq, int32_t nF, int32_t nV, const double* fw, const double* sg,
                      int32_t sgl, int32_t TO, int32_t n_tile, int32_t VT, int32_t max_cell, const int32_t* cell_off,
                      const int32_t* n_cell, const int32_t* qidx, float* fv, void* stream);

/* dvh_disp_fv with the Savitzky-Golay filter on the float64 matrix pipe (map_fv's savgol,
 * modules/utils.py:473): each (16 velocities x 16 frequencies) output tile is one banded GEMM of
 * 10 v_mfma_f64_16x16x4_f64 steps over the float32-rounded bilinear samples.  Plan tables
 * (DispPlan.mfma_tables): hx[nF][nV][2] float64 = the FITPACK weights {fx (khi - q), fx (q - klo)} of
 * every clamped query on its interval m, cb[nF][nV] int32 = m * n_fb + fj[f] (the (m, j) cell of the
 * compact grid), fw[nF][2] as dvh_disp_fv.  G images per block (0: chosen by the launcher).  Needs
 * sgl == 25, nF >= 32, n_kb * n_fb <= 8192.  Same outputs as dvh_disp_fv. */
int dvh_disp_fv_mfma(const double* FK, int32_t B, int32_t n_kb, int32_t n_fb, const double* hx, const int32_t* cb,
                     int32_t nF, int32_t nV, const double* fw, const double* sg, int32_t sgl, int32_t G, float* fv,
                     void* stream);

/* ---------------------------------------------------------------- bootstrap / convergence
 * bootstrap_disp (apis/imaging_classes.py:8-48): per-pass gathers once, then per resample the mean
 * stack, its f-v image (dvh_disp_*) and the ridge picks (extract_ridge_ref_idx, modules/utils.py:621-678). */

/* out[b][k] = (sum_{j < m} G[sel[b * m + j] * pass_stride + k]) / m for k < K, summed in selection
 * order (sum(images) / len(images), apis/imaging_classes.py:106-107). */
int dvh_select_mean(const float* G, int64_t pass_stride, int64_t K, const int32_t* sel, int32_t B, int32_t m,
                    float* out, int64_t out_stride, void* stream);

/* dvh_select_mean for resamples of different sizes in one launch: resample b averages the cnt[b] >= 1 passes
 * sel[off[b] .. off[b] + cnt[b]) (device arrays; convergence_test's bt_size = 1 .. max_size draws). */
int dvh_select_mean_var(const float* G, int64_t pass_stride, int64_t K, const int32_t* sel, const int32_t* off,
                        const int32_t* cnt, int32_t B, float* out, int64_t out_stride, void* stream);

/* extract_ridge_ref_idx on the frequency band [c0, c0 + nb) of fv[b] ([nV][nF], b_stride elements
 * apart), rows = velocities vel[nV] strictly descending.  ref == INT32_MIN: vel_max mode (raw picks
 * below argmin |vel_max - vel|); vref (nullable, [nb]): per-frequency reference velocities; otherwise
 * the walk from column ref with the window (v - sigma, v + sigma); -nb <= ref < 0 indexes like Python
 * (column nb + ref, then the reference's loop order: forward to the end, then 0 .. nb - 1 again).  Picks of the last two modes are
 * smoothed by savgol(sgl, 2) given as sg = {h[sgl], left[sgl/2][sgl], right[sgl/2][sgl]}.
 * out[B][nb] float64; status[b] = 1 when a window held no velocity (the reference raises); picks
 * (nullable, [B][nb] float64) receives the raw picks before the smoothing. */
int dvh_ridge(const float* fv, int64_t b_stride, int32_t B, int32_t nV, int32_t nF, int32_t c0, int32_t nb,
              const double* vel, int32_t ref, double sigma, double vel_max, const double* vref, const double* sg,
              int32_t sgl, double* out, int32_t* status, double* picks, void* stream);

/* ---------------------------------------------------------------- preprocessing
 * dtype: 0 float32, 1 float64; data modified in place. */

/* scipy.signal.sosfiltfilt(sos, x, axis=-1) per row (bandpass_data, modules/utils.py:179-189);
 * zi = sosfilt_zi(sos) [n_sec][2] (device); n_sec <= 16.  Time-parallel: each row is filtered in blocks
 * (zero-state block filters, a scan of the 2 n_sec block states, re-filter), forward then backward, the blocks by
 * the filter's own recursion (any stable design).  work: 16-byte aligned device buffer of
 * dvh_sosfiltfilt_workspace(n_rows, n_t, n_sec, padlen) bytes. */
int64_t dvh_sosfiltfilt_workspace(int64_t n_rows, int32_t n_t, int32_t n_sec, int32_t padlen);
int dvh_sosfiltfilt(void* x, int32_t dtype, int64_t n_rows, int64_t row_stride, int32_t n_t, const double* sos,
                    int32_t n_sec, int32_t padlen, const double* zi, double* work, void* stream);
/* The matrix-pipe form: the blocks as float64 MFMA GEMMs with the block operators (impulse response, zero-input
 * responses, state responses, the block and group transitions), formed once per filter design and record length n_t
 * (they depend on n_t + 2 padlen through the scan's group size): plan = device buffer of dvh_sosfiltfilt_plan_bytes(
 * n_sec) bytes.  dvh_sosfiltfilt_planned filters with them (work: 16-byte aligned, dvh_sosfiltfilt_workspace bytes;
 * plan NULL: the recursion, as dvh_sosfiltfilt).  Its rounding grows with the largest pole radius r (host sos: dvh_sos_pole_radius):
 * 1e-13 relative at r = 0.9956, 5e-10 at r = 0.99973, so plan it only for r <= DVH_SOS_MFMA_MAX_POLE.
 * bandpass_data (modules/utils.py:179-189) called once per record of the same shape designs the same filter every
 * time; the drop-in caches the plan per (design, n_t).  A plan is valid only for the (n_t, padlen) it was formed for:
 * it records its group sizes, and a call whose scans need another group transition gets NaN in the output there
 * (records short enough to need no carried groups never read the transition and filter correctly). */
#define DVH_SOS_MFMA_MAX_POLE 0.999
double dvh_sos_pole_radius(const double* sos_host, int32_t n_sec);
int64_t dvh_sosfiltfilt_plan_bytes(int32_t n_sec);
int dvh_sosfiltfilt_plan(const double* sos, int32_t n_sec, const double* zi, int32_t n_t, int32_t padlen, double* plan,
                         void* stream);
int dvh_sosfiltfilt_planned(void* x, int32_t dtype, int64_t n_rows, int64_t row_stride, int32_t n_t, const double* sos,
                            int32_t n_sec, int32_t padlen, const double* zi, const double* plan, double* work,
                            void* stream);

/* SurfaceWaveWindow.mute_along_traj (apis/data_classes.py:49-72): tab[n_pass][n_t][3] =
 * {start, end, taper_start} per time sample; contiguous [n_ch][n_t] per pass. */
int dvh_mute_traj(void* data, int32_t dtype, int32_t n_pass, int64_t pass_stride, int32_t n_ch, int32_t n_t,
                  const int32_t* tab, const double* taper, void* stream);

/* TimeLapseImaging._preprocessing_for_surface_waves after the bandpass (apis/timeLapseImaging.py:
 * 51-71) on traces x[n_rows][n_t] (row_stride elements): flags 1 = impute the first empty trace
 * (||x_r|| < noise_threshold), 2 = then the first noisy trace (max x_r > noise_threshold), 4 = then
 * divide every trace by its L2 norm.  find_noise_idx / impute_noisy_trace (modules/utils.py:316-329)
 * semantics: np.argmax picks trace 0 when none qualifies; an interior trace becomes the SUM of its
 * neighbours.  stats: n_rows * 2 doubles of work ({sum x^2, max x} per trace); idx_out (nullable,
 * 2 ints) receives the imputed trace indices. */
int dvh_trace_cleanup(void* x, int32_t dtype, int64_t n_rows, int64_t row_stride, int32_t n_t, int32_t flags,
                      double noise_threshold, double* stats, int32_t* idx_out, void* stream);

/* SurfaceWaveSelector.locate_windows' cut (apis/data_classes.py:208-216): for every accepted pass w,
 * out[w][c][t] = rec[x_start + c][t_start[w] + t] (c < n_ch, t < n_t) into a contiguous batch,
 * converted from in_dtype to out_dtype (0 = float32, 1 = float64).  rec is [n_rows][rec_n_t] with
 * row_stride elements; t_start (device, n_win int64) is checked on the device: a window outside the
 * record sets *status (nullable) to 1 and is left unwritten. */
int dvh_cut_windows(const void* rec, int32_t in_dtype, int64_t n_rows, int64_t row_stride, int64_t rec_n_t,
                    const int64_t* t_start, int32_t n_win, int64_t x_start, int32_t n_ch, int32_t n_t, void* out,
                    int32_t out_dtype, int32_t* status, void* stream);

/* SurfaceWaveWindow.mute_along_time (apis/data_classes.py:100-104). */
int dvh_mute_time(void* data, int32_t dtype, int64_t n_rows, int32_t n_t, const double* taper, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DVH_H */
