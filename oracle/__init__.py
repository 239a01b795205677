"""ORACLE — TEST INFRASTRUCTURE ONLY.

A CPU restatement (numpy / scipy, float64) of the reference's hot path, used as the CHECKER in
``tests/``, in ``__graft_entry__.smoke()`` and as the ``cpu_baseline`` leg of ``bench.py``.
Nothing in ``das_diff_veh_amd/`` imports this package; the product path runs only the HIP
kernels of ``libdvh.so`` and fails loudly when they are missing.

Pinning: every function here is checked against golden vectors produced by running the reference
itself (NohPei/das_diff_veh, imported from /root/reference in the build container with the shims
listed in SURVEY.md §8(c)) by ``tests/golden/make_golden.py``; see ``tests/test_oracle.py``.
Third-party arithmetic the reference delegates to (SciPy 1.15.3 / NumPy 2.2.6 as installed here):
``scipy.signal.correlate``, ``scipy.interpolate.interp1d``, FITPACK bilinear splines (for the removed
``interp2d``), ``scipy.signal.savgol_filter`` and ``scipy.signal.sosfiltfilt``.  ``interp2d``'s exact
behaviour is pinned only through SciPy's documented ``RectBivariateSpline`` equivalence (the authors'
SciPy version is unknown): the dispersion image is "parity pinned to the shim", see DESIGN.md.

Modules:
  vsg        -- VirtualShotGather restatement (FFT-based circular xcorr, index tables, conventions)
  disp       -- map_fv / fk restatement (FK grid, bilinear clamp, Savitzky-Golay)
  preprocess -- bandpass_data (sosfiltfilt), mute_along_traj / mute_along_time
  ref_loop   -- CPU baseline that keeps the reference's per-row scipy.signal.correlate loop
  ridge      -- extract_ridge_ref_idx and bootstrap_disp restatements (bootstrap / convergence)
"""
