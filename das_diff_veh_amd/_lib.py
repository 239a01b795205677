"""ctypes binding of libdvh.so (C-ABI declared in include/dvh.h).

The library is loaded from ``das_diff_veh_amd/lib/libdvh.so``; if it is missing the import of any
compute entry point raises, there is no CPU fallback.  Every entry point takes raw device pointers
(``tensor.data_ptr()``) and the HIP stream of the current torch stream, and returns 0 or a negative
status whose message is ``dvh_last_error()``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DVH_LIB") or os.path.join(_PKG, "lib", "libdvh.so")

_i32, _i64, _p, _f32, _f64 = C.c_int32, C.c_int64, C.c_void_p, C.c_float, C.c_double

# name -> argtypes (restype is int32 status unless listed in _RESTYPES)
SIGNATURES = {
    "dvh_abi_version": [],
    "dvh_last_error": [],
    "dvh_vsg_fft_length": [_i32],
    "dvh_random_sample": [_p, _i64, _i64, _i32, _i32, _p],
    "dvh_host_gather": [_p, _p, _i64, _i32],
    "dvh_window_sumsq": [_p, _i64, _i64, _i32, _i32, _i32, _p, _p],
    "dvh_pass_geometry": [_p, _i64, _p, _i64, _i32, _p, _p, _i64, _p, _p, _p, _i32, _i32, _f64, _i32, _i32, _p,
                          _p, _p],
    "dvh_vsg_scales": [_p, _i64, _i64, _i32, _p, _p, _i32, _i32, _i32, _i32, _p, _p, _p],
    "dvh_vsg_gathers": [_p, _i64, _i64, _i32, _p, _p, _i32, _i32, _i32, _i32, _p, _p, _p],
    "dvh_vsg_stack": [_p, _i64, _i64, _i32, _p, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _i32, _p, _p, _p, _p],
    "dvh_vsg_stack_workspace": [_i32, _i32],
    "dvh_vsg_stack_validated": [_p, _i64, _i64, _i32, _i32, _i32, _p, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _i32,
                                _i32, _p, _p, _p, _i32, _p, _p, _p, _p],
    "dvh_disp_row_l1": [_p, _i64, _i64, _i32, _i32, _i32, _p, _p],
    "dvh_disp_tdft": [_p, _i64, _i64, _i32, _i32, _i32, _p, _i32, _p, _p, _p],
    "dvh_disp_fk": [_p, _i32, _i32, _i32, _p, _i32, _i32, _i32, _p, _p, _p, _i32, _p],
    "dvh_disp_fv": [_p, _i32, _i32, _i32, _p, _f64, _f64, _p, _i32, _i32, _p, _p, _p, _i32, _p, _p],
    "dvh_disp_fv_cells": [_p, _i32, _i32, _i32, _p, _f64, _f64, _p, _i32, _i32, _p, _p, _i32, _i32, _i32, _i32, _i32,
                          _p, _p, _p, _p, _p],
    "dvh_disp_fv_mfma": [_p, _i32, _i32, _i32, _p, _p, _i32, _i32, _p, _p, _i32, _i32, _p, _p],
    "dvh_select_mean": [_p, _i64, _i64, _p, _i32, _i32, _p, _i64, _p],
    "dvh_select_mean_var": [_p, _i64, _i64, _p, _p, _p, _i32, _p, _i64, _p],
    "dvh_ridge": [_p, _i64, _i32, _i32, _i32, _i32, _i32, _p, _i32, _f64, _f64, _p, _p, _i32, _p, _p, _p, _p],
    "dvh_sosfiltfilt_workspace": [_i64, _i32, _i32, _i32],
    "dvh_sosfiltfilt": [_p, _i32, _i64, _i64, _i32, _p, _i32, _i32, _p, _p, _p],
    "dvh_sosfiltfilt_plan_bytes": [_i32],
    "dvh_sos_pole_radius": [_p, _i32],
    "dvh_sosfiltfilt_plan": [_p, _i32, _p, _i32, _i32, _p, _p],
    "dvh_sosfiltfilt_planned": [_p, _i32, _i64, _i64, _i32, _p, _i32, _i32, _p, _p, _p, _p],
    "dvh_trace_cleanup": [_p, _i32, _i64, _i64, _i32, _i32, _f64, _p, _p, _p],
    "dvh_cut_windows": [_p, _i32, _i64, _i64, _i64, _p, _i32, _i64, _i32, _i32, _p, _i32, _p, _p],
    "dvh_mute_traj": [_p, _i32, _i32, _i64, _i32, _i32, _p, _p, _p],
    "dvh_mute_time": [_p, _i32, _i64, _i32, _p, _p],
}
_RESTYPES = {"dvh_last_error": C.c_char_p, "dvh_vsg_stack_workspace": C.c_int64, "dvh_sosfiltfilt_workspace": C.c_int64,
             "dvh_sosfiltfilt_plan_bytes": C.c_int64, "dvh_sos_pole_radius": C.c_double}

_lock = threading.Lock()
_lib = None


class DvhError(RuntimeError):
    pass


def load():
    """Load libdvh.so (once).  Raises if it has not been built: there is no CPU fallback."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise DvhError(f"{LIB_PATH} is missing: build it with `python -m das_diff_veh_amd.build` "
                               "(the product path has no CPU fallback)")
            lib = C.CDLL(LIB_PATH)
            for name, argtypes in SIGNATURES.items():
                fn = getattr(lib, name, None)
                if fn is None:
                    continue
                fn.argtypes = argtypes
                fn.restype = _RESTYPES.get(name, _i32)
            _lib = lib
    return _lib


def exported_symbols():
    lib = load()
    return [n for n in SIGNATURES if getattr(lib, n, None) is not None]


def call(name, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.dvh_last_error().decode(errors="replace")
        if rc == -4:
            raise ValueError(f"{name}: {msg}")
        raise DvhError(f"{name} failed ({rc}): {msg}")
    return rc


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else C.c_void_p(t.data_ptr())


def stream_of(device=None):
    import torch
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)
