"""Device selection and host<->device staging for the drop-in API (PyTorch is plumbing only)."""
from __future__ import annotations

import atexit
import os
import threading

import numpy as np
import torch


def default_device():
    if not torch.cuda.is_available():
        raise RuntimeError("das_diff_veh_amd needs a HIP device (MI355X): the hot path has no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


# Host windows reach the device through a pipeline (stage_windows): chunks of about STAGE_BYTES (64 MB) are copied
# by a thread pool into one of two pinned buffers (in the windows' own dtype, no host-side conversion), sent
# by an asynchronous H2D copy on a side stream, and converted to float32 on the device, so that the host copy
# of chunk k + 1 runs while chunk k crosses PCIe.
STAGE_BYTES = int(os.environ.get("DVH_STAGE_MB", "64")) << 20  # 64 MB: 36.2-36.3 k vs 35.0-35.4 k windows/s at 128
_STAGE = {}
# One staging at a time per (device, dtype): the pinned and device chunk buffers are shared by every caller (the
# background thread of stage_async and the caller's own to_device_f32), so a staging holds its stager's lock from
# its first host copy to its last H2D issue.
_STAGE_LOCK = threading.Lock()


def _stager(device, dtype, nbytes):
    """(side stream, two pinned host buffers, two device buffers, two events, lock) for chunks of <= nbytes.
    A stager that must grow first drains its side stream (the old buffers' copies are done before they are
    dropped); its device buffers are allocated on the side stream, the only stream that touches them."""
    key = (str(device), str(dtype))
    with _STAGE_LOCK:
        st = _STAGE.get(key)
        if st is None:
            st = dict(nbytes=0, stream=torch.cuda.Stream(device=device), lock=threading.Lock(),
                      free=[torch.cuda.Event() for _ in range(2)])
            _STAGE[key] = st
    return st


def _grow(st, device, nbytes):
    """Called with st['lock'] held: buffers of >= nbytes (at least STAGE_BYTES, so they are sized once)."""
    if st["nbytes"] >= nbytes:
        return
    st["stream"].synchronize()  # the copies that read or write the old buffers are done
    nb = max(nbytes, STAGE_BYTES)
    st["pinned"] = [torch.empty(nb, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    with torch.cuda.stream(st["stream"]):
        st["dev"] = [torch.empty(nb, dtype=torch.uint8, device=device) for _ in range(2)]
    st["nbytes"] = nb


def sync_staging():
    """Wait for every staging side stream's queued copies (process exit, tests)."""
    with _STAGE_LOCK:
        sts = [v for k, v in _STAGE.items() if isinstance(k, tuple)]
    for st in sts:
        st["stream"].synchronize()


atexit.register(lambda: sync_staging() if torch.cuda.is_initialized() else None)


import ctypes  # noqa: E402

_NTHREADS = max(1, min(16, os.cpu_count() or 1))
# the host copy into pinned memory: native (dvh_host_gather on the thread pool, float32 C-contiguous windows;
# others take the pool path) | pool (np.copyto per window on the thread pool) | torch (torch.stack)
STAGE_MODE = os.environ.get("DVH_STAGE_MODE", "native")
STAGE_RAMP = int(os.environ.get("DVH_STAGE_RAMP", "0"))  # 0: off, r: first chunk k / r windows, doubling up to k


def _pool():
    import concurrent.futures as cf
    with _STAGE_LOCK:
        if "pool" not in _STAGE:
            _STAGE["pool"] = cf.ThreadPoolExecutor(_NTHREADS)
        return _STAGE["pool"]


def stage_windows(hosts, device, out=None, wait=True):
    """Same-shape 2-D NumPy arrays -> one float32 device tensor [n, C, T] (or into ``out``), pipelined:
    pinned double buffering, thread-parallel host copies, asynchronous H2D on a side stream, float64 ->
    float32 conversion on the device.  wait=True: the current stream waits for the copies; wait=False: the
    caller waits on the returned event (stage_async).  The call returns when the last host copy is done (the
    caller's arrays are free to change afterwards)."""
    n = len(hosts)
    shape = hosts[0].shape
    if any(h.shape != shape for h in hosts):
        raise ValueError("windows of one batch must share their shape")
    src = np.float32 if all(h.dtype == np.float32 for h in hosts) else np.float64
    if out is None:
        out = torch.empty((n,) + tuple(shape), dtype=torch.float32, device=device)
    per = int(np.prod(shape)) * np.dtype(src).itemsize
    k = max(1, min(n, STAGE_BYTES // max(per, 1)))
    st = _stager(device, src, k * per)
    with st["lock"]:
        _grow(st, device, k * per)
        return _stage_chunks(hosts, st, out, n, shape, src, per, k, device, wait)


def _stage_chunks(hosts, st, out, n, shape, src, per, k, device, wait):
    pool = _pool()
    tdt = torch.float32 if src == np.float32 else torch.float64
    # chunk starts: with STAGE_RAMP = r the first chunks are k / r, 2 k / r, ... windows, so that the first H2D
    # copy starts after a short host copy instead of a full one
    starts, a, kc = [], 0, max(1, k // STAGE_RAMP) if STAGE_RAMP > 0 else k
    while a < n:
        starts.append((a, min(kc, n - a)))
        a += kc
        kc = min(k, 2 * kc)
    for ci, (a, kk) in enumerate(starts):
        b = ci & 1
        st["free"][b].synchronize()  # the H2D that last read this pinned buffer is done
        if STAGE_MODE == "torch":  # torch's parallel CPU cat into the pinned buffer
            pin_t = st["pinned"][b][:kk * per].view(tdt).view((kk,) + tuple(shape))
            torch.stack([torch.from_numpy(np.ascontiguousarray(h, dtype=src)) for h in hosts[a:a + kk]], out=pin_t)
        else:  # thread pool, contiguous runs of windows per task
            view = st["pinned"][b].numpy()[:kk * per].view(src).reshape((kk,) + tuple(shape))
            nt = min(kk, _NTHREADS)
            bounds = [kk * q // nt for q in range(nt + 1)]
            chunk = hosts[a:a + kk]
            if STAGE_MODE == "native" and all(h.dtype == src and h.flags.c_contiguous for h in chunk):
                from . import _lib
                srcs = (ctypes.c_void_p * kk)(*[h.ctypes.data for h in chunk])
                base = view.ctypes.data

                def run(q):  # one native call per thread: no interpreter work per window, the lock released
                    j0, j1 = bounds[q], bounds[q + 1]
                    _lib.call("dvh_host_gather", ctypes.c_void_p(base + j0 * per),
                              ctypes.byref(srcs, j0 * ctypes.sizeof(ctypes.c_void_p)), per, j1 - j0)
            else:
                def run(q):
                    for j in range(bounds[q], bounds[q + 1]):
                        np.copyto(view[j], chunk[j], casting="unsafe")
            list(pool.map(run, range(nt)))
        with torch.cuda.stream(st["stream"]):
            pin = st["pinned"][b][:kk * per].view(tdt).view((kk,) + tuple(shape))
            if src == np.float32:
                out[a:a + kk].copy_(pin, non_blocking=True)
            else:
                d = st["dev"][b][:kk * per].view(tdt).view((kk,) + tuple(shape))
                d.copy_(pin, non_blocking=True)
                out[a:a + kk].copy_(d)
            st["free"][b].record(st["stream"])
    # `out` may come from another stream's pool (stage_async allocates it on the caller's stream): the allocator
    # must not hand its memory out again before the side stream's copies into it are done, even if the caller
    # drops it without waiting (an exception between staging and launch)
    out.record_stream(st["stream"])
    done = torch.cuda.Event()
    done.record(st["stream"])
    if wait:
        torch.cuda.current_stream(device).wait_event(done)
        return out
    return out, done


def stage_async(hosts, device):
    """stage_windows on a background thread: the host copies overlap the caller's own host work (e.g. the batch's
    tables).  Returns a _Staged: calling it yields the device tensor, the current stream made to wait for it."""
    import concurrent.futures as cf
    with _STAGE_LOCK:
        if "bg" not in _STAGE:
            _STAGE["bg"] = cf.ThreadPoolExecutor(1)
    n = len(hosts)
    out = torch.empty((n,) + tuple(hosts[0].shape), dtype=torch.float32, device=device)  # caller's stream
    fut = _STAGE["bg"].submit(stage_windows, hosts, device, out, False)
    return _Staged(fut, device)


class _Staged:
    """A staging in flight: call it for the device tensor (the current stream then waits for its copies);
    drain() waits for the host copies and the DMA without using the tensor (an abandoned staging: the pinned
    buffers are free for the next staging and no copy writes memory the caller has released)."""

    def __init__(self, fut, device):
        self._fut, self._device = fut, device

    def __call__(self):
        t, ev = self._fut.result()
        torch.cuda.current_stream(self._device).wait_event(ev)
        return t

    def drain(self):
        try:
            _, ev = self._fut.result()
        except Exception:  # the staging's own error belongs to whoever uses the tensor
            return
        ev.synchronize()


def to_device_f32(arrays, device=None):
    """Stack same-shape 2-D arrays (numpy or tensors) into one float32 device tensor [n, C, T]."""
    device = device or default_device()
    if all(isinstance(a, torch.Tensor) for a in arrays):
        return torch.stack([a.to(device=device, dtype=torch.float32) for a in arrays]).contiguous()
    hosts = [np.asarray(a.detach().cpu() if isinstance(a, torch.Tensor) else a) for a in arrays]
    if all(h.dtype in (np.float32, np.float64) and h.ndim == 2 for h in hosts) and hosts:
        return stage_windows(hosts, device)
    host = np.stack([np.asarray(h, dtype=np.float32) for h in hosts])
    return torch.from_numpy(host).to(device, non_blocking=False)


def upload(arrays, device):
    """Small host arrays -> device tensors through ONE pinned buffer and ONE asynchronous copy on the current
    stream (the caller does not wait; kernels queued after it on the stream see the data).  A plan's few
    tables cost one DMA queue slot instead of one blocking copy each, which matters while the window staging
    keeps the H2D engine busy with 128 MB chunks."""
    arrs = [np.ascontiguousarray(a) for a in arrays]
    offs, total = [], 0
    for a in arrs:
        offs.append(total)
        total += (a.nbytes + 15) & ~15
    host = torch.empty(max(total, 16), dtype=torch.uint8, pin_memory=True)
    hv = host.numpy()
    for a, o in zip(arrs, offs):
        hv[o:o + a.nbytes] = a.reshape(-1).view(np.uint8)
    dev = host.to(device, non_blocking=True)  # the pinned block is held by torch's host allocator until the copy ends
    return [dev[o:o + a.nbytes].view(torch.from_numpy(np.empty(0, a.dtype)).dtype).view(a.shape)
            for a, o in zip(arrs, offs)]


def to_host_f64(t):
    return t.detach().to("cpu").numpy().astype(np.float64)
