"""Device selection and host<->device staging for the drop-in API (PyTorch is plumbing only)."""
from __future__ import annotations

import numpy as np
import torch


def default_device():
    if not torch.cuda.is_available():
        raise RuntimeError("das_diff_veh_amd needs a HIP device (MI355X): the hot path has no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def to_device_f32(arrays, device=None):
    """Stack same-shape 2-D arrays (numpy or tensors) into one float32 device tensor [n, C, T]."""
    device = device or default_device()
    if all(isinstance(a, torch.Tensor) for a in arrays):
        return torch.stack([a.to(device=device, dtype=torch.float32) for a in arrays]).contiguous()
    host = np.stack([np.asarray(a.detach().cpu() if isinstance(a, torch.Tensor) else a, dtype=np.float32)
                     for a in arrays])
    return torch.from_numpy(host).to(device, non_blocking=False)


def to_host_f64(t):
    return t.detach().to("cpu").numpy().astype(np.float64)
