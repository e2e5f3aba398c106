"""Tiny array-API shims so the solver loops accept NumPy arrays (as the
reference's callers pass) and HIP-resident torch tensors alike."""
import numpy as np


def is_torch(a):
    try:
        import torch
    except ImportError:
        return False
    return isinstance(a, torch.Tensor)


def norm(a):
    if is_torch(a):
        return float(a.norm())
    return float(np.linalg.norm(a))


def dot(a, b):
    if is_torch(a):
        return float(a.dot(b))
    return a.dot(b)


def builtin_sum(a):
    """BB.py:22 uses Python's builtin sum (left-to-right); a device tensor sums on
    the device instead (only `== 0` is tested)."""
    if is_torch(a):
        return float(a.sum())
    return sum(a)


def to_numpy(a):
    if is_torch(a):
        return a.detach().cpu().numpy()
    return np.asarray(a)


def copy(a):
    return a.clone() if is_torch(a) else np.array(a)
