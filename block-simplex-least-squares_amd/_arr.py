"""Tiny array-API shims so the solver loops accept NumPy arrays (as the
reference's callers pass) and HIP-resident torch tensors alike."""
import numpy as np


def is_torch(a):
    try:
        import torch
    except ImportError:
        return False
    return isinstance(a, torch.Tensor)


class Normed:
    """A vector whose norm is already known on the host (the device L-BFGS
    loop reads it with its other scalars): norm(v) is that value, and t * v
    (solvers.stopping's step test) keeps |t| times it, without a device read."""
    __slots__ = ('v', 'bsls_norm')

    def __init__(self, v, n):
        self.v, self.bsls_norm = v, float(n)

    def __rmul__(self, t):
        return Normed(None, abs(float(t)) * self.bsls_norm)


def norm(a):
    if isinstance(a, Normed):
        return a.bsls_norm
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
