"""The host path of the c_extensions drop-in (include/bsls_cpu.h): the
reference's Cython wrappers (python/c_extensions/c_extensions.pyx:22-248) over
lib/libbsls_cpu.so, for NumPy inputs when the CPU is selected explicitly
(BSLS_DEVICE=cpu / _native.set_device('cpu')).  Same buffer semantics as the
Cython module: np.ascontiguousarray(y) -- a non-contiguous y is projected into
a copy and the caller sees no change; weight=None -> fresh ones; a weight that
is already int32 and C-contiguous is updated in place, any other is copied.
The callers (c_extensions.py) have already made the type and layout checks."""
import ctypes

import numpy as np

import _native


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else ctypes.c_void_p(0)


def _i64(blocks):
    return np.ascontiguousarray(blocks, dtype=np.int64)


def proj_simplex(y, start, end):
    y_c = np.ascontiguousarray(y, dtype=np.float64)
    if _native.cpu_lib().bsls_cpu_proj_simplex(_p(y_c), int(start), int(end)) != 0:
        raise ValueError('proj_simplex_c: invalid arguments')


def proj_multi(ball, y, blocks):
    y_c = np.ascontiguousarray(y, dtype=np.float64)
    b = _i64(blocks)
    L = _native.cpu_lib()
    fn = L.bsls_cpu_proj_multi_ball if ball else L.bsls_cpu_proj_multi_simplex
    if fn(_p(y_c), _p(b), b.shape[0], y_c.shape[0], _native.cpu_threads()) != 0:
        raise ValueError('proj_multi: invalid arguments')


def isotonic(variant, y, blocks, n, weight, update):
    """isotonic_regression_multi{,_2,_3} over blocks of y[:n] (the single-block
    entries pass one start and end = n)."""
    y_c = np.ascontiguousarray(y, dtype=np.float64)
    b = _i64(blocks)
    w = None
    if variant != 2:
        if weight is None:
            w = np.ones(y_c.shape[0], dtype=np.int32)          # c_extensions.pyx:84
        else:
            w = np.ascontiguousarray(weight, dtype=np.int32)   # in place iff already int32
            if w.shape[0] < n:
                raise ValueError('weight must have at least len(y) entries')
            if np.any(w[int(b[0]):n] < 1):
                # the reference loops forever (weight 0) or reads out of bounds here
                raise ValueError('weight: run lengths must be >= 1')
    rc = _native.cpu_lib().bsls_cpu_isotonic_multi(int(variant), _p(y_c), _p(b), b.shape[0],
                                                   int(n), _p(w), int(update),
                                                   _native.cpu_threads())
    if rc != 0:
        raise ValueError('isotonic_regression: invalid arguments')


def quad_obj(x, Q, c, g):
    x_c, Q_c, c_c, g_c = (np.ascontiguousarray(a, dtype=np.float64) for a in (x, Q, c, g))
    return float(_native.cpu_lib().bsls_cpu_quad_obj(_p(x_c), _p(Q_c), _p(c_c), _p(g_c),
                                                     x_c.shape[0]))


def line_search(x, f, g, x_new, f_new, g_new, Q, c):
    x_c, g_c, xn_c, gn_c, Q_c, c_c = (np.ascontiguousarray(a, dtype=np.float64)
                                      for a in (x, g, x_new, g_new, Q, c))
    return float(_native.cpu_lib().bsls_cpu_line_search(_p(x_c), float(f), _p(g_c), _p(xn_c),
                                                        float(f_new), _p(gn_c), _p(Q_c),
                                                        _p(c_c), x_c.shape[0]))


def x2z(x, z, blocks, nz):
    """z[j] written through the caller's buffer (the reference's typed
    memoryview writes strided arrays too)."""
    x_c = np.ascontiguousarray(x, dtype=np.float64)
    z_c = z if z.flags['C_CONTIGUOUS'] else np.zeros(max(nz, 1))
    b = _i64(blocks)
    if _native.cpu_lib().bsls_cpu_x2z(_p(x_c), _p(z_c), _p(b), b.shape[0], x_c.shape[0]) != 0:
        raise ValueError('x2z_c: invalid arguments')
    if z_c is not z:
        z[:nz] = z_c[:nz]
    return z


def z2x(x, z, blocks):
    z_c = np.ascontiguousarray(z, dtype=np.float64)
    x_c = x if x.flags['C_CONTIGUOUS'] else np.zeros(x.shape[0])
    b = _i64(blocks)
    if _native.cpu_lib().bsls_cpu_z2x(_p(x_c), _p(z_c), _p(b), b.shape[0], x_c.shape[0]) != 0:
        raise ValueError('z2x_c: invalid arguments')
    if x_c is not x:
        x[:] = x_c
    return x
