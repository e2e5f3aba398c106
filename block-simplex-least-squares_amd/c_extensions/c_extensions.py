"""Drop-in replacement for the reference's Cython module ``c_extensions.c_extensions``
(python/c_extensions/c_extensions.pyx:22-248), running on MI355X through the C ABI
of include/bsls_hip.h.

Same function names, argument meaning, asserts and in-place behaviour:
  * ``y`` is modified in place and the functions return None (x2z_c / z2x_c
    return the output array, quad_obj_c / line_search_quad_obj_c a float);
  * NumPy ``y`` must be 1-D float64 and ``blocks`` 1-D int64 (Cython buffer
    typing -> ValueError otherwise); layout violations raise AssertionError
    before anything is launched (c_extensions.pyx:24,33-34,203,231);
  * like ``np.ascontiguousarray`` in the reference, a NumPy ``y`` that is not
    C-contiguous is projected into a temporary and the caller sees no change;
  * a caller-supplied int32 C-contiguous ``weight`` array is updated in place
    (the reference passes it straight to C); any other weight is copied.

Inputs may be NumPy arrays (staged to HBM and back over PCIe for each call) or
float64 ``torch`` tensors already on the GPU (projected in place, no copies) --
the fused solver path uses the latter.  There is no CPU fallback: without the
HIP library or a HIP device every function raises RuntimeError.  The host path
(include/bsls_cpu.h, c_extensions/_cpu.py: the reference's own CPU path,
BASELINE configs[0]) runs NumPy inputs only when selected explicitly
(BSLS_DEVICE=cpu or _native.set_device('cpu')).

Projections (proj_simplex_c, proj_multi_simplex_c, proj_multi_ball_c) take the
sorting kernels, which reproduce the reference bit for bit; BSLS_PROJ=fast
selects the sort-free ones (bsls_proj_multi_*_fast: within 1e-12 * max(1,
|ref|), the north star's projection contract -- measured no faster on C2,
DESIGN.md §4).
"""
import os

import numpy as np

import _native
from _native import check, ptr, stream_handle
from c_extensions import _cpu

__all__ = ['proj_simplex_c', 'proj_multi_simplex_c', 'proj_multi_ball_c',
           'isotonic_regression_c', 'isotonic_regression_multi_c',
           'isotonic_regression_c_2', 'isotonic_regression_multi_c_2',
           'isotonic_regression_c_3', 'isotonic_regression_multi_c_3',
           'quad_obj_c', 'line_search_quad_obj_c', 'x2z_c', 'z2x_c']


def _torch():
    import torch
    return torch


def _is_tensor(a):
    try:
        import torch
    except ImportError:
        return False
    return isinstance(a, torch.Tensor)


def _check_y(y, name='y'):
    """Cython typing of `np.ndarray[np.double_t, ndim=1]`."""
    if _is_tensor(y):
        torch = _torch()
        if y.dtype != torch.float64 or y.dim() != 1:
            raise ValueError('%s must be a 1-D float64 tensor' % name)
        if not y.is_cuda:
            raise ValueError('%s: torch tensors must live on the HIP device' % name)
        if not y.is_contiguous():
            raise ValueError('%s: device tensors must be contiguous' % name)
        return
    if not isinstance(y, np.ndarray):
        raise TypeError("Argument '%s' has incorrect type (expected numpy.ndarray, got %s)"
                        % (name, type(y).__name__))
    if y.ndim != 1:
        raise ValueError('Buffer has wrong number of dimensions (expected 1, got %d)' % y.ndim)
    if y.dtype != np.float64:
        raise ValueError("Buffer dtype mismatch, expected 'double_t' but got '%s'" % y.dtype)


def _cpu_sel(*arrays):
    """The explicitly selected host path, for NumPy inputs (device tensors stay
    on the device)."""
    return _native.device_mode() == 'cpu' and not any(_is_tensor(a) for a in arrays)


def _host_blocks(blocks):
    if _is_tensor(blocks):
        return blocks.detach().cpu().numpy()
    return blocks


def _check_blocks_typed(blocks):
    """Cython typing of `np.ndarray[np.int_t, ndim=1]` (int64 on Linux)."""
    if _is_tensor(blocks):
        torch = _torch()
        if blocks.dtype != torch.int64 or blocks.dim() != 1:
            raise ValueError('blocks must be a 1-D int64 tensor')
        return
    if not isinstance(blocks, np.ndarray):
        raise TypeError("Argument 'blocks' has incorrect type (expected numpy.ndarray, got %s)"
                        % type(blocks).__name__)
    if blocks.ndim != 1:
        raise ValueError('Buffer has wrong number of dimensions (expected 1, got %d)'
                         % blocks.ndim)
    if blocks.dtype != np.int64:
        raise ValueError("Buffer dtype mismatch, expected 'int_t' but got '%s'" % blocks.dtype)


def _assert_multi(blocks_h, n):
    # c_extensions.pyx:33-34
    assert False not in ((blocks_h[1:] - blocks_h[:-1]) > 0)
    assert blocks_h[0] >= 0 and blocks_h[-1] < n


def _max_block(blocks_h, n):
    ends = np.append(blocks_h[1:], n)
    return int(np.max(ends - blocks_h))


class _Staged:
    """A float64 vector on the device: the caller's tensor itself, or a NumPy
    array copied over (and copied back on commit if the reference would have
    written into the caller's buffer)."""

    def __init__(self, a):
        torch = _torch()
        self.host = None
        if _is_tensor(a):
            self.dev = a
        else:
            self.host = a
            self.dev = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()

    def commit(self):
        if self.host is not None and self.host.flags['C_CONTIGUOUS']:
            self.host[...] = self.dev.cpu().numpy()


def _dev_i64(a):
    torch = _torch()
    if _is_tensor(a):
        return a.to(device='cuda', dtype=torch.int64).contiguous()
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64)).cuda()


def _work(nbytes):
    torch = _torch()
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device='cuda')


def _proj_entry(fn_name):
    """The C entry for a projection: the bit-identical sorting kernels, or
    the sort-free _fast ones with BSLS_PROJ=fast (read per call, so a test or
    caller can switch)."""
    mode = os.environ.get('BSLS_PROJ', 'exact')
    if mode not in ('fast', 'exact'):
        raise ValueError('BSLS_PROJ must be fast or exact, not %r' % mode)
    return fn_name + ('_fast' if mode == 'fast' else '')


def _run_proj(fn_name, y, blocks_h, n, first_offset=0):
    fn_name = _proj_entry(fn_name)
    L = _native.lib()
    st = _Staged(y)
    dev = st.dev if first_offset == 0 else st.dev
    b = _dev_i64(blocks_h)
    mb = _max_block(blocks_h, n)
    ws_bytes = L.bsls_proj_workspace_size(n, len(blocks_h), mb)
    ws = _work(ws_bytes)
    rc = getattr(L, fn_name)(ptr(dev), ptr(b), len(blocks_h), n, mb, ptr(ws), ws.numel(),
                             stream_handle())
    check(rc, fn_name)
    _torch().cuda.synchronize()
    st.commit()


# ---------------------------------------------------------------- simplex / ball

def proj_simplex_c(y, start, end):
    """c_extensions.pyx:22-28 -> proj_simplex.h:17-34 on y[start:end]."""
    _check_y(y)
    n = y.shape[0]
    assert start >= 0 and start < n and end > 0 and end <= n
    if start >= end:
        return
    if _cpu_sel(y):
        return _cpu.proj_simplex(y, start, end)
    st = _Staged(y)
    L = _native.lib()
    sub = st.dev[:end]
    b = _dev_i64(np.array([start], dtype=np.int64))
    ws = _work(L.bsls_proj_workspace_size(end, 1, end - start))
    fn = getattr(L, _proj_entry('bsls_proj_multi_simplex'))
    check(fn(ptr(sub), ptr(b), 1, end, end - start, ptr(ws), ws.numel(), stream_handle()),
          'proj_simplex_c')
    _torch().cuda.synchronize()
    st.commit()


def proj_multi_simplex_c(y, blocks):
    """c_extensions.pyx:31-39 -> proj_multi_simplex (proj_simplex.h:37-47)."""
    _check_y(y)
    _check_blocks_typed(blocks)
    bh = _host_blocks(blocks)
    _assert_multi(bh, y.shape[0])
    if _cpu_sel(y, blocks):
        return _cpu.proj_multi(False, y, bh)
    _run_proj('bsls_proj_multi_simplex', y, bh, y.shape[0])


def proj_multi_ball_c(y, blocks):
    """c_extensions.pyx:42-50 -> proj_multi_ball (proj_simplex.h:50-74)."""
    _check_y(y)
    _check_blocks_typed(blocks)
    bh = _host_blocks(blocks)
    _assert_multi(bh, y.shape[0])
    if _cpu_sel(y, blocks):
        return _cpu.proj_multi(True, y, bh)
    _run_proj('bsls_proj_multi_ball', y, bh, y.shape[0])


# ---------------------------------------------------------------- isotonic

def _weights(weight, n, first):
    """Return (device int32 weights, host array to write back or None)."""
    torch = _torch()
    if weight is None:
        return None, None       # fresh ones, nothing to hand back (c_extensions.pyx:84)
    if _is_tensor(weight):
        if weight.dtype != torch.int32 or not weight.is_cuda or not weight.is_contiguous():
            w = weight.to(device='cuda', dtype=torch.int32).contiguous()
            return w, None
        if bool((weight[first:] < 1).any()):
            raise ValueError('weight: run lengths must be >= 1')
        return weight, None
    w_c = np.ascontiguousarray(weight, dtype=np.int32)
    if w_c.shape[0] < n:
        raise ValueError('weight must have at least len(y) entries')
    if np.any(w_c[first:n] < 1):
        # the reference loops forever (weight 0) or reads out of bounds here
        raise ValueError('weight: run lengths must be >= 1')
    back = weight if (w_c is weight) else None
    return torch.from_numpy(w_c).cuda(), back


def _run_iso(variant, y, blocks_h, n, weight, update, name):
    if _cpu_sel(y, weight):
        return _cpu.isotonic(variant, y, blocks_h, n, weight, update)
    torch = _torch()
    L = _native.lib()
    if variant == 1 and weight is None and update:
        # main.py's call (fresh unit run lengths, expanded): the layout's pack
        # plan, made once and cached by content (device.iso_plan), one launch
        from device import iso_plan
        st = _Staged(y)
        iso_plan(np.asarray(blocks_h, dtype=np.int64), n).apply(st.dev)
        st.commit()
        return
    st = _Staged(y)
    dev = st.dev[:n]
    wdev, wback = (None, None) if variant == 2 else _weights(weight, n, int(blocks_h[0]))
    b = _dev_i64(blocks_h)
    ws = _work(L.bsls_isotonic_workspace_size(n))
    status = torch.zeros(1, dtype=torch.int32, device='cuda')
    rc = L.bsls_isotonic_multi(variant, ptr(dev), ptr(b), len(blocks_h), n, ptr(wdev),
                               int(update), _max_block(blocks_h, n), ptr(ws), ws.numel(),
                               ptr(status), stream_handle())
    check(rc, name)
    if int(status.item()) != 0:
        raise RuntimeError('%s: inconsistent run-length weights' % name)
    st.commit()
    if wback is not None:
        wback[...] = wdev.cpu().numpy()


def isotonic_regression_c(y, start, end, weight=None, update=1):
    """c_extensions.pyx:63-73 -> isotonic_regression (isotonic_regression.h:13-58)."""
    _check_y(y)
    n = y.shape[0]
    assert start >= 0 and start < n and end > 0 and end <= n
    if start >= end:
        return
    _run_iso(1, y, np.array([start], dtype=np.int64), end, weight, update,
             'isotonic_regression_c')


def isotonic_regression_multi_c(y, blocks, weight=None, update=1):
    """c_extensions.pyx:76-89 -> isotonic_regression_multi (isotonic_regression.h:85-92)."""
    _check_y(y)
    _check_blocks_typed(blocks)
    bh = _host_blocks(blocks)
    _assert_multi(bh, y.shape[0])
    _run_iso(1, y, bh, y.shape[0], weight, update, 'isotonic_regression_multi_c')


def isotonic_regression_c_2(y, start, end):
    """c_extensions.pyx:92-98 -> isotonic_regression_2 (isotonic_regression.h:61-82)."""
    _check_y(y)
    n = y.shape[0]
    assert start >= 0 and start < n and end > 0 and end <= n
    if start >= end:
        return
    _run_iso(2, y, np.array([start], dtype=np.int64), end, None, 1, 'isotonic_regression_c_2')


def isotonic_regression_multi_c_2(y, blocks):
    """c_extensions.pyx:101-109 -> isotonic_regression_multi_2."""
    _check_y(y)
    _check_blocks_typed(blocks)
    bh = _host_blocks(blocks)
    _assert_multi(bh, y.shape[0])
    _run_iso(2, y, bh, y.shape[0], None, 1, 'isotonic_regression_multi_c_2')


def isotonic_regression_c_3(y, start, end, weight=None, update=1):
    """c_extensions.pyx:112-122 -> isotonic_regression_3 (isotonic_regression.h:105-155)."""
    _check_y(y)
    n = y.shape[0]
    assert start >= 0 and start < n and end > 0 and end <= n
    if start >= end:
        return
    _run_iso(3, y, np.array([start], dtype=np.int64), end, weight, update,
             'isotonic_regression_c_3')


def isotonic_regression_multi_c_3(y, blocks, weight=None, update=1):
    """c_extensions.pyx:125-138 -> isotonic_regression_multi_3."""
    _check_y(y)
    _check_blocks_typed(blocks)
    bh = _host_blocks(blocks)
    _assert_multi(bh, y.shape[0])
    _run_iso(3, y, bh, y.shape[0], weight, update, 'isotonic_regression_multi_c_3')


# ---------------------------------------------------------------- dense QP (ABI parity)

def quad_obj_c(x, Q, c, g):
    """c_extensions.pyx:148-160 -> quad_obj (quadratic_objective.h:15-26); returns f,
    writes g in place (when g is C-contiguous float64, like the reference)."""
    for name, a in (('x', x), ('Q', Q), ('c', c), ('g', g)):
        _check_y(a, name)
    if _cpu_sel(x, Q, c, g):
        return _cpu.quad_obj(x, Q, c, g)
    torch = _torch()
    L = _native.lib()
    n = x.shape[0]
    sx, sQ, sc, sg = _Staged(x), _Staged(Q), _Staged(c), _Staged(g)
    f = torch.zeros(1, dtype=torch.float64, device='cuda')
    check(L.bsls_quad_obj(ptr(sx.dev), ptr(sQ.dev), ptr(sc.dev), ptr(sg.dev), n, ptr(f),
                          stream_handle()), 'quad_obj_c')
    out = float(f.item())
    sg.commit()
    return out


def line_search_quad_obj_c(x, f, g, x_new, f_new, g_new, Q, c):
    """c_extensions.pyx:171-192 -> line_search (quadratic_objective.h:29-61); returns
    f_new, updates x_new / g_new in place.  The reference's out-of-bounds store
    g_new[n] on its "step too small" path is not reproduced (g_new keeps its
    last value there, as it does on valid memory in the reference)."""
    for name, a in (('x', x), ('g', g), ('x_new', x_new), ('g_new', g_new), ('Q', Q), ('c', c)):
        _check_y(a, name)
    if _cpu_sel(x, g, x_new, g_new, Q, c):
        return _cpu.line_search(x, f, g, x_new, f_new, g_new, Q, c)
    torch = _torch()
    L = _native.lib()
    n = x.shape[0]
    sx, sg, sxn, sgn, sQ, sc = (_Staged(a) for a in (x, g, x_new, g_new, Q, c))
    fo = torch.zeros(1, dtype=torch.float64, device='cuda')
    check(L.bsls_line_search(ptr(sx.dev), float(f), ptr(sg.dev), ptr(sxn.dev), float(f_new),
                             ptr(sgn.dev), ptr(sQ.dev), ptr(sc.dev), n, ptr(fo),
                             stream_handle()), 'line_search_quad_obj_c')
    out = float(fo.item())
    sxn.commit()
    sgn.commit()
    return out


# ---------------------------------------------------------------- x <-> z

def _xz_blocks(blocks, n):
    bh = np.asarray(_host_blocks(blocks))
    assert False not in ((bh[1:] - bh[:-1]) > 0)
    assert bh[0] == 0 and bh[-1] < n          # c_extensions.pyx:203,231
    return bh


def x2z_c(x, z, blocks):
    """c_extensions.pyx:195-220: z = per-block running sums of x (last entry dropped).
    Returns z (written in place, strided NumPy views included)."""
    _check_y(x, 'x')
    _check_y(z, 'z')
    n = x.shape[0]
    bh = _xz_blocks(blocks, n)
    nz = n - len(bh)
    if z.shape[0] < nz:
        raise IndexError('Out of bounds on buffer access (axis 0)')
    if _cpu_sel(x, z):
        return _cpu.x2z(x, z, bh, nz)
    L = _native.lib()
    sx = _Staged(x)
    torch = _torch()
    zd = z if _is_tensor(z) else torch.zeros(max(nz, 1), dtype=torch.float64, device='cuda')
    check(L.bsls_x2z(ptr(sx.dev), ptr(zd), ptr(_dev_i64(bh)), len(bh), n, stream_handle()),
          'x2z_c')
    if not _is_tensor(z):
        z[:nz] = zd[:nz].cpu().numpy()
    return z


def z2x_c(x, z, blocks):
    """c_extensions.pyx:223-248: x = x0 + N z (per-block differences, last entry
    1 - z_last).  Returns x (written in place, strided NumPy views included)."""
    _check_y(x, 'x')
    _check_y(z, 'z')
    n = x.shape[0]
    bh = _xz_blocks(blocks, n)
    nz = n - len(bh)
    if z.shape[0] < nz:
        raise IndexError('Out of bounds on buffer access (axis 0)')
    if _cpu_sel(x, z):
        return _cpu.z2x(x, z, bh)
    L = _native.lib()
    torch = _torch()
    sz = _Staged(z)
    xd = x if _is_tensor(x) else torch.empty(n, dtype=torch.float64, device='cuda')
    check(L.bsls_z2x(ptr(xd), ptr(sz.dev), ptr(_dev_i64(bh)), len(bh), n, stream_handle()),
          'z2x_c')
    if not _is_tensor(x):
        x[:] = xd.cpu().numpy()
    return x
