"""CPU oracle for the block-simplex LSQ hot path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / the timed CPU baseline.  The product
(block-simplex-least-squares_amd/) never imports it and has no CPU fallback.

Contents
  * ctypes bindings to oracle/libbsls_oracle.so -- the C restatement of the
    reference kernels (oracle/bsls_oracle.c), exposed with the reference's
    c_extensions call signatures (python/c_extensions/c_extensions.pyx:22-248);
  * optional bindings to oracle/_ref/libbsls_ref.so -- the reference's own
    headers compiled in this container (oracle/Makefile) -- used to pin the
    restatement;
  * numpy restatements of the solver loops the hot path runs inside:
      bb_solve            python/BB.py:7-45
      lbfgs_solve         python/LBFGS.py:56-123 (+ weak_wolfe_ls :9-53)
      stopping            python/solvers.py:40-63
      dore_solve          python/DORE.py:6-90
      md_least_squares    python/mirror_descent.py:7-53
      solve_in_z_parts    python/main.py:41-65 (f, nabla_f, proj closures)
      lsv_operator        python/bsls_utils.py:334-369
      batch_solve_bb      python/BATCH.py:55-106 over algorithm_utils.get_solver_parts
                          (is_sparse=True), line_search_np, stopping
                          (python/algorithm_utils.py:88-94,113-137,158-172,182-271)
      batch_solve_md      python/BATCH.py:217-250 (+ normalization :175-179)
    SpMV inside them is SciPy csr_matvec, exactly what the reference calls.

Parity status: pinned (tests/test_oracle_pinning.py checks every function
against tests/golden/*.npz captured from the reference by
tests/golden/make_golden.py, and against _ref when it is present).
"""
import ctypes
import logging
import math
import os
import subprocess
import time

import numpy as np
import numpy.linalg as la
import scipy.sparse as sps
import scipy.sparse.linalg as sla

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, 'libbsls_oracle.so')
CPUBB_SO = os.path.join(HERE, 'libbsls_cpubb.so')
REF_SO = os.path.join(HERE, '_ref', 'libbsls_ref.so')

_D = ctypes.POINTER(ctypes.c_double)
_I32 = ctypes.POINTER(ctypes.c_int32)
_I64 = ctypes.POINTER(ctypes.c_int64)
_i64 = ctypes.c_int64


def build():
    """Compile the checker libraries (oracle/Makefile)."""
    subprocess.check_call(['make', '-s', '-C', HERE])


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = ctypes.CDLL(ORACLE_SO)
        for name in ('orc_proj_multi_simplex', 'orc_proj_multi_ball', 'orc_iso_multi_v2'):
            getattr(L, name).argtypes = [_D, _I64, _i64, _i64]
        L.orc_proj_simplex.argtypes = [_D, _i64, _i64]
        for name in ('orc_iso_multi_v1', 'orc_iso_multi_v3'):
            getattr(L, name).argtypes = [_D, _I64, _i64, _i64, _I32, ctypes.c_int]
        for name in ('orc_iso_v1', 'orc_iso_v3'):
            getattr(L, name).argtypes = [_D, _i64, _i64, _I32, ctypes.c_int]
        L.orc_iso_v2.argtypes = [_D, _i64, _i64]
        L.orc_quad_obj.argtypes = [_D, _D, _D, _D, _i64]
        L.orc_quad_obj.restype = ctypes.c_double
        L.orc_line_search.argtypes = [_D, ctypes.c_double, _D, _D, ctypes.c_double, _D, _D,
                                      _D, _i64]
        L.orc_line_search.restype = ctypes.c_double
        L.orc_x2z.argtypes = [_D, _D, _I64, _i64, _i64]
        L.orc_z2x.argtypes = [_D, _D, _I64, _i64, _i64]
        L.orc_csr_matvec.argtypes = [_i64, _I32, _I32, _D, _D, _D]
        _lib = L
    return _lib


_cpubb = None


def cpu_bb_run(A, b, block_sizes, iters, threads=1, AT=None, z0=None):
    """The z-space BB loop as a C + OpenMP port (bsls_cpu_bb.c: BB.py over
    main.py's closures, the reference's work per iteration, early exits off):
    `iters` iterations from z0 (default x2z(particular_x0) = 0) on `threads`
    threads.  Returns (z, f).  bench.py's all-cores CPU baseline."""
    global _cpubb
    if _cpubb is None:
        if not os.path.exists(CPUBB_SO):
            build()
        L = ctypes.CDLL(CPUBB_SO)
        L.cpubb_run.argtypes = [_i64, _i64, _i64, _I64, _I64, _I32, _D, _I64, _I32, _D, _D, _D,
                                _i64, ctypes.c_int]
        L.cpubb_run.restype = ctypes.c_double
        _cpubb = L
    A = sps.csr_matrix(A)
    AT = sps.csr_matrix(AT) if AT is not None else A.T.tocsr()
    sizes = np.asarray(block_sizes, dtype=np.int64)
    xs = np.concatenate(([0], np.cumsum(sizes)[:-1])).astype(np.int64)
    m, n = A.shape
    x0 = particular_x0(sizes)
    target = np.ascontiguousarray(A.dot(x0) - b, dtype=np.float64)
    z = np.zeros(n - sizes.size) if z0 is None else np.array(z0, dtype=np.float64)
    ip, ix, v = _p64c(A.indptr), np.ascontiguousarray(A.indices, np.int32), A.data
    ipt, ixt, vt = _p64c(AT.indptr), np.ascontiguousarray(AT.indices, np.int32), AT.data
    v, vt = np.ascontiguousarray(v, np.float64), np.ascontiguousarray(vt, np.float64)
    fx = _cpubb.cpubb_run(m, n, sizes.size, _p64(xs), _p64(ip), _p32(ix), _pd(v), _p64(ipt),
                          _p32(ixt), _pd(vt), _pd(target), _pd(z), int(iters), int(threads))
    return z, fx


def _p64c(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def ref_lib():
    """The reference's own kernels (None where /root/reference was absent)."""
    global _ref
    if _ref is None and os.path.exists(REF_SO):
        R = ctypes.CDLL(REF_SO)
        ci = ctypes.c_int
        R.ref_proj_simplex.argtypes = [_D, ci, ci]
        for nm in ('ref_proj_multi_simplex', 'ref_proj_multi_ball',
                   'ref_isotonic_regression_multi_2'):
            getattr(R, nm).argtypes = [_D, _I32, ci, ci]
        for nm in ('ref_isotonic_regression_multi', 'ref_isotonic_regression_multi_3'):
            getattr(R, nm).argtypes = [_D, _I32, ci, ci, _I32, ci]
        R.ref_quad_obj.argtypes = [_D, _D, _D, _D, ci]
        R.ref_quad_obj.restype = ctypes.c_double
        R.ref_line_search.argtypes = [_D, ctypes.c_double, _D, _D, ctypes.c_double, _D, _D,
                                      _D, ci]
        R.ref_line_search.restype = ctypes.c_double
        _ref = R
    return _ref


def _pd(a):
    return a.ctypes.data_as(_D)


def _p64(a):
    return a.ctypes.data_as(_I64)


def _p32(a):
    return a.ctypes.data_as(_I32)


def _check_multi(y, blocks):
    blocks = np.asarray(blocks)
    assert False not in ((blocks[1:] - blocks[:-1]) > 0)
    assert blocks[0] >= 0 and blocks[-1] < y.shape[0]
    return np.ascontiguousarray(blocks, dtype=np.int64)


# ----- c_extensions-shaped wrappers (in place on contiguous float64 y) -------

def proj_simplex_c(y, start, end):
    n = y.shape[0]
    assert start >= 0 and start < n and end > 0 and end <= n
    if start >= end:
        return
    lib().orc_proj_simplex(_pd(y), start, end)


def proj_multi_simplex_c(y, blocks):
    b = _check_multi(y, blocks)
    lib().orc_proj_multi_simplex(_pd(y), _p64(b), len(b), y.shape[0])


def proj_multi_ball_c(y, blocks):
    b = _check_multi(y, blocks)
    lib().orc_proj_multi_ball(_pd(y), _p64(b), len(b), y.shape[0])


def _weights(weight, n):
    if weight is None:
        return np.ones(n, dtype=np.int32)
    return np.ascontiguousarray(weight, dtype=np.int32)


def isotonic_regression_multi_c(y, blocks, weight=None, update=1):
    b = _check_multi(y, blocks)
    w = _weights(weight, y.shape[0])
    lib().orc_iso_multi_v1(_pd(y), _p64(b), len(b), y.shape[0], _p32(w), update)
    return w


def isotonic_regression_multi_c_2(y, blocks):
    b = _check_multi(y, blocks)
    lib().orc_iso_multi_v2(_pd(y), _p64(b), len(b), y.shape[0])


def isotonic_regression_multi_c_3(y, blocks, weight=None, update=1):
    b = _check_multi(y, blocks)
    w = _weights(weight, y.shape[0])
    lib().orc_iso_multi_v3(_pd(y), _p64(b), len(b), y.shape[0], _p32(w), update)
    return w


def isotonic_regression_c(y, start, end, weight=None, update=1):
    w = _weights(weight, y.shape[0])
    lib().orc_iso_v1(_pd(y), start, end, _p32(w), update)
    return w


def quad_obj_c(x, Q_flat, c, g):
    return lib().orc_quad_obj(_pd(x), _pd(Q_flat), _pd(c), _pd(g), x.shape[0])


def line_search_quad_obj_c(x, f, g, x_new, f_new, g_new, Q_flat, c):
    return lib().orc_line_search(_pd(x), f, _pd(g), _pd(x_new), f_new, _pd(g_new),
                                 _pd(Q_flat), _pd(c), x.shape[0])


def x2z_c(x, z, blocks):
    b = np.ascontiguousarray(blocks, dtype=np.int64)
    lib().orc_x2z(_pd(x), _pd(z), _p64(b), len(b), x.shape[0])
    return z


def z2x_c(x, z, blocks):
    b = np.ascontiguousarray(blocks, dtype=np.int64)
    lib().orc_z2x(_pd(x), _pd(z), _p64(b), len(b), x.shape[0])
    return x


def csr_matvec(A, x):
    A = sps.csr_matrix(A)
    out = np.zeros(A.shape[0])
    ip = np.ascontiguousarray(A.indptr, dtype=np.int32)
    ix = np.ascontiguousarray(A.indices, dtype=np.int32)
    lib().orc_csr_matvec(A.shape[0], _p32(ip), _p32(ix), _pd(np.ascontiguousarray(A.data)),
                         _pd(np.ascontiguousarray(x, dtype=np.float64)), _pd(out))
    return out


# ----- problem algebra (python/bsls_utils.py) --------------------------------

def particular_x0(block_sizes):
    """bsls_utils.py:327-328: 1 at the last entry of every block."""
    x0 = np.zeros(int(np.sum(block_sizes)))
    x0[np.cumsum(block_sizes) - 1] = 1
    return x0


def block_sizes_to_N(block_sizes):
    """bsls_utils.py:139-162 (+1 at (r+j, c+j), -1 at (r+j+1, c+j))."""
    rows, cols, vals = [], [], []
    r = c = 0
    for k in np.asarray(block_sizes, dtype=np.int64):
        if k >= 2:
            j = np.arange(k - 1)
            rows += [r + j, r + j + 1]
            cols += [c + j, c + j]
            vals += [np.ones(k - 1), -np.ones(k - 1)]
        r += k
        c += k - 1
    n = int(np.sum(block_sizes))
    nz = n - len(block_sizes)
    if not rows:
        return sps.csr_matrix((n, nz))
    return sps.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                          shape=(n, nz))


def x2z(x, block_sizes):
    """bsls_utils.py:267-287 (numpy cumsum per block, last entry dropped)."""
    ends = np.cumsum(block_sizes)
    starts = np.hstack(([0], ends[:-1]))
    parts = [np.cumsum(x[i:j - 1]) for i, j in zip(starts, ends) if i < j - 1]
    return np.concatenate(parts) if parts else np.zeros(0)


def lsv_operator(A, N):
    """bsls_utils.py:334-369: sqrt of the top eigenvalue of N'A'AN (ARPACK)."""
    op = sla.LinearOperator((N.shape[1], N.shape[1]),
                            matvec=lambda v: N.T.dot(A.T.dot(A.dot(N.dot(v)))),
                            dtype=A.dtype)
    ev = sla.eigs(op, k=1, tol=0, maxiter=None, ncv=10, which='LM', return_eigenvectors=False)
    return np.sqrt(ev)[0].real


# ----- solver loops ----------------------------------------------------------

def stopping(g, fx, i, t, d=None, delta_g=None, options=None, TOLER=1e-6):
    """solvers.py:40-63."""
    if options and 'max_iter' in options:
        if i >= options['max_iter']:
            return True
    if options and 'opt_tol' in options:
        TOLER = options['opt_tol']
    norm2 = np.square(la.norm(g))
    if norm2 <= TOLER * (1 + abs(fx)):
        return True
    if d is not None and la.norm(t * d) <= 1e-12:
        return True
    if delta_g is not None and la.norm(delta_g) == 0:
        return True
    return False


def bb_solve(x0, f, nabla_f, stopping_fn, record_every=500, proj=None, log=None,
             options=None):
    """BB.py:7-45 (projected Barzilai-Borwein, BB2 step)."""
    start = log(0, x0, 0)
    i, stop = 0, False
    x = x0
    x_prev = x + 1
    g_prev = nabla_f(x_prev)
    while not stop:
        i += 1
        g = nabla_f(x)
        delta_g = g - g_prev
        if sum(delta_g) == 0:        # builtin sum, as BB.py:22
            break
        delta_x = x - x_prev
        t = delta_x.dot(delta_g) / delta_g.dot(delta_g)
        x_next = x - t * g
        x_prev, x = x, x_next
        g_prev = g
        if proj:
            x = proj(x)
        fx = f(x)
        stop = stopping_fn(g, fx, i, t, delta_g=delta_g, options=options)
        if i % record_every == 0:
            start = log(i, x, time.time() - start)
    log(i, x, time.time() - start)
    return x


def solve_in_z_parts(A, b, block_sizes):
    """The closures of main.solve_in_z (main.py:47-65)."""
    A = sps.csr_matrix(A)
    block_sizes = np.asarray(block_sizes, dtype=np.int64)
    x0 = particular_x0(block_sizes)
    N = block_sizes_to_N(block_sizes)
    z0 = x2z(x0, block_sizes)
    target = A.dot(x0) - b
    AT = A.T.tocsr()
    NT = N.T.tocsr()
    f = lambda z: 0.5 * la.norm(A.dot(N.dot(z)) + target) ** 2
    nabla_f = lambda z: NT.dot(AT.dot(A.dot(N.dot(z)) + target))
    cum = np.concatenate(([0], np.cumsum(block_sizes - 1)))

    def proj(x):
        isotonic_regression_multi_c(x, cum[:-1])
        return np.maximum(np.minimum(x, 1.), 0.)
    return dict(z0=z0, x0=x0, N=N, target=target, f=f, nabla_f=nabla_f, proj=proj,
                zstarts=cum[:-1])


def bb_trace(A, b, block_sizes, iters, record_every=1, options=None):
    """Run bb_solve on main.solve_in_z's closures; return {iter: z}."""
    P = solve_in_z_parts(A, b, block_sizes)
    rec = {}

    def log(i, state, dt):
        rec[i] = np.array(state)
        return 0.0
    opts = options or {'max_iter': iters, 'verbose': 0, 'opt_tol': 1e-30}
    bb_solve(P['z0'], P['f'], P['nabla_f'], stopping, record_every=record_every,
             proj=P['proj'], log=log, options=opts)
    return rec


def weak_wolfe_ls(x, d, f, nabla_f, proj=lambda v: v, c1=1e-3, c2=0.9):
    """LBFGS.py:9-53: bisection on t until the Armijo and curvature
    conditions hold (f(proj x) and d.nabla_f(proj x) fixed, as :18-19)."""
    lo, hi, t = 0.0, float('inf'), 1
    px = proj(x)
    gx = nabla_f(px)
    while True:
        pt = proj(x + t * d)
        stop = False
        if f(pt) >= f(px) + c1 * t * d.dot(gx):
            hi = t
            t = 0.5 * (lo + hi)
        elif d.dot(nabla_f(pt)) < c2 * d.dot(gx):
            lo = t
            t = 2 * lo if hi == float('inf') else 0.5 * (lo + hi)
        else:
            stop = True
        if stop or abs(lo - hi) <= 1e-14 or la.norm(t * d) <= 1e-8:
            return t


def lbfgs_solve(x0, f, nabla_f, stopping_fn, m=50, record_every=500, proj=None, log=None,
                options=None):
    """LBFGS.solve (LBFGS.py:56-123): the two-loop recursion over the last m
    pairs (search_dir :60-71, lists of m zero pairs initially :80), the weak
    Wolfe line search, the y.s == 0 exit (:105-108)."""
    def search_dir(g_new, y_new, s_new, rho, y, s):
        q = g_new
        alpha = [0] * m
        for k in range(m - 1, -1, -1):
            alpha[k] = rho[k] * (s[k].dot(q))
            q = q - alpha[k] * y[k]
        r = (y_new.dot(s_new) / (y_new.dot(y_new))) * q
        for k in range(m):
            beta = rho[k] * y[k].dot(r)
            r = r + s[k] * (alpha[k] - beta)
        return -r

    start = log(0, x0, 0)
    i, stop = 0, False
    x = x0
    n = x.shape[0]
    y, s = [np.zeros(n)] * m, [np.zeros(n)] * m
    g_new = nabla_f(x)
    y_new, s_new = g_new, np.ones(n)
    rho, rho_new = [0] * m, 1 / (y_new.dot(s_new))
    while not stop:
        i += 1
        d = search_dir(g_new, y_new, s_new, rho, y, s)
        y = y[1:] + [y_new]
        s = s[1:] + [s_new]
        rho = rho[1:] + [rho_new]
        t = weak_wolfe_ls(x, d, f, nabla_f, proj=proj)
        s_new = t * d
        x_next = x + s_new
        if proj:
            x_next = proj(x_next)
        g = g_new
        g_new = nabla_f(x_next)
        y_new = g_new - g
        if y_new.dot(s_new) == 0:
            break
        rho_new = 1 / (y_new.dot(s_new))
        x = x_next
        fx = f(x)
        if math.isnan(fx):
            raise ArithmeticError('objective function evaluates to NaN')
        stop = stopping_fn(g_new, fx, i, t, d=d, options=options)
        if i % record_every == 0:
            start = log(i, x, time.time() - start)
    log(i, x, time.time() - start)
    return x


def lbfgs_trace(A, b, block_sizes, iters, record_every=1):
    """lbfgs_solve from GradientDescent('LBFGS')'s start (z0 + 1,
    gradient_descent.py:49) on main.solve_in_z's closures; return {iter: z}."""
    P = solve_in_z_parts(A, b, block_sizes)
    rec = {}

    def log(i, state, dt):
        rec[i] = np.array(state)
        return 0.0
    lbfgs_solve(P['z0'] + 1, P['f'], P['nabla_f'], stopping, record_every=record_every,
                proj=P['proj'], log=log,
                options={'max_iter': iters, 'verbose': 0, 'opt_tol': 1e-30})
    return rec


def batch_stopping(i, max_iter, f, f_old, opt_tol, prog_tol, f_min=None):
    """algorithm_utils.py:158-172."""
    flag, stop = False, 'continue'
    if i == max_iter:
        stop, flag = 'max_iter', True
    if f_min is not None and f - f_min < opt_tol:
        stop, flag = 'f-f_min = {} < opt_tol'.format(f - f_min), True
    if abs(f_old - f) < prog_tol:
        stop, flag = '|f_old-f| = {} < prog_tol'.format(abs(f_old - f)), True
    return flag, stop


def sparse_parts(A, b, block_starts, lasso=False):
    """get_solver_parts(data=(A, b), is_sparse=True, f=None) closures
    (algorithm_utils.py:88-94,113-137,197-203,226-231,268-271)."""
    A = sps.csr_matrix(A)
    AT = sps.csr_matrix(A.T)
    starts = np.asarray(block_starts, dtype=np.int64)

    def obj(x, g):
        tmp = A.dot(x) - b
        np.copyto(g, AT.dot(tmp))
        return .5 * tmp.T.dot(tmp)

    def proj(x):
        (proj_multi_ball_c if lasso else proj_multi_simplex_c)(x, starts)

    def line_search(x, f, g, x_new, f_new, g_new, i):
        t, suffDec, progTol = 1.0, 1e-4, 1e-12
        upper_line = f + suffDec * g.dot(x_new - x)
        while f_new > upper_line:
            t *= .8
            if la.norm(x_new - x, np.inf) < progTol:
                f_new = f
                np.copyto(g_new, g)
                np.copyto(x_new, x)
                break
            np.copyto(x_new, (1.0 - t) * x + t * x_new)
            f_new = obj(x_new, g_new)
            upper_line = f + suffDec * g.dot(x_new - x)
        return f_new
    return obj, proj, line_search


def batch_solve(obj, proj, step_size, x_init, line_search=None, f_min=None, opt_tol=1e-6,
                max_iter=2000, prog_tol=1e-12):
    """BATCH.py:7-52, projected gradient descent with an optional line search
    (progress times dropped: [k, f])."""
    n = x_init.shape[0]
    x = np.copy(x_init)
    g, g_new, x_new = np.zeros(n), np.zeros(n), np.zeros(n)
    f_old = np.inf
    i = 1
    f = obj(x, g)
    progress = [f]
    while True:
        flag, stop = batch_stopping(i, max_iter, f, f_old, opt_tol, prog_tol, f_min)
        if flag:
            break
        t = step_size(i)
        np.add(x, -t * g, x_new)
        proj(x_new)
        f_new = obj(x_new, g_new)
        if line_search is not None:
            f_new = line_search(x, f, g, x_new, f_new, g_new, i)
        f_old, f = f, f_new
        np.copyto(x, x_new)
        np.copyto(g, g_new)
        i += 1
        progress.append(f)
    return {'f': f, 'x': x, 'stop': stop, 'iterations': i, 'progress': np.array(progress)}


def batch_solve_bb(obj, proj, line_search, x_init, f_min=None, opt_tol=1e-6, max_iter=2000,
                   prog_tol=1e-12):
    """BATCH.py:55-106 (progress times dropped: [k, f])."""
    n = x_init.shape[0]
    x = np.copy(x_init)
    g = np.zeros(n)
    delta_x, delta_g = np.zeros(n), np.zeros(n)
    g_new, x_new = np.zeros(n), np.zeros(n)
    f_old = np.inf
    i = 1
    f = obj(x, g)
    progress = [f]
    while True:
        flag, stop = batch_stopping(i, max_iter, f, f_old, opt_tol, prog_tol, f_min)
        if flag:
            break
        if i == 1:
            np.add(x, -g, x_new)
        else:
            t = delta_x.T.dot(delta_g) / delta_g.T.dot(delta_g)
            np.add(x, -t * g, x_new)
        proj(x_new)
        f_new = obj(x_new, g_new)
        f_new = line_search(x, f, g, x_new, f_new, g_new, i)
        f_old, f = f, f_new
        np.add(x_new, -x, delta_x)
        np.add(g_new, -g, delta_g)
        np.copyto(x, x_new)
        np.copyto(g, g_new)
        i += 1
        progress.append(f)
    return {'f': f, 'x': x, 'stop': stop, 'iterations': i, 'progress': np.array(progress)}


def batch_solve_lbfgs(obj, proj, line_search, x_init, f_min=None, opt_tol=1e-6, max_iter=1000,
                      prog_tol=1e-12, corrections=50):
    """BATCH.py:110-193 with LBFGS_helper (:196-214), vector operations in the
    reference's order; the history queues hold the one delta_x / delta_g
    buffer (updated in place every iteration), as the reference's do."""
    from collections import deque
    q_dg, q_dx, q_rho = deque(), deque(), deque()
    n = x_init.shape[0]
    x = np.copy(x_init)
    g = np.zeros(n)
    d = np.zeros(n)
    alpha = np.zeros(corrections)
    delta_x, delta_g = np.zeros(n), np.zeros(n)
    g_new, x_new = np.zeros(n), np.zeros(n)
    f_old = np.inf
    i = 1
    f = obj(x, g)
    progress = [f]
    while True:
        flag, stop = batch_stopping(i, max_iter, f, f_old, opt_tol, prog_tol, f_min)
        if flag:
            break
        if i == 1:
            np.add(x, -g, x_new)
        else:
            q_dg.append(delta_g)
            q_dx.append(delta_x)
            q_rho.append(1 / delta_g.T.dot(delta_x))
            if i > corrections + 1:
                q_dg.popleft()
                q_dx.popleft()
                q_rho.popleft()
            if i <= 5:
                d = -(delta_x.T.dot(delta_g) / delta_g.T.dot(delta_g)) * g
            else:
                m = len(q_dg)
                np.copyto(d, g)
                for j in range(1, m + 1):
                    alpha[-j] = q_rho[-j] * q_dx[-j].T.dot(d)
                    d -= alpha[-j] * q_dg[-j]
                t = q_dx[-1].T.dot(q_dg[-1]) / q_dg[-1].T.dot(q_dg[-1])
                d *= t
                for j in range(m):
                    beta = q_rho[j] * q_dg[j].T.dot(d)
                    d += q_dx[j] * (alpha[-m + j] - beta)
                d *= -1.0
            np.add(x, d, x_new)
        proj(x_new)
        f_new = obj(x_new, g_new)
        f_new = line_search(x, f, g, x_new, f_new, g_new, i)
        f_old, f = f, f_new
        np.add(x_new, -x, delta_x)
        np.add(g_new, -g, delta_g)
        np.copyto(x, x_new)
        np.copyto(g, g_new)
        i += 1
        progress.append(f)
    return {'f': f, 'x': x, 'stop': stop, 'iterations': i, 'progress': np.array(progress)}


def batch_solve_md(obj, block_starts, step_size, x_init, f_min=None, opt_tol=1e-6,
                   max_iter=1000, prog_tol=0.0):
    """BATCH.py:217-250 with normalization (algorithm_utils.py:175-179)."""
    n = x_init.shape[0]
    starts = np.asarray(block_starts)
    ends = np.append(starts[1:], [n])
    x = np.copy(x_init)
    g, g_new, x_new = np.zeros(n), np.zeros(n), np.zeros(n)
    f_old = np.inf
    i = 1
    f = obj(x, g)
    progress = [f]
    while True:
        flag, stop = batch_stopping(i, max_iter, f, f_old, opt_tol, prog_tol, f_min)
        if flag:
            break
        t = step_size(i)
        np.copyto(x_new, x * np.exp(-t * g))
        for s_, e_ in zip(starts, ends):
            np.copyto(x_new[s_:e_], x_new[s_:e_] / np.sum(x_new[s_:e_]))
        f_new = obj(x_new, g_new)
        f_old, f = f, f_new
        np.copyto(x, x_new)
        np.copyto(g, g_new)
        i += 1
        progress.append(f)
    return {'f': f, 'x': x, 'stop': stop, 'iterations': i, 'progress': np.array(progress)}


def dore_solve(x0, linop, linop_T, target, record_every=5, proj=None, log=None,
               options=None, i=10000, eps=10 ** -16):
    """DORE.py:6-90."""
    start = log(0, x0, 0)
    if options and 'max_iter' in options:
        i = options['max_iter']
    if options and 'opt_tol' in options:
        eps = options['opt_tol']
    b = -np.array(target)
    x = np.array(x0)
    x_prev = x
    Ax = 0
    Ax_prev = 0
    iter_ = 0
    for iter_ in range(i):
        Ax_prev_prev = Ax_prev
        Ax_prev = Ax
        Ax = linop(x)
        err = b - Ax
        norm_change = la.norm(x - x_prev) ** 2
        if iter_ > 0 and norm_change <= eps:
            break
        x_new = x + linop_T(err)
        x_new = proj(x_new)
        Ax = linop(x_new)
        err = b - Ax
        x_select = x_new
        if iter_ > 2:
            delta_Ax = Ax - Ax_prev
            dp = delta_Ax.dot(delta_Ax)
            if dp > 0:
                a1 = delta_Ax.dot(err) / dp
                Ax_1 = (1 + a1) * Ax - a1 * Ax_prev
                x_1 = x_new + a1 * (x_new - x)
                err_1 = b - Ax_1
                delta_Ax = Ax_1 - Ax_prev_prev
                dp = delta_Ax.dot(delta_Ax)
                if dp > 0:
                    a2 = delta_Ax.dot(err_1) / dp
                    x_2 = x_1 + a2 * (x_1 - x_prev)
                    x_2 = proj(x_2)
                    Ax_2 = linop(x_2)
                    err_2 = b - Ax_2
                    if err_2.dot(err_2) / err.dot(err) < 1:
                        x_select = x_2
                        Ax = Ax_2
        x_prev = x
        x = x_select
        if iter_ % record_every == 0:
            start = log(iter_, x, time.time() - start)
    log(iter_, x, time.time() - start)
    return x


def dore_run(A, b, block_sizes, max_iter, record_every=100):
    """GradientDescent(method='DORE').run() (gradient_descent.py:55-67)."""
    P = solve_in_z_parts(A, b, block_sizes)
    A = sps.csr_matrix(A)
    N = P['N']
    lsv = lsv_operator(A, N)
    A_dore = A * 0.99 / lsv
    target_dore = P['target'] * 0.99 / lsv
    iters, states = [], []

    def log(i, state, dt):
        iters.append(i)
        states.append(state)
        return 0.0
    dore_solve(P['z0'], lambda z: A_dore.dot(N.dot(z)), lambda r: N.T.dot(A_dore.T.dot(r)),
               target_dore, proj=P['proj'], log=log,
               options={'max_iter': max_iter, 'verbose': 0, 'opt_tol': 1e-30},
               record_every=record_every)
    return iters, states, lsv


def md_least_squares(A, b, blocks, iters=1000, tolerance=1e-9, return_iters=False):
    """mirror_descent.py:7-53 (blocks = list of block sizes); return_iters: also
    the iteration the loop ended at (test helper)."""
    n_vector = np.concatenate([[k] * k for k in blocks]).astype(float)
    x = np.divide(1.0, n_vector)
    if sps.issparse(A):
        Lf = sla.svds(A, 1, return_singular_vectors=False)[0]
    else:
        Lf = np.linalg.svd(A, compute_uv=False)[0]

    def t_(k):
        return np.sqrt(2 * np.log(n_vector)) / (np.sqrt(k) * Lf)

    def grad(x):
        inside = np.asarray(A.dot(x)).ravel() - b
        return np.asarray(A.T.dot(inside)).ravel()
    for it in range(1, iters + 1):
        x_prev = x
        up = grad(x)
        up *= t_(it)
        x = x * np.exp(-up)
        beg = 0
        for k in blocks:
            sec = x[beg:beg + k]
            x[beg:beg + k] = sec / np.sum(sec)
            beg += k
        if np.linalg.norm(x - x_prev, np.inf) < tolerance:
            break
    return (x, it) if return_iters else x


logging.getLogger(__name__).addHandler(logging.NullHandler())
