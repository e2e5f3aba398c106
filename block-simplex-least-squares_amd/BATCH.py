"""Allocation-free batch solvers (reference: python/BATCH.py).

Same signatures, loops, stopping rules and return dicts as the reference
(solve :7-52, solve_BB :55-106, solve_LBFGS :110-193, LBFGS_helper :196-214,
solve_MD :217-250).  Every vector lives on the MI355X as an fp64 torch tensor;
the closures come from algorithm_utils.get_solver_parts and launch the HIP
kernels.  `x_init` may be a NumPy array (as the reference's callers pass); the
result dict holds `x` as a NumPy array, like the reference.

solve_BB and solve_LBFGS on a sparse least-squares objective with a block
projection (get_solver_parts(..., is_sparse=True)) run by default on the fused
device engine (device.XBBEngine: one stage per quantity, the line search and
the stopping test on the device, no host round trip per iteration); pass
fused=False for the closure-by-closure loops below.
"""
import time
from collections import deque

import numpy as np

from algorithm_utils import stopping


def _torch():
    import torch
    return torch


def _to_dev(x):
    torch = _torch()
    if isinstance(x, torch.Tensor):
        return x.to(device='cuda', dtype=torch.float64).clone()
    return torch.from_numpy(np.array(x, dtype=np.float64)).cuda()


def _zeros(n):
    torch = _torch()
    return torch.zeros(n, dtype=torch.float64, device='cuda')


def _axpy(x, t, g, out, scratch):
    """np.add(x, -t*g, out): the scaled vector is rounded first, then added."""
    torch = _torch()
    torch.mul(g, -t, out=scratch)
    torch.add(x, scratch, out=out)


def _result(f, x, stop, i, progress):
    return {'f': f, 'x': x.cpu().numpy(), 'stop': stop, 'iterations': i,
            'progress': progress}


def solve(obj, proj, step_size, x_init, line_search=None, f_min=None, opt_tol=1e-6,
          max_iter=2000, prog_tol=1e-12):
    """Projected batch gradient descent with line search (BATCH.py:7-52)."""
    n = x_init.shape[0]
    x = _to_dev(x_init)
    g = _zeros(n)
    g_new = _zeros(n)
    x_new = _zeros(n)
    tmp = _zeros(n)
    f_old = np.inf
    i = 1
    f = obj(x, g)
    progress = [[0.0, f]]
    start_time = time.time()
    while True:
        flag, stop = stopping(i, max_iter, f, f_old, opt_tol, prog_tol, f_min)
        if flag is True:
            break
        t = step_size(i)
        _axpy(x, t, g, x_new, tmp)
        proj(x_new)
        f_new = obj(x_new, g_new)
        if line_search is not None:
            f_new = line_search(x, f, g, x_new, f_new, g_new, i)
        f_old = f
        f = f_new
        x.copy_(x_new)
        g.copy_(g_new)
        i += 1
        progress.append([time.time() - start_time, f])
    return _result(f, x, stop, i, progress)


def _fusable(obj, proj, line_search):
    from algorithm_utils import SparseLSQ, BlockProj
    return (isinstance(obj, SparseLSQ) and isinstance(proj, BlockProj)
            and proj.kind in ('simplex', 'ball') and proj.flows is None
            and getattr(line_search, 'obj', None) is obj)


def solve_BB(obj, proj, line_search, x_init, f_min=None, opt_tol=1e-6, max_iter=2000,
             prog_tol=1e-12, fused=True):
    """Projected batch gradient descent with Barzilai-Borwein step (BATCH.py:55-106)."""
    if fused and _fusable(obj, proj, line_search):
        from device import XBBEngine
        eng = XBBEngine(obj, proj)
        return eng.solve(x_init, f_min=f_min, opt_tol=opt_tol, max_iter=max_iter,
                         prog_tol=prog_tol)
    n = x_init.shape[0]
    x = _to_dev(x_init)
    g = _zeros(n)
    delta_x = _zeros(n)
    delta_g = _zeros(n)
    g_new = _zeros(n)
    x_new = _zeros(n)
    tmp = _zeros(n)
    f_old = np.inf
    i = 1
    f = obj(x, g)
    progress = [[0.0, f]]
    start_time = time.time()
    while True:
        flag, stop = stopping(i, max_iter, f, f_old, opt_tol, prog_tol, f_min)
        if flag is True:
            break
        if i == 1:
            _axpy(x, 1.0, g, x_new, tmp)          # np.add(x, -g, x_new)
        else:
            t = float(delta_x.dot(delta_g)) / float(delta_g.dot(delta_g))
            _axpy(x, t, g, x_new, tmp)
        proj(x_new)
        f_new = obj(x_new, g_new)
        f_new = line_search(x, f, g, x_new, f_new, g_new, i)
        f_old = f
        f = f_new
        _torch().sub(x_new, x, out=delta_x)
        _torch().sub(g_new, g, out=delta_g)
        x.copy_(x_new)
        g.copy_(g_new)
        i += 1
        progress.append([time.time() - start_time, f])
    return _result(f, x, stop, i, progress)


def solve_LBFGS(obj, proj, line_search, x_init, f_min=None, opt_tol=1e-6, max_iter=1000,
                prog_tol=1e-12, corrections=50, fused=True):
    """Projected L-BFGS (BATCH.py:110-193).  As in the reference, the history
    queues hold the one delta_x / delta_g buffer that every iteration
    overwrites in place, so all stored corrections alias the latest one.
    On a sparse least-squares objective with a block projection it runs on the
    fused device engine (device.XBBEngine(lbfgs=corrections): the BB rounds
    with LBFGS_helper's recursion in place of the BB step from iteration 6,
    every decision on the device); fused=False runs the loop below."""
    if fused and _fusable(obj, proj, line_search) and int(corrections) > 0:
        from device import XBBEngine
        eng = XBBEngine(obj, proj, lbfgs=int(corrections))
        return eng.solve(x_init, f_min=f_min, opt_tol=opt_tol, max_iter=max_iter,
                         prog_tol=prog_tol)
    torch = _torch()
    q_delta_g = deque()
    q_delta_x = deque()
    q_rho = deque()
    n = x_init.shape[0]
    x = _to_dev(x_init)
    g = _zeros(n)
    d = _zeros(n)
    alpha = np.zeros(corrections)
    delta_x = _zeros(n)
    delta_g = _zeros(n)
    g_new = _zeros(n)
    x_new = _zeros(n)
    tmp = _zeros(n)
    f_old = np.inf
    i = 1
    f = obj(x, g)
    progress = [[0.0, f]]
    time_direction = 0
    time_line_search = 0
    time_proj = 0
    start_time = time.time()
    while True:
        flag, stop = stopping(i, max_iter, f, f_old, opt_tol, prog_tol, f_min)
        if flag is True:
            break
        start_time_2 = time.time()
        if i == 1:
            _axpy(x, 1.0, g, x_new, tmp)
        else:
            q_delta_g.append(delta_g)
            q_delta_x.append(delta_x)
            q_rho.append(1 / float(delta_g.dot(delta_x)))
            if i > corrections + 1:
                q_delta_g.popleft()
                q_delta_x.popleft()
                q_rho.popleft()
            if i <= 5:
                t = float(delta_x.dot(delta_g)) / float(delta_g.dot(delta_g))
                torch.mul(g, -t, out=d)
            else:
                LBFGS_helper(q_delta_g, q_delta_x, q_rho, g, d, alpha)
            torch.add(x, d, out=x_new)
        time_direction = time.time() - start_time_2
        start_time_2 = time.time()
        proj(x_new)
        time_proj += time.time() - start_time_2
        start_time_2 = time.time()
        f_new = obj(x_new, g_new)
        f_new = line_search(x, f, g, x_new, f_new, g_new, i)
        time_line_search += time.time() - start_time_2
        f_old = f
        f = f_new
        torch.sub(x_new, x, out=delta_x)
        torch.sub(g_new, g, out=delta_g)
        x.copy_(x_new)
        g.copy_(g_new)
        i += 1
        progress.append([time.time() - start_time, f])
    print('time_proj', time_proj)
    print('time_direction', time_direction)
    print('time_line_search', time_line_search)
    return _result(f, x, stop, i, progress)


def LBFGS_helper(q_delta_g, q_delta_x, q_rho, g, d, alpha):
    """Two-loop recursion (BATCH.py:196-214), in place on d."""
    m = len(q_delta_g)
    d.copy_(g)
    for j in range(1, m + 1):
        alpha[-j] = q_rho[-j] * float(q_delta_x[-j].dot(d))
        d.sub_(alpha[-j] * q_delta_g[-j])
    t = float(q_delta_x[-1].dot(q_delta_g[-1])) / float(q_delta_g[-1].dot(q_delta_g[-1]))
    d.mul_(t)
    for j in range(m):
        beta = q_rho[j] * float(q_delta_g[j].dot(d))
        d.add_(q_delta_x[j] * (alpha[-m + j] - beta))
    d.mul_(-1.0)


def solve_MD(obj, block_starts, step_size, x_init, line_search=None, f_min=None, opt_tol=1e-6,
             max_iter=1000, prog_tol=0.0):
    """Entropic mirror descent (BATCH.py:217-250): x <- x exp(-t g), then every
    block normalised -- one fused kernel (bsls_md_step)."""
    import _native
    from _native import check, ptr, stream_handle
    L = _native.lib()
    n = x_init.shape[0]
    starts = np.asarray(block_starts, dtype=np.int64)
    st_dev = _torch().from_numpy(starts.copy()).cuda()
    x = _to_dev(x_init)
    g = _zeros(n)
    g_new = _zeros(n)
    x_new = _zeros(n)
    f_old = np.inf
    i = 1
    f = obj(x, g)
    progress = [[0.0, f]]
    start_time = time.time()
    while True:
        flag, stop = stopping(i, max_iter, f, f_old, opt_tol, prog_tol, f_min)
        if flag is True:
            break
        t = step_size(i)
        # np.copyto(x_new, x * np.exp(-t*g)); normalize(x_new): blocks are
        # [starts[k], starts[k+1]) and the last ends at n, so one launch
        check(L.bsls_md_step(ptr(x), ptr(g), ptr(x_new), ptr(st_dev), starts.shape[0], n,
                             float(t), stream_handle()), 'bsls_md_step')
        f_new = obj(x_new, g_new)
        f_old = f
        f = f_new
        x.copy_(x_new)
        g.copy_(g_new)
        i += 1
        progress.append([time.time() - start_time, f])
    return _result(f, x, stop, i, progress)
