"""Solver "parts" for the batch solvers (reference: python/algorithm_utils.py).

get_solver_parts(data, block_starts, min_eig, in_z, is_sparse, lasso, f)
returns (step_size, proj, line_search, obj) like the reference
(algorithm_utils.py:182-271), but every closure computes on the MI355X: the
vectors the batch solvers (BATCH.py) hand them are HIP-resident fp64 torch
tensors, and

  * obj, sparse   r = A x - b, g = A' r (CSR SpMV kernels, explicit A'),
                  f = 0.5 r.r                       (algorithm_utils.py:88-94)
  * obj, dense    g = Q x + c, f = 0.5 x.(g + c)    (bsls_quad_obj; :79-85)
  * proj, x       proj_multi_simplex / proj_multi_ball kernels (:226-231)
  * proj, z       PAVA v1 kernel + clip to [0, 1] (:215-224; the reference
                  calls sklearn's IsotonicRegression there, which equals PAVA
                  up to the last bits)
  * the f= variants divide each block by its flow before projecting and
    multiply back after (:233-265), fused into one kernel pass each.

obj is a SparseLSQ / DenseQP object, proj a BlockProj and line_search carries
`.obj`, so BATCH.solve_BB can recognise the sparse x-space case and hand the
whole loop to the fused device engine (device.XBBEngine, csrc/xbb.hip).
"""
import os

import numpy as np
import scipy.sparse as sps

import _native
from _native import check, ptr, stream_handle


def _torch():
    import torch
    return torch


def _dev(a):
    """fp64 HIP tensor view/copy of a NumPy array or tensor."""
    torch = _torch()
    if isinstance(a, torch.Tensor):
        return a.to(device='cuda', dtype=torch.float64).contiguous()
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()


def _starts_dev(block_starts):
    torch = _torch()
    return torch.from_numpy(np.ascontiguousarray(block_starts, dtype=np.int64)).cuda()


def _check_starts(blocks, n):
    """The Cython wrapper's asserts (c_extensions.pyx:33-34)."""
    b = np.asarray(blocks)
    assert False not in ((b[1:] - b[:-1]) > 0), 'block indices not increasing'
    assert b[0] >= 0 and b[-1] < n, 'indices out of range'


# -- projections on the device ------------------------------------------------

class BlockProj:
    """proj_multi_simplex_c / proj_multi_ball_c / PAVA+clip on a device vector,
    in place (the reference's proj closures mutate x and return None)."""

    def __init__(self, block_starts, n, kind='simplex', flows=None):
        torch = _torch()
        L = _native.lib()
        st = np.ascontiguousarray(block_starts, dtype=np.int64)
        _check_starts(st, n)
        self.kind, self.n, self.p = kind, int(n), int(st.shape[0])
        self.starts = _starts_dev(st)
        ends = np.append(st[1:], n)
        self.max_block = int(np.max(ends - st))
        if kind == 'pava':
            self.ws = torch.zeros(L.bsls_isotonic_workspace_size(self.n), dtype=torch.uint8,
                                  device='cuda')
        else:
            self.ws = torch.zeros(L.bsls_proj_workspace_size(self.n, self.p, self.max_block),
                                  dtype=torch.uint8, device='cuda')
        self.flows = None
        if flows is not None:
            fl = np.asarray(flows, dtype=np.float64)
            if fl.shape[0] != self.p:
                raise ValueError('one flow per block expected')
            scale = np.ones(self.n)
            scale[st[0]:] = np.repeat(fl, ends - st)
            self.flows = _dev(scale)

    def __call__(self, x):
        torch = _torch()
        L = _native.lib()
        if self.flows is not None:
            # np.copyto(x[i:j], x[i:j] / k) per block  (algorithm_utils.py:236-237)
            torch.div(x, self.flows, out=x)
        if self.kind == 'simplex':
            check(L.bsls_proj_multi_simplex(ptr(x), ptr(self.starts), self.p, self.n,
                                            self.max_block, ptr(self.ws), self.ws.numel(),
                                            stream_handle()), 'bsls_proj_multi_simplex')
        elif self.kind == 'ball':
            check(L.bsls_proj_multi_ball(ptr(x), ptr(self.starts), self.p, self.n,
                                         self.max_block, ptr(self.ws), self.ws.numel(),
                                         stream_handle()), 'bsls_proj_multi_ball')
        else:
            check(L.bsls_isotonic_multi(1, ptr(x), ptr(self.starts), self.p, self.n, None, 1,
                                        self.max_block, ptr(self.ws), self.ws.numel(), None,
                                        stream_handle()), 'bsls_isotonic_multi')
            torch.clamp(x, 0.0, 1.0, out=x)     # np.maximum(0.,x,x); np.minimum(1.,x,x)
        if self.flows is not None:
            torch.mul(x, self.flows, out=x)


def proj_simplex(y, start, end):
    """Projects y[start:end] onto the simplex, in place (algorithm_utils.py:63-69)."""
    assert start >= 0 and start < len(y) and end > 0 and end <= len(y)
    if start >= end:
        return
    from c_extensions.c_extensions import proj_simplex_c
    proj_simplex_c(y, start, end)


def proj_multi_simplex(y, blocks):
    """algorithm_utils.py:72-76 (same asserts), on the device kernel."""
    from c_extensions.c_extensions import proj_multi_simplex_c
    blocks = np.asarray(blocks)
    _check_starts(blocks, len(y))
    proj_multi_simplex_c(y, blocks.astype(np.int64))


# -- objectives -----------------------------------------------------------------

class SparseLSQ:
    """sparse_least_squares_obj (algorithm_utils.py:88-94) over device CSR:
    tmp = A x - b; g = A' tmp; f = .5 tmp.tmp.

    `panels`: also build the images of device.DeviceLSQ (csrc/lsq.hip) and run
    both products on them -- the default from PANEL_MIN_NNZ nonzeros up: the
    residual on a dealt tile image of A with two-word fixed-point row sums
    (k1='tiles_fixed': order-free, so f repeats bit for bit at the same x, as
    the solvers' revert exit needs; BSLS_LSQ_K1=panels keeps the fixed-order
    panel walk), the gradient on the A' panels (bit-identical to SciPy).
    tmp differs from SciPy's row order by <= 1e-12 relative."""

    PANEL_MIN_NNZ = 1 << 20

    def __init__(self, A, b, A_T=None, panels=None):
        from device import DeviceCSR, lsq_operator
        torch = _torch()
        A = sps.csr_matrix(A)
        self.A_host = A
        self.m, self.n = A.shape
        AT = sps.csr_matrix(A_T) if A_T is not None else A.T.tocsr()
        self.A = DeviceCSR(A)
        self.AT = DeviceCSR(AT)
        if panels is None:
            panels = A.nnz >= self.PANEL_MIN_NNZ
        self.lsq = (lsq_operator(A, AT, k1=os.environ.get('BSLS_LSQ_K1', 'tiles_fixed'))
                    if panels else None)
        self.b = _dev(np.asarray(b, dtype=np.float64).ravel())
        self.neg_b = -self.b
        self.tmp = torch.empty(self.m, dtype=torch.float64, device='cuda')

    def __call__(self, x, g=None):
        torch = _torch()
        gd = g if isinstance(g, torch.Tensor) else torch.empty(self.n, dtype=torch.float64,
                                                                 device='cuda')
        if self.lsq is not None:
            sq = torch.zeros(1, dtype=torch.float64, device='cuda')
            self.lsq.residual(_dev(x), self.tmp, add=self.neg_b, sq=sq)
            self.lsq.gradient(self.tmp, gd)
        else:
            _, sq = self.A.matvec(_dev(x), out=self.tmp, add=self.neg_b, want_sq=True)
            self.AT.matvec(self.tmp, out=gd)
        if g is not None and gd is not g:
            np.copyto(g, gd.cpu().numpy())      # a NumPy g is written in place, as np.copyto
        return .5 * float(sq.item())


class DenseQP:
    """quad_obj_np (algorithm_utils.py:79-85): g = Q x + c, f = .5 x.(g + c),
    on the device (bsls_quad_obj, quadratic_objective.h:15-26)."""

    def __init__(self, Q, c):
        torch = _torch()
        self.Q = _dev(np.asarray(Q, dtype=np.float64))
        self.c = _dev(np.asarray(c, dtype=np.float64).ravel())
        self.n = int(self.c.shape[0])
        self.f = torch.zeros(1, dtype=torch.float64, device='cuda')

    def __call__(self, x, g=None):
        torch = _torch()
        gd = g if isinstance(g, torch.Tensor) else torch.empty(self.n, dtype=torch.float64,
                                                                 device='cuda')
        xd = _dev(x)
        check(_native.lib().bsls_quad_obj(ptr(xd), ptr(self.Q), ptr(self.c), ptr(gd), self.n,
                                          ptr(self.f), stream_handle()), 'bsls_quad_obj')
        if g is not None and gd is not g:
            np.copyto(g, gd.cpu().numpy())
        return float(self.f.item())


def quad_obj_np(x, Q, c, g=None):
    return DenseQP(Q, c)(_dev(x), g)


def sparse_least_squares_obj(x, A_sparse_T, A_sparse, b, g):
    """algorithm_utils.py:88-94 (one-off call: builds the device operator)."""
    return SparseLSQ(A_sparse, b, A_T=A_sparse_T)(_dev(x), g)


# -- step sizes, line search, stopping --------------------------------------------

def decreasing_step_size(i, t0, alpha):
    """t = t0 / (alpha i + t0)  (algorithm_utils.py:97-100)."""
    return t0 / (alpha * i + t0)


def line_search_np(x, f, g, x_new, f_new, g_new, obj):
    """Backtracking line search (algorithm_utils.py:113-137): x_new / g_new are
    updated in place on the device; the reference's compounding t (t *= .8 on
    an already shrunk x_new) is kept."""
    t = 1.0
    suffDec = 1e-4
    progTol = 1e-12
    upper_line = f + suffDec * float(g.dot(x_new - x))
    while f_new > upper_line:
        t *= .8
        step = float((x_new - x).abs().max())
        if step < progTol:
            t = 0.0
            f_new = f
            g_new.copy_(g)
            x_new.copy_(x)
            break
        x_new.copy_((1.0 - t) * x + t * x_new)
        f_new = obj(x_new, g_new)
        upper_line = f + suffDec * float(g.dot(x_new - x))
    return f_new


def line_search_exact_quad_obj(x, f, g, x_new, f_new, g_new, Q, c):
    """Exact line search for a quadratic (algorithm_utils.py:140-155)."""
    progTol = 1e-8
    Qd, cd = _dev(Q), _dev(c)
    d = x_new - x
    if float(d.abs().max()) < progTol:
        g_new.copy_(g)
        x_new.copy_(x)
        return f
    tmp = Qd.matmul(d)
    t = -(float(x.dot(tmp)) + float(d.dot(cd))) / float(d.dot(tmp))
    x_new.copy_(x + t * d)
    return DenseQP(Qd, cd)(x_new, g_new)


def stopping(i, max_iter, f, f_old, opt_tol, prog_tol, f_min=None):
    """algorithm_utils.py:158-172 (host scalars)."""
    flag = False
    stop = 'continue'
    if i == max_iter:
        stop = 'max_iter'
        flag = True
    if f_min is not None and f - f_min < opt_tol:
        stop = 'f-f_min = {} < opt_tol'.format(f - f_min)
        flag = True
    if abs(f_old - f) < prog_tol:
        stop = '|f_old-f| = {} < prog_tol'.format(abs(f_old - f))
        flag = True
    return flag, stop


def normalization(x, block_starts, block_ends):
    """Each block divided by its sum, in place (algorithm_utils.py:175-179).
    Contiguous blocks (block_ends[k] == block_starts[k+1]) run as one
    bsls_md_step launch; any other layout block by block."""
    starts = np.asarray(block_starts, dtype=np.int64)
    ends = np.asarray(block_ends, dtype=np.int64)
    xd = x if hasattr(x, 'data_ptr') else None
    if xd is None:
        raise TypeError('normalization works on device tensors (BATCH.py passes them)')
    L = _native.lib()
    if np.array_equal(ends[:-1], starts[1:]) and ends[-1] == xd.shape[0]:
        check(L.bsls_md_step(ptr(xd), None, ptr(xd), ptr(_starts_dev(starts)), starts.shape[0],
                             xd.shape[0], 0.0, stream_handle()), 'bsls_md_step')
        return
    for s, e in zip(starts, ends):
        seg = xd[s:e]
        one = _starts_dev(np.zeros(1, dtype=np.int64))
        check(L.bsls_md_step(ptr(seg), None, ptr(seg), ptr(one), 1, int(e - s), 0.0,
                             stream_handle()), 'bsls_md_step')


# -- the parts factory ------------------------------------------------------------

def get_solver_parts(data, block_starts, min_eig, in_z=False, is_sparse=False, lasso=False,
                     f=None):
    """Returns (step_size, proj, line_search, obj) -- algorithm_utils.py:182-271."""
    block_starts = np.asarray(block_starts, dtype=np.int64)
    if is_sparse:
        A, b = data
        obj = SparseLSQ(A, b)
        n = obj.n
    else:
        Q, c = data
        obj = DenseQP(Q, c)
        n = obj.n

    def step_size(i):
        return decreasing_step_size(i, 1.0, min_eig)

    if in_z:
        tmp = np.copy(block_starts)
        if not lasso:
            tmp = tmp - np.arange(len(tmp))
        kind = 'pava'
        starts = tmp
    else:
        kind = 'ball' if lasso else 'simplex'
        starts = block_starts
    proj = BlockProj(starts, n, kind, flows=f)
    proj.lasso, proj.in_z = lasso, in_z

    def line_search(x, f_, g, x_new, f_new, g_new, i):
        return line_search_np(x, f_, g, x_new, f_new, g_new, obj)
    line_search.obj = obj
    return step_size, proj, line_search, obj
