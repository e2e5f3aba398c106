"""Projected limited-memory BFGS with a bisection weak-Wolfe line search
(reference: python/LBFGS.py:9-123).  Off the north-star hot path; kept so that
GradientDescent(method='LBFGS') dispatches.  Works on NumPy arrays or on
HIP-resident torch tensors through the device closures.

On the device the search direction (LBFGS.py:59-71) and the history rotation
(:75-77) run on csrc/lbfgs.hip (_DeviceHistory): the m pairs live in a ring of
device slots with their Gram matrices, and one direction is one multi-dot pass,
one one-wave recursion on the dots and one combine pass -- instead of 2m
dependent dot products (each a device -> host read) and 2m AXPYs.  When the
closures are a device.BBEngine's, the weak Wolfe line search (LBFGS.py:9-53)
runs on the device too (device.LineSearch: every trial's projection, f, and
when Armijo holds the gradient and the curvature test, decided by gated
kernels; the host reads the state once per chunk of trials), and the rest of
an iteration -- s, y, y.s, the stopping rule's norms -- costs one more read.
BSLS_LBFGS_LS=host keeps the line search's decisions on the host (the
reference's structure) for A/B."""
import ctypes
import math
import os
import time

from _arr import Normed, copy, dot, is_torch, norm

MAX_DEVICE_CORRECTIONS = 127     # bsls_lbfgs_coef


class _DeviceHistory:
    """The reference's lists Y, S, rho (m zero pairs initially, LBFGS.py:51)
    as a ring of device slots: slot (head + k) % m = pair k (0 the oldest)."""

    def __init__(self, x, m):
        import torch
        import _native
        self.L, self.torch, self.native = _native.lib(), torch, _native
        self.m, self.n, self.head = m, x.numel(), 0
        dev, f64 = x.device, torch.float64
        self.S = torch.zeros((m, self.n), dtype=f64, device=dev)
        self.Y = torch.zeros((m, self.n), dtype=f64, device=dev)
        self.g = torch.empty(self.n, dtype=f64, device=dev)
        self.yn = torch.empty_like(self.g)
        self.sn = torch.empty_like(self.g)
        self.state = torch.zeros(self.L.bsls_lbfgs_state_size(m) // 8, dtype=f64, device=dev)
        self.K = 2 * m + 2
        self.dots = torch.empty(3 * self.K, dtype=f64, device=dev)
        wb = self.L.bsls_multi_dot_workspace_size(3, self.K)
        self.work = torch.empty((wb + 7) // 8, dtype=f64, device=dev)
        self.wbytes = self.work.numel() * 8
        S, Y = [r.data_ptr() for r in self.S], [r.data_ptr() for r in self.Y]
        ptrs = lambda v: torch.tensor(v, dtype=torch.int64).to(dev)
        self.rows = ptrs([self.g.data_ptr(), self.yn.data_ptr(), self.sn.data_ptr()])
        self.cols = ptrs(S + Y + [self.yn.data_ptr(), self.sn.data_ptr()])
        self.vecs = ptrs([self.g.data_ptr()] + S + Y)
        coef_off = m + 2 * m * m                       # bsls_lbfgs_state_size's layout
        self.coef = self.state[coef_off:coef_off + 2 * m + 1]

    def direction(self, g_new, y_new, s_new):
        """-r of LBFGS.py:59-71 (no host read)."""
        P, ck, L = self.native.ptr, self.native.check, self.L
        st = self.native.stream_handle()
        for buf, v in ((self.g, g_new), (self.yn, y_new), (self.sn, s_new)):
            if v is not buf:       # (the device line search writes y, s in place)
                buf.copy_(v.reshape(-1))
        ck(L.bsls_multi_dot(P(self.rows), 3, P(self.cols), self.K, self.n, P(self.dots),
                            P(self.work), self.wbytes, st), 'bsls_multi_dot')
        ck(L.bsls_lbfgs_coef(self.m, self.head, P(self.state), P(self.dots), st), 'bsls_lbfgs_coef')
        d = self.torch.empty_like(self.g)
        ck(L.bsls_multi_axpy(P(self.vecs), 2 * self.m + 1, P(self.coef), self.n, P(d), st),
           'bsls_multi_axpy')
        return d.reshape(g_new.shape)

    def push(self, rho_new):
        """Y = Y[1:] + [y_new] etc. (LBFGS.py:75-77): the oldest slot takes the
        pair of the last direction() call, its Gram rows from the same dots."""
        P, L = self.native.ptr, self.L
        st = self.native.stream_handle()
        h = self.head
        self.native.check(L.bsls_lbfgs_push(self.m, h, ctypes.c_double(rho_new), P(self.state),
                                            P(self.dots), P(self.yn), P(self.sn), P(self.Y[h]),
                                            P(self.S[h]), self.n, st), 'bsls_lbfgs_push')
        self.head = (h + 1) % self.m


def weak_wolfe_ls(x, d, f, nabla_f, proj=lambda v: v, c1=1e-3, c2=0.9):
    """Bisection on t until Armijo (sufficient decrease) and curvature hold
    (LBFGS.py:9-53).  Returns t."""
    lo, hi = 0.0, float('inf')
    t = 1.0
    px = proj(x)
    gx = nabla_f(px)
    fx = f(px)
    slope = dot(d, gx)
    while True:
        pt = proj(x + t * d)
        if f(pt) >= fx + c1 * t * slope:          # Armijo violated
            hi = t
            t = 0.5 * (lo + hi)
        elif dot(d, nabla_f(pt)) < c2 * slope:     # curvature violated
            lo = t
            t = 2 * lo if hi == float('inf') else 0.5 * (lo + hi)
        else:
            return t
        if abs(lo - hi) <= 1e-14 or norm(t * d) <= 1e-8:
            return t


def _host_floats(*vals):
    """Device scalars to host floats in one read."""
    import torch
    return [float(v) for v in torch.stack(list(vals)).cpu()]


def _device_engine(f, nabla_f, proj, x):
    """The BBEngine whose closures f / nabla_f / proj these are (x on its
    device), or None -- then the line search runs over the closures."""
    eng = getattr(f, '__self__', None)
    if (eng is None or not hasattr(eng, 'line_search') or proj is None
            or getattr(nabla_f, '__self__', None) is not eng
            or getattr(proj, '__self__', None) is not eng):
        return None
    if not (is_torch(x) and x.is_cuda and x.dim() == 1 and x.numel() == eng.nz):
        return None
    if os.environ.get('BSLS_LBFGS_LS', 'device') == 'host':
        return None
    return eng


def solve(x0, f, nabla_f, stopping, m=50, record_every=500, proj=None, log=None, options=None):
    def direction(g_new, y_new, s_new, rho, Y, S):
        q = g_new
        alpha = [0.0] * len(Y)
        for k in range(len(Y) - 1, -1, -1):
            alpha[k] = rho[k] * dot(S[k], q)
            q = q - alpha[k] * Y[k]
        r = (dot(y_new, s_new) / dot(y_new, y_new)) * q
        for k in range(len(Y)):
            beta = rho[k] * dot(Y[k], r)
            r = r + S[k] * (alpha[k] - beta)
        return -r

    start = log(0, x0, 0)
    i, stop = 0, False
    x = x0
    zero = x * 0
    hist = None
    if is_torch(x) and x.is_cuda and 1 <= m <= MAX_DEVICE_CORRECTIONS:
        hist = _DeviceHistory(x, m)
    else:
        Y, S, rho = [zero] * m, [zero] * m, [0.0] * m
    g_new = nabla_f(x)
    y_new, s_new = g_new, zero + 1
    rho_new = 1 / dot(y_new, s_new)
    eng = _device_engine(f, nabla_f, proj, x)
    ls = eng.line_search() if eng is not None else None
    import solvers
    normed_ok = stopping is solvers.stopping
    fx_dev = None          # f(x) on the device once x is a projected point
    while not stop:
        i += 1
        if hist is not None:
            d = hist.direction(g_new, y_new, s_new)
            hist.push(rho_new)
        else:
            d = direction(g_new, y_new, s_new, rho, Y, S)
            Y = Y[1:] + [y_new]
            S = S[1:] + [s_new]
            rho = rho[1:] + [rho_new]
        if ls is not None:
            # the search's proj(x), nabla_f(proj(x)), f(proj(x)) (LBFGS.py:18-20):
            # after the first iteration x is the last x_next (projected) and
            # g_new = nabla_f(x), f(x) already on the device; the first
            # iteration's x0 is not projected, so they are formed here once
            # (the trials project x + t d themselves).  On the accepted exit
            # the search's one read per chunk also brings f(x_next), y.s and
            # g.g, and y / s land in the history's buffers -- except on the
            # first iteration, whose y = g(x_next) - nabla_f(x0) is not the
            # search's g(x_next) - nabla_f(proj(x0)).
            first = fx_dev is None
            if first:
                px = proj(x)
                gx = nabla_f(px)
                fx_dev = px.new_tensor([f(px)])
            else:
                gx = g_new
            yb = hist.yn if (hist is not None and not first) else None
            sb = hist.sn if (hist is not None and not first) else None
            t, why, _, dnorm = ls.search(x, d, gx, fx_dev, y_out=yb, s_out=sb)
            g = g_new
            if why == 1 and ls.last is not None:     # accepted: the last trial is x_next
                x_next, g_new, fx_dev = ls.take()
                fx, ys, gg = ls.last
                if yb is not None:
                    y_new, s_new = hist.yn, hist.sn
                else:
                    s_new = t * d
                    y_new = g_new - g
                    if first:
                        ys, gg = _host_floats(y_new.dot(s_new), g_new.dot(g_new))
            else:              # t was never evaluated (the two other exits)
                s_new = t * d
                x_next = proj(x + s_new)
                g_new = nabla_f(x_next)
                y_new = g_new - g
                vals = _host_floats(y_new.dot(s_new), g_new.dot(g_new))
                ys, gg = vals[0], vals[1]
                fx = f(x_next)
                fx_dev = g_new.new_tensor([fx])
            if ys == 0:
                print('iter=%d, f=%8.5e' % (i, fx))
                print('Exiting... no change in gradient')
                break
            rho_new = 1 / ys
            x = x_next
            if math.isnan(fx):
                raise ArithmeticError('objective function evaluates to NaN')
            if normed_ok:
                # solvers.stopping only takes norms and t * d: the norms the
                # search already read, no device round trip
                stop = stopping(Normed(g_new, math.sqrt(gg)), fx, i, t, d=Normed(d, dnorm),
                                options=options)
            else:
                # any other rule gets the vectors themselves
                stop = stopping(g_new, fx, i, t, d=d, options=options)
            if i % record_every == 0:
                start = log(i, copy(x), time.time() - start)
            continue
        t = weak_wolfe_ls(x, d, f, nabla_f, proj=proj or (lambda v: v))
        s_new = t * d
        x_next = x + s_new
        if proj:
            x_next = proj(x_next)
        g = g_new
        g_new = nabla_f(x_next)
        y_new = g_new - g
        ys = dot(y_new, s_new)
        if ys == 0:
            print('iter=%d, f=%8.5e' % (i, f(x_next)))
            print('Exiting... no change in gradient')
            break
        rho_new = 1 / ys
        x = x_next
        fx = f(x)
        if math.isnan(fx):
            raise ArithmeticError('objective function evaluates to NaN')
        if ls is not None:
            fx_dev = x.new_tensor([fx])      # x is proj(x + s): the device search can take over
        stop = stopping(g_new, fx, i, t, d=d, options=options)
        if i % record_every == 0:
            start = log(i, copy(x), time.time() - start)
    log(i, x, time.time() - start)
    return x
