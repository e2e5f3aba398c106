"""Projected limited-memory BFGS with a bisection weak-Wolfe line search
(reference: python/LBFGS.py:9-123).  Off the north-star hot path; kept so that
GradientDescent(method='LBFGS') dispatches.  Works on NumPy arrays or on
HIP-resident torch tensors through the device closures."""
import math
import time

from _arr import copy, dot, norm


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
    Y, S, rho = [zero] * m, [zero] * m, [0.0] * m
    g_new = nabla_f(x)
    y_new, s_new = g_new, zero + 1
    rho_new = 1 / dot(y_new, s_new)
    while not stop:
        i += 1
        d = direction(g_new, y_new, s_new, rho, Y, S)
        Y = Y[1:] + [y_new]
        S = S[1:] + [s_new]
        rho = rho[1:] + [rho_new]
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
        stop = stopping(g_new, fx, i, t, d=d, options=options)
        if i % record_every == 0:
            start = log(i, copy(x), time.time() - start)
    log(i, x, time.time() - start)
    return x
