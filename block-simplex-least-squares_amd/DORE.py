"""DORE: projected Landweber step + two residual extrapolations
(reference: python/DORE.py:6-90).

Same signature and control flow; linop / linop_T / proj are the device
closures built by gradient_descent (fused SpMV + N / N' on the GPU), and the
vectors are HIP-resident torch tensors.  The scalar branch decisions
(dp > 0, ||err_2||^2 / ||err||^2 < 1) are made on the host, as in the
reference, one small device->host read per decision.
"""
import logging
import time

from _arr import copy, dot, norm


def solve(x0, linop, linop_T, target, record_every=5, proj=None, log=None, options=None,
          i=10000, eps=10 ** -16):
    start = log(0, x0, 0)
    if options and 'max_iter' in options:
        i = options['max_iter']
    if options and 'opt_tol' in options:
        eps = options['opt_tol']
    b = -copy(target)
    x = copy(x0)
    x_prev = x
    Ax = 0
    Ax_prev = 0
    iter_ = 0
    err = None
    for iter_ in range(i):
        Ax_prev_prev = Ax_prev
        Ax_prev = Ax
        Ax = linop(x)
        err = b - Ax
        nc = norm(x - x_prev)
        norm_change = nc * nc
        if iter_ > 0 and norm_change <= eps:
            break
        x_new = x + linop_T(err)
        x_new = proj(x_new)
        Ax = linop(x_new)
        err = b - Ax
        x_select = x_new
        if iter_ > 2:
            delta_Ax = Ax - Ax_prev
            dp = dot(delta_Ax, delta_Ax)
            if dp > 0:
                a1 = dot(delta_Ax, err) / dp
                Ax_1 = (1 + a1) * Ax - a1 * Ax_prev
                x_1 = x_new + a1 * (x_new - x)
                err_1 = b - Ax_1
                delta_Ax = Ax_1 - Ax_prev_prev
                dp = dot(delta_Ax, delta_Ax)
                if dp > 0:
                    a2 = dot(delta_Ax, err_1) / dp
                    x_2 = x_1 + a2 * (x_1 - x_prev)
                    x_2 = proj(x_2)
                    Ax_2 = linop(x_2)
                    err_2 = b - Ax_2
                    if dot(err_2, err_2) / dot(err, err) < 1:
                        x_select = x_2
                        Ax = Ax_2
        x_prev = x
        x = x_select
        if iter_ % record_every == 0:
            start = log(iter_, x, time.time() - start)
        if options and options.get('verbose', 0) >= 1 and iter_ % 100 == 0:
            logging.debug('iter=%d: %e %e %e' % (iter_, dot(err, err), norm_change, norm(x)))
    log(iter_, x, time.time() - start)
    return x
