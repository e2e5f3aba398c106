"""Solver plugin glue (reference: python/solvers.py).

`stopping` is the termination rule BB / LBFGS call every iteration
(python/solvers.py:40-63); `least_squares` is the DORE wrapper (:35-37).  The
fused device engine (device.BBEngine) evaluates the same rule on the GPU.
The reference's dead `qp`/`qp2` (cvxopt / an undefined `spg`) are not carried.
"""
import logging

from _arr import norm


def stopping(g, fx, i, t, d=None, delta_g=None, options=None, TOLER=1e-6):
    """True when: i >= max_iter; ||g||^2 <= opt_tol (1 + |f|); ||t d|| <= 1e-12;
    or ||delta_g|| == 0 -- in that order (python/solvers.py:40-63)."""
    if options and 'max_iter' in options:
        if i >= options['max_iter']:
            return True
    if options and 'opt_tol' in options:
        TOLER = options['opt_tol']
    ng = norm(g)
    norm2_nabla_f = ng * ng
    thresh = TOLER * (1 + abs(float(fx)))
    if options and options.get('verbose', 0) >= 1 and i % 100 == 0:
        logging.debug('iter=%d: %e %e %e %f' % (i, float(t), norm2_nabla_f, thresh, float(fx)))
    if norm2_nabla_f <= thresh:
        logging.info('iter=%d: %e %e %e %f' % (i, float(t), norm2_nabla_f, thresh, float(fx)))
        logging.warning('Exiting... norm(grad) too small')
        return True
    if d is not None and norm(t * d) <= 1e-12:
        logging.info('iter=%d: %e %e %e %f' % (i, float(t), norm2_nabla_f, thresh, float(fx)))
        logging.warning('Exiting... step too small')
        return True
    if delta_g is not None and norm(delta_g) == 0:
        logging.info('iter=%d: %e %e %e %f' % (i, float(t), norm2_nabla_f, thresh, float(fx)))
        logging.warning('Exiting... no change in gradient')
        return True
    return False


def least_squares(x, linop, linop_transpose, target, proj=None, diagnostics=None,
                  options=None, log=None):
    """DORE accelerated projected least squares (python/solvers.py:35-37)."""
    import DORE
    if log is None:
        log = lambda i, s, d: 0.0
    return DORE.solve(x, linop, linop_transpose, target, proj=proj, log=log, options=options)
