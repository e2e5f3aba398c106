"""Solver dispatch (reference: python/gradient_descent.py:13-69).

GradientDescent(z0, f, nabla_f, proj, method, options, A, N, target).run()
returns (iters, times, states) exactly like the reference: states logged at
iteration 0, every `record_every` iterations and at the end.

On MI355X the z-space problem is carried by a device.BBEngine (`engine=`):
  'BB'    -> the fused device loop (three kernels per iteration, no host sync
             between polls) -- the hot path;
  'DORE'  -> DORE.solve over the engine's linops (its K1 / K2 images), with
             the largest singular value of A N from ARPACK over the same;
  'LBFGS' -> LBFGS.solve over the engine's closures f / nabla_f / proj.
Without an engine the plain closures f / nabla_f / proj are used (they must
then already compute on the device).
"""
import logging
import time

import numpy as np

import BB
import DORE
import LBFGS
import solvers
from bsls_utils import lsv_operator


class GradientDescent:

    def __init__(self, z0=None, f=None, nabla_f=None, proj=None, method='BB', options=None,
                 A=None, N=None, target=None, engine=None, to_host=True):
        self.z0 = z0
        self.f = f
        self.nabla_f = nabla_f
        self.proj = proj
        self.method = method
        self.A, self.N, self.target = A, N, target      # DORE only (reference)
        self.engine = engine
        self.to_host = to_host
        if options is None:
            self.options = {'max_iter': 300000, 'verbose': 1, 'opt_tol': 1e-30,
                            'suff_dec': 0.003, 'corrections': 500}
        else:
            self.options = options
        self.iters, self.times, self.states = [], [], []

        def log(iter_, state, duration):
            self.iters.append(iter_)
            self.times.append(duration)
            if self.to_host and hasattr(state, 'detach'):
                state = state.detach().cpu().numpy()
            self.states.append(state)
            return time.time()
        self.log = log

    def _device_closures(self):
        e = self.engine
        return e.f, e.nabla_f, e.proj

    def run(self):
        logging.debug('Starting %s solver...' % self.method)
        e = self.engine
        if self.method == 'LBFGS':
            f, nabla_f, proj = self._device_closures() if e else (self.f, self.nabla_f, self.proj)
            z0 = self._z0_device() if e else self.z0
            LBFGS.solve(z0 + 1, f, nabla_f, solvers.stopping, log=self.log, proj=proj,
                        options=self.options)
            logging.debug('Took %s time' % str(np.sum(self.times)))
        elif self.method == 'BB':
            if e is not None:
                e.P.max_iter = int(self.options.get('max_iter', 300000))
                e.P.opt_tol = float(self.options.get('opt_tol', 1e-6))
                BB.solve_engine(e, z0=self.z0, log=self.log, to_host=self.to_host)
            else:
                BB.solve(self.z0, self.f, self.nabla_f, solvers.stopping, log=self.log,
                         proj=self.proj, options=self.options)
        elif self.method == 'DORE':
            if e is None:
                if self.A is None or self.N is None or self.target is None:
                    raise ValueError("method 'DORE' needs the device engine (main.solve_in_z) "
                                     "or A, N and target (the host path, main.solve_in_z_cpu)")
                # the host path (gradient_descent.py:55-67 as the reference runs it)
                alpha = 0.99
                lsv = lsv_operator(self.A, self.N)
                logging.info('Largest singular value: %s' % lsv)
                A_dore = self.A * alpha / lsv
                target_dore = self.target * alpha / lsv
                N = self.N
                DORE.solve(self.z0, lambda z: A_dore.dot(N.dot(z)),
                           lambda r: N.T.dot(A_dore.T.dot(r)), target_dore, proj=self.proj,
                           log=self.log, options=self.options, record_every=100)
                self.lsv = lsv
                return self.iters, self.times, self.states
            alpha = 0.99
            lsv = lsv_operator(e, None)
            logging.info('Largest singular value: %s' % lsv)
            scale = alpha / lsv
            b_t = e.target * scale

            # the whole loop on the device (linop = scale A N, linop_T =
            # scale N'A', proj = PAVA v1 + clip on the engine's images)
            DORE.solve_engine(e, self._z0_device(), scale, b_t, log=self.log,
                              options=self.options, record_every=100)
            self.lsv = lsv
        else:
            raise ValueError('unknown method %r' % self.method)
        logging.debug('Stopping %s solver...' % self.method)
        return self.iters, self.times, self.states

    def _z0_device(self):
        import torch
        z0 = self.z0
        if isinstance(z0, torch.Tensor):
            return z0.to('cuda', torch.float64)
        return torch.from_numpy(np.ascontiguousarray(z0, dtype=np.float64)).cuda()
