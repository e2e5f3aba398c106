"""Per-iteration trace of LBFGS.solve on the plugins fixture (the
test_lbfgs_vs_reference run) with the device line search and with the host
one: t, exit, f, y.s, ||g||^2 per iteration, to locate a divergence."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    import device
    import solvers
    import LBFGS
    from test_gpu_plugins import _gd_run
    G = dict(np.load(os.path.join(ROOT, 'tests', 'golden', 'plugins.npz')))
    orig = device.LineSearch.search

    def search(self, *a, **k):
        r = orig(self, *a, **k)
        print('  search t=%.17g exit=%d trials=%d dnorm=%.6e last=%s' % (r + (self.last,)), flush=True)
        return r
    device.LineSearch.search = search
    ostop = solvers.stopping

    def stopping(g, fx, i, t, d=None, options=None):
        print('  iter %d f=%.17g t=%.17g |g|=%.17g' % (i, fx, t, float(LBFGS.norm(g))), flush=True)
        return ostop(g, fx, i, t, d=d, options=options)
    solvers.stopping = stopping
    LBFGS.stopping = stopping
    for mode in ('device', 'host'):
        os.environ['BSLS_LBFGS_LS'] = mode
        print(mode, flush=True)
        eng, gd, iters, states = _gd_run(G, 'lbfgs', 'LBFGS', {'max_iter': 5, 'verbose': 0,
                                                                'opt_tol': 1e-30})
        for k, s in enumerate(states):
            ref = G['lbfgs_states'][k]
            print('  state %d rel %.3e' % (iters[k], np.max(np.abs(s - ref)) / max(1, np.max(np.abs(ref)))))


if __name__ == '__main__':
    main()
