"""GradientDescent('LBFGS') on the C3 z-space problem, several device runs in
one process: ms per iteration, searches, state reads and fallbacks per run
(device.LineSearch instrumented), to see what makes a run slower."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))


def main():
    import torch
    import device
    from synthetic import make_shard, add_noise, CONFIGS, SEED
    from gradient_descent import GradientDescent
    c = CONFIGS['C3']
    sh = make_shard(c['n'], c['p'], c['m'], c['per_col'], seed=SEED)
    b = add_noise(sh['Ax'], 0.02, seed=SEED)
    opts = {'max_iter': 20, 'verbose': 0, 'opt_tol': 1e-30}
    eng = device.BBEngine(sh['A'], b, sh['block_sizes'], options=opts, AT=sh['AT'])
    cnt = {}
    orig = device.LineSearch.search

    def search(self, *a, **k):
        cnt['search'] = cnt.get('search', 0) + 1
        t0 = time.perf_counter()
        r = orig(self, *a, **k)
        cnt['search_s'] = cnt.get('search_s', 0.0) + time.perf_counter() - t0
        cnt['trials'] = cnt.get('trials', 0) + r[2]
        if r[1] != 1 or self.last is None:
            cnt['fallback'] = cnt.get('fallback', 0) + 1
        return r
    device.LineSearch.search = search
    for run in range(4):
        mode = 'host' if run == 2 else 'device'
        os.environ['BSLS_LBFGS_LS'] = mode
        cnt.clear()
        gd = GradientDescent(z0=np.zeros(eng.nz), method='LBFGS', options=dict(opts), engine=eng)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        it, _, _ = gd.run()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print('run %d %-6s %.3f ms/iteration  %s' % (run, mode, el * 1e3 / it[-1],
              {k: (round(v, 4) if isinstance(v, float) else v) for k, v in cnt.items()}), flush=True)


if __name__ == '__main__':
    main()
