"""Where a short GradientDescent('LBFGS') run's fixed cost goes: runs of 1,
20 and 40 iterations (the per-run overhead vs the marginal iteration), and a
cProfile of a 1-iteration run."""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))


def main():
    import torch
    from device import BBEngine
    from synthetic import make_shard, add_noise, CONFIGS, SEED
    from gradient_descent import GradientDescent
    c = CONFIGS['C3']
    sh = make_shard(c['n'], c['p'], c['m'], c['per_col'], seed=SEED)
    b = add_noise(sh['Ax'], 0.02, seed=SEED)
    opts = {'max_iter': 20, 'verbose': 0, 'opt_tol': 1e-30}
    eng = BBEngine(sh['A'], b, sh['block_sizes'], options=opts, AT=sh['AT'])

    def run(k, prof=None):
        gd = GradientDescent(z0=np.zeros(eng.nz), method='LBFGS', options=dict(opts, max_iter=k),
                             engine=eng)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if prof:
            prof.enable()
        gd.run()
        torch.cuda.synchronize()
        if prof:
            prof.disable()
        return time.perf_counter() - t0
    run(20)
    for k in (1, 1, 20, 40, 1):
        print('max_iter %2d: %.2f ms' % (k, run(k) * 1e3), flush=True)
    p = cProfile.Profile()
    run(1, p)
    pstats.Stats(p).sort_stats('cumulative').print_stats(30)


if __name__ == '__main__':
    main()
