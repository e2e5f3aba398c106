"""GradientDescent('LBFGS') on the C3 z-space problem with the device line
search and with the host-decided one (BSLS_LBFGS_LS=host): wall time per
iteration, trials per search, and where an iteration's time goes (cProfile of
the device run's Python side)."""
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
    from synthetic import make_shard, add_noise, CONFIGS, SEED
    from device import BBEngine
    from gradient_descent import GradientDescent
    c = CONFIGS['C3']
    sh = make_shard(c['n'], c['p'], c['m'], c['per_col'], seed=SEED)
    b = add_noise(sh['Ax'], 0.02, seed=SEED)
    iters = int(os.environ.get('ITERS', '20'))
    opts = {'max_iter': iters, 'verbose': 0, 'opt_tol': 1e-30}
    eng = BBEngine(sh['A'], b, sh['block_sizes'], options=opts, AT=sh['AT'])
    for mode in ('device', 'host', 'device'):
        os.environ['BSLS_LBFGS_LS'] = mode
        gd = GradientDescent(z0=np.zeros(eng.nz), method='LBFGS', options=dict(opts), engine=eng)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        prof = cProfile.Profile() if mode == 'device' else None
        if prof:
            prof.enable()
        it, _, _ = gd.run()
        torch.cuda.synchronize()
        if prof:
            prof.disable()
        el = time.perf_counter() - t0
        st = eng.line_search().st.cpu().numpy()
        print('%-6s %3d iterations  %.3f ms/iteration  last search: t=%g exit=%d trials=%d'
              % (mode, it[-1], el * 1e3 / max(1, it[-1]), st[0], st[3], st[7]), flush=True)
    pstats.Stats(prof).sort_stats('cumulative').print_stats(25)


if __name__ == '__main__':
    main()
