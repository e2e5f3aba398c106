"""C2 projection A/B over BSLS_PROJ_WAVES (waves per workgroup, staggered
loads): bench.py's own proj leg (16 distinct HBM-resident copies back to
back) plus a bit-exact check of one launch against the oracle, for U[0,1) and
5 N(0,1) inputs.  The variant is read once per process, so run one process
per setting:  BSLS_PROJ_WAVES=2 python tools/proj_waves.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))


def main():
    import torch
    import _native
    from _native import ptr, stream_handle, check
    from synthetic import proj_input
    from oracle import oracle as orc
    import bench
    L = _native.lib()
    w = os.environ.get('BSLS_PROJ_WAVES', '1')
    for kind in ('unif', 'normal'):
        y_h, st_h = proj_input(kind=kind)
        n, p = y_h.shape[0], st_h.shape[0]
        mb = int(np.max(np.diff(np.append(st_h, n))))
        y = torch.from_numpy(y_h).cuda()
        st = torch.from_numpy(st_h).cuda()
        ws = torch.zeros(L.bsls_proj_workspace_size(n, p, mb), dtype=torch.uint8, device='cuda')
        check(L.bsls_proj_multi_simplex(ptr(y), ptr(st), p, n, mb, ptr(ws), ws.numel(),
                                        stream_handle()), 'proj')
        yc = y_h.copy()
        orc.proj_multi_simplex_c(yc, st_h)
        ok = np.array_equal(yc.view(np.int64), y.cpu().numpy().view(np.int64))
        print('waves %s %-6s bit-exact %s' % (w, kind, ok), flush=True)
    r = bench.bench_proj()
    print('waves %s bench avg_us %.2f frac %.3f isolated %s'
          % (w, r['avg_us'], r['frac_hbm_peak'],
             {k: v for k, v in r.items() if k.startswith('isolated')}), flush=True)


if __name__ == '__main__':
    main()
