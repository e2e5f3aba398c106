"""Time the product projection (bsls_proj_multi_simplex) on the C2 input the
way bench.py does (fresh copy per launch, events around each launch, stream
held while enqueuing), for U[0,1), 5 N(0,1) and a re-projected (already
projected) input; checks bit-exactness against the oracle.
python tools/proj_time.py"""
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
    L = _native.lib()
    for kind in ('unif', 'normal', 'reproj'):
        y_h, st_h = proj_input(kind='normal' if kind == 'normal' else 'unif')
        if kind == 'reproj':
            orc.proj_multi_simplex_c(y_h, st_h)
        n, p = y_h.shape[0], st_h.shape[0]
        mb = int(np.max(np.diff(np.append(st_h, n))))
        y0 = torch.from_numpy(y_h).cuda()
        y = y0.clone()
        st = torch.from_numpy(st_h).cuda()
        ws = torch.zeros(L.bsls_proj_workspace_size(n, p, mb), dtype=torch.uint8, device='cuda')
        reps = 30
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(reps)]
        for _ in range(3):
            y.copy_(y0)
            check(L.bsls_proj_multi_simplex(ptr(y), ptr(st), p, n, mb, ptr(ws), ws.numel(),
                                            stream_handle()), 'proj')
        torch.cuda.synchronize()
        torch.cuda._sleep(int(2e8))
        for k in range(reps):
            y.copy_(y0)
            evs[k][0].record()
            check(L.bsls_proj_multi_simplex(ptr(y), ptr(st), p, n, mb, ptr(ws), ws.numel(),
                                            stream_handle()), 'proj')
            evs[k][1].record()
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in evs)
        yc = y_h.copy()
        orc.proj_multi_simplex_c(yc, st_h)
        ok = np.array_equal(yc.view(np.int64), y.cpu().numpy().view(np.int64))
        byt = 16 * n + 4 * (p + 1)
        med = ms[len(ms) // 2]
        print('%-7s median %6.1f us  min %6.1f us  %7.1f GB/s  frac %.3f  bit-exact %s'
              % (kind, med * 1e3, ms[0] * 1e3, byt / med / 1e6, byt / med / 8e9, ok), flush=True)


if __name__ == '__main__':
    main()
