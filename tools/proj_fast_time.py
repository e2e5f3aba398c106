"""Time the sort-free projection (bsls_proj_multi_simplex_fast) beside the exact
one on the C2 input the way bench.py does (16 distinct copies back to back
between two events: HBM-fed), and check the fast result against the oracle at
|d| <= 1e-12 max(1, |ref|).  BSLS_PROJ_LPB picks lanes per block (2 / 4 / 8).
python tools/proj_fast_time.py"""
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
    batch = 16
    for kind in ('unif', 'normal'):
        y_h, st_h = proj_input(kind=kind)
        n, p = y_h.shape[0], st_h.shape[0]
        mb = int(np.max(np.diff(np.append(st_h, n))))
        y0 = torch.from_numpy(y_h).cuda()
        st = torch.from_numpy(st_h).cuda()
        ws = torch.zeros(L.bsls_proj_workspace_size(n, p, mb), dtype=torch.uint8, device='cuda')
        ref = y_h.copy()
        orc.proj_multi_simplex_c(ref, st_h)
        for name in ('bsls_proj_multi_simplex', 'bsls_proj_multi_simplex_fast'):
            fn = getattr(L, name)
            ys = [y0.clone() for _ in range(batch)]
            for t in ys[:2]:
                check(fn(ptr(t), ptr(st), p, n, mb, ptr(ws), ws.numel(), stream_handle()), name)
            per = []
            for _ in range(5):
                for t in ys:
                    t.copy_(y0)
                torch.cuda.synchronize()
                torch.cuda._sleep(int(2e8))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for t in ys:
                    check(fn(ptr(t), ptr(st), p, n, mb, ptr(ws), ws.numel(), stream_handle()), name)
                e1.record()
                torch.cuda.synchronize()
                per.append(e0.elapsed_time(e1) / batch * 1e3)
            us = sorted(per)[len(per) // 2]
            out = ys[0].cpu().numpy()
            d = np.abs(out - ref) / np.maximum(1.0, np.abs(ref))
            byt = 16 * n + 4 * (p + 1)
            print('%-6s %-30s %6.2f us  %7.1f GB/s  frac %.3f  max rel %.2e  exact %s'
                  % (kind, name, us, byt / us / 1e3, byt / us / 8e6, d.max(),
                     np.array_equal(out.view(np.int64), ref.view(np.int64))), flush=True)
            del ys


if __name__ == '__main__':
    main()
