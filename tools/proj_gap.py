"""Where the C2 projection's per-launch time goes between launches (design
aid): 16 launches back to back between two events -- on 16 distinct copies
(bench.py's avg_us), on one buffer (input warm in the Infinity Cache), as one
captured HIP graph -- against 16 tiny kernels (the launch floor) and 16
25.6-MB device copies (the streaming floor).  python tools/proj_gap.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))


def timed(fn, reps=3):
    import torch
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        torch.cuda._sleep(int(2e8))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) * 1e3 / 16)
    return sorted(out)[len(out) // 2]


def main():
    import torch
    import _native
    from _native import ptr, stream_handle, check
    from synthetic import proj_input
    L = _native.lib()
    y_h, st_h = proj_input()
    n, p = y_h.shape[0], st_h.shape[0]
    mb = int(np.max(np.diff(np.append(st_h, n))))
    y0 = torch.from_numpy(y_h).cuda()
    st = torch.from_numpy(st_h).cuda()
    ws = torch.zeros(L.bsls_proj_workspace_size(n, p, mb), dtype=torch.uint8, device='cuda')

    def proj(t):
        check(L.bsls_proj_multi_simplex(ptr(t), ptr(st), p, n, mb, ptr(ws), ws.numel(),
                                        stream_handle()), 'proj')
    ys = [y0.clone() for _ in range(16)]
    for t in ys:
        proj(t)
    res = {}

    def distinct():
        for t in ys:
            proj(t)
    for t in ys:
        t.copy_(y0)
    res['distinct_copies'] = timed(distinct, 1)
    one = ys[0]
    res['one_buffer'] = timed(lambda: [proj(one) for _ in range(16)])
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        proj(one)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(16):
                proj(one)
    res['graph_one_buffer'] = timed(lambda: g.replay())
    tiny = torch.zeros(1, device='cuda')
    res['tiny_kernel'] = timed(lambda: [tiny.add_(1.0) for _ in range(16)])
    dst = torch.empty_like(y0)
    res['copy_25MB'] = timed(lambda: [dst.copy_(y0) for _ in range(16)])
    for k, v in res.items():
        print('%-18s %7.2f us per launch' % (k, v), flush=True)


if __name__ == '__main__':
    main()
