"""Lane-per-block PAVA (iso_kernel, pava.hip) on the C3 z layout -- 950k
entries in 50k blocks, inputs like K3's (z - t g) -- to set against K3's
wave-parallel PAVA.  python tools/iso_time.py  (GPU box)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))


def main():
    import numpy as np
    import torch
    import _native
    from _native import ptr, stream_handle, check
    from synthetic import make_shard, CONFIGS, SEED
    L = _native.lib()
    c = CONFIGS['C3']
    sh = make_shard(c['n'], c['p'], c['m'], c['per_col'], seed=SEED)
    zs = np.concatenate(([0], np.cumsum(sh['block_sizes'] - 1)[:-1])).astype(np.int64)
    nz = int((sh['block_sizes'] - 1).sum())
    rs = np.random.RandomState(3)
    y0 = torch.from_numpy(rs.rand(nz) - 0.3 * rs.randn(nz)).cuda()
    st = torch.from_numpy(zs).cuda()
    mb = int(np.max(sh['block_sizes']))
    ws = torch.zeros(L.bsls_isotonic_workspace_size(nz), dtype=torch.uint8, device='cuda')
    status = torch.zeros(4, dtype=torch.int32, device='cuda')
    batch = 16
    ys = [y0.clone() for _ in range(batch)]

    def iso(t):
        check(L.bsls_isotonic_multi(1, ptr(t), ptr(st), zs.size, nz, None, 1, mb, ptr(ws),
                                    ws.numel(), ptr(status), stream_handle()), 'iso')
    for t in ys[:2]:
        iso(t)
    out = []
    for _ in range(3):
        for t in ys:
            t.copy_(y0)
        torch.cuda.synchronize()
        torch.cuda._sleep(int(2e8))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for t in ys:
            iso(t)
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / batch * 1e3)
    print(json.dumps({'iso_v1_us': sorted(out)[1], 'nz': nz, 'blocks': int(zs.size)}))


if __name__ == '__main__':
    main()
