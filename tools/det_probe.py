import sys, numpy as np, torch
sys.path.insert(0,'block-simplex-least-squares_amd')
from device import BBEngine
from synthetic import make_shard, add_noise
sh = make_shard(50_000, 2_500, 5_000, per_col=16, seed=3)
b = add_noise(sh['Ax'], 0.02, seed=3)
eng = BBEngine(sh['A'], b, sh['block_sizes'], options={'max_iter': 30, 'opt_tol': 1e-30}, fmt='tiles', tile_plans=((1024, 4, 0), (1536, 2, 0)))
rs = np.random.RandomState(0)
x = torch.from_numpy(rs.rand(eng.n)).cuda(); eng.x.copy_(x)
r = torch.from_numpy(rs.randn(eng.m)).cuda()
outs = {}
for k in range(5):
    eng.x.copy_(x); eng.stage(7, 0); outs.setdefault('k1', []).append(eng.r.clone())
    eng.r.copy_(r); eng.stage(3, 0); outs.setdefault('k2', []).append(eng.g[0].clone())
for k, v in outs.items():
    print(k, [bool(torch.equal(v[0], w)) for w in v[1:]], [int((v[0] != w).sum()) for w in v[1:]])
