"""Partition stability of K3's PAVA between BB iterations (CPU, oracle replay):
the share of blocks / packs whose final run partition equals the previous
iteration's -- the case for K3's warm start (pava_wave.hpp pava_warm).
python tools/k3_warm.py [n]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tools'))
from k3_passes import packs_of

def final_heads(y):
    # stack PAVA (increasing fit): returns tuple of run start indices
    st = []  # (start, sum, cnt)
    for i, v in enumerate(y):
        st.append([i, v, 1])
        while len(st) > 1 and st[-2][1] / st[-2][2] >= st[-1][1] / st[-1][2]:
            s, sm, c = st.pop()
            st[-1][1] += sm; st[-1][2] += c
    return tuple(s[0] for s in st)

import synthetic
from oracle import oracle as orc
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
sh = synthetic.make_shard(n, n // 20, n // 10, 16)
b = synthetic.add_noise(sh['Ax'], 0.02)
sizes = sh['block_sizes']
P = orc.solve_in_z_parts(sh['A'], b, sizes)
kz = sizes - 1; zst = P['zstarts']
packs = packs_of(kz)
prev = [None]
it = [0]
proj0 = P['proj']
at = {2, 3, 5, 10, 20, 50, 100, 150, 200}
def proj(x):
    it[0] += 1
    H = [final_heads(x[zst[bb]:zst[bb] + kz[bb]]) for bb in range(kz.size)]
    if prev[0] is not None and it[0] in at:
        same = np.array([H[i] == prev[0][i] for i in range(kz.size)])
        pk = np.mean([all(same[bb] for bb in p) for p in packs])
        print('iter %d: blocks same partition %.3f, packs %.3f' % (it[0], same.mean(), pk), flush=True)
    prev[0] = H
    return proj0(x)
orc.bb_solve(P['z0'], P['f'], P['nabla_f'], orc.stopping, record_every=10 ** 9, proj=proj,
             log=lambda i, s, dt: 0.0, options={'max_iter': max(at), 'verbose': 0, 'opt_tol': 1e-30})
