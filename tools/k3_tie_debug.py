"""Debug helper: K3 on tie-heavy input vs the oracle, printing mismatches."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))
import numpy as np, scipy.sparse as sps, torch
import _native
from device import BBEngine
from oracle import oracle as orc
rs = np.random.RandomState(7)
sizes = np.concatenate([rs.randint(2, 40, size=300), [66, 65, 130, 2, 150, 64, 3]])
rs.shuffle(sizes)
n = int(sizes.sum()); m = 200
A = sps.random(m, n, density=0.02, random_state=rs, format='csr')
eng = BBEngine(A, rs.randn(m), sizes, options={'max_iter': 10, 'opt_tol': 1e-30})
nz = eng.nz
zst = eng.layout.zstarts_h
for mode in ('round0', 'round0_nozero', 'round1'):
    zc = np.round(rs.randn(nz), 1 if mode == 'round1' else 0)
    if mode != 'round0_nozero':
        zc[rs.rand(nz) < 0.1] = -0.0
    g = np.zeros(nz)
    eng.z[0][:nz].copy_(torch.from_numpy(zc)); eng.g[1][:nz].copy_(torch.from_numpy(g))
    sc = np.zeros(_native.S_COUNT); sc[_native.S_SUMDG] = 1.0; sc[_native.S_DZDG] = 1.0; sc[_native.S_DGDG] = 1.0
    eng.scal.copy_(torch.from_numpy(sc)); eng.stage(4, 1)
    got = eng.z[1][:nz].cpu().numpy()
    y = zc - 1.0 * g
    ref = y.copy(); orc.isotonic_regression_multi_c(ref, zst)
    refc = np.maximum(np.minimum(ref, 1.0), 0.0)
    bad = np.nonzero(got.view(np.int64) != refc.view(np.int64))[0]
    print(mode, 'mismatches', bad.size, 'value-mismatches', int(np.sum(got != refc)))
    for i in bad[:6]:
        b = np.searchsorted(zst, i, side='right') - 1
        s0 = zst[b]; e0 = zst[b + 1] if b + 1 < zst.size else nz
        print(' idx', i, 'block', b, 'len', e0 - s0, 'got', repr(got[i]), 'ref(clipped)', repr(refc[i]), 'ref', repr(ref[i]))
        print('   y   ', np.array2string(y[s0:e0], precision=3, max_line_width=200))
        print('   ref ', np.array2string(ref[s0:e0], precision=5, max_line_width=200))
        print('   got ', np.array2string(got[s0:e0], precision=5, max_line_width=200))
