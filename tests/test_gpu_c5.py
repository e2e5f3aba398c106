"""Config C5 at full size on one GPU (BASELINE.json configs[4]): 10M routes /
500k blocks / 1M links / 160M nnz, the world-independent problem
(synthetic.make_partitioned) that bench.py shards over N GPUs.  Its sparse row
blocks take the streamed-tile kernels (csrc/tiles.hpp):
  * K2 (g = N'A'r, one column group): on the deterministic engine (thread
    streams) bit-identical to SciPy; on the default dealt image within 1e-12;
  * K1 (r = A x + target, column-group partials) within 1e-12;
  * K3 (PAVA v1 + clip + N z on the 9.5M-entry z layout) bit-identical to the
    oracle;
  * BB iterates 1..3 within 1e-12 per element of the oracle's BB trajectory
    (the north star allows 1e-6).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def c5(cuda):
    from synthetic import make_partitioned, add_noise, SEED
    from device import BBEngine
    sh = make_partitioned(10_000_000, 500_000, 1_000_000)
    b = add_noise(sh['Ax'], 0.02, seed=SEED)
    eng = BBEngine(sh['A'], b, sh['block_sizes'], options={'max_iter': 3, 'opt_tol': 1e-30},
                   AT=sh['AT'], colv=sh['colv'])
    return sh, b, eng


def _nt(sizes, w):
    """N'w as SciPy's N.T.dot forms it: w_i - w_{i+1} for every non-last entry."""
    last = np.cumsum(sizes) - 1
    keep = np.ones(w.shape[0], dtype=bool)
    keep[last] = False
    return (w[:-1] - w[1:])[keep[:-1]]


def test_c5_takes_the_tile_kernels(c5):
    _, _, eng = c5
    assert eng.fmt_A == 'tiles' and eng.fmt_AT == 'tiles'
    assert eng.AT_til.img['ngroups'] == 1


def test_c5_k2_vs_scipy(c5):
    """The default (dealt, 3-byte entries) K2: LDS atomic sums, equal to SciPy to rounding."""
    import torch
    sh, _, eng = c5
    assert eng.AT_til.img['layout'] == 2
    r = np.random.RandomState(5).randn(eng.m)
    eng.r.copy_(torch.from_numpy(r))
    eng.stage(3, 0)
    got = eng.g[0][:eng.nz].cpu().numpy()
    want = _nt(sh['block_sizes'], sh['AT'].dot(r))
    assert np.max(np.abs(got - want)) <= 1e-12 * np.max(np.abs(want))


def test_c5_k2_bit_exact_vs_scipy_deterministic(c5):
    """deterministic=True: K2 on thread streams, every row in CSR order --
    bit-identical to SciPy at full C5 size."""
    import torch
    from device import BBEngine
    sh, b, _ = c5
    eng = BBEngine(sh['A'], b, sh['block_sizes'], options={'max_iter': 3, 'opt_tol': 1e-30},
                   AT=sh['AT'], colv=sh['colv'], deterministic=True)
    assert eng.AT_til.img['layout'] == 0 and eng.AT_til.img['ngroups'] == 1
    r = np.random.RandomState(5).randn(eng.m)
    eng.r.copy_(torch.from_numpy(r))
    eng.stage(3, 0)
    got = eng.g[0][:eng.nz].cpu().numpy()
    want = _nt(sh['block_sizes'], sh['AT'].dot(r))
    assert np.array_equal(got, want)
    del eng


def test_c5_k1_residual_vs_scipy(c5):
    import torch
    sh, _, eng = c5
    x = np.random.RandomState(6).rand(eng.n)
    eng.x.copy_(torch.from_numpy(sh['colv'] * x))
    eng.stage(7, 0)
    got = eng.r.cpu().numpy()
    want = sh['A'].dot(x) + eng.target.cpu().numpy()
    assert np.max(np.abs(got - want)) <= 1e-12 * np.max(np.abs(want))


def test_c5_k3_bit_exact_vs_oracle(c5, orc):
    import torch
    import _native
    sh, _, eng = c5
    rs = np.random.RandomState(7)
    nz = eng.nz
    zc = rs.rand(nz)
    g = rs.randn(nz) * 0.5
    t = 0.37
    eng.z[0][:nz].copy_(torch.from_numpy(zc))
    eng.g[1][:nz].copy_(torch.from_numpy(g))
    sc = np.zeros(_native.S_COUNT)
    sc[_native.S_SUMDG], sc[_native.S_DZDG], sc[_native.S_DGDG] = 1.0, t, 1.0
    eng.scal.copy_(torch.from_numpy(sc))
    warm, eng.P.pava_warm = eng.P.pava_warm, 0      # the reference passes: bit-identical
    try:
        eng.stage(4, 1)
    finally:
        eng.P.pava_warm = warm
    got = eng.z[1][:nz].cpu().numpy()
    ref = zc - t * g
    orc.isotonic_regression_multi_c(ref, eng.layout.zstarts_h)
    ref = np.maximum(np.minimum(ref, 1.0), 0.0)
    assert np.array_equal(got.view(np.int64), ref.view(np.int64))
    # x = colv * (N z): per-block differences, last entry -z_last
    sizes = sh['block_sizes']
    zs = eng.layout.zstarts_h
    xs = np.zeros(eng.n)
    xstart = eng.layout.xstarts_h
    prev = np.zeros(nz)
    head = np.zeros(nz, dtype=bool)
    head[zs] = True
    prev[~head] = ref[:-1][~head[1:]]
    xidx = np.arange(nz) + np.repeat(np.arange(sizes.size), sizes - 1)
    xs[xidx] = ref - prev
    xs[xstart + sizes - 1] = -ref[zs + sizes - 2]
    assert np.array_equal(eng.x.cpu().numpy(), sh['colv'] * xs)


def test_c5_bb_iterates_vs_oracle(c5, orc, parity):
    sh, b, eng = c5
    rec = {}

    def log(i, s, dt):
        rec[i] = s
        return 0.0
    eng.solve(log=log, record_every=1, poll=1)
    ref = orc.bb_trace(sh['A'], b, sh['block_sizes'], 3, record_every=1)
    for i in (1, 2, 3):
        d = np.max(np.abs(rec[i] - ref[i])) / max(1.0, np.max(np.abs(ref[i])))
        parity('c5_bb_%d' % i, d, 1e-12)
