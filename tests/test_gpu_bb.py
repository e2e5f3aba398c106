"""Fused BB engine (K1/K2/K3 on device) vs the reference's own BB trajectories.

The north star allows 1e-6 relative on iterates; they are held to 1e-12 per
element (measured ~1e-15: only the SpMV summation order differs from SciPy;
profiles/r06_parity_errors.jsonl).  Needs an MI355X.
"""
import numpy as np
import pytest
import scipy.sparse as sps

pytestmark = pytest.mark.gpu


def _csr(G, tag):
    return sps.csr_matrix((G['%s_A_data' % tag], G['%s_A_indices' % tag],
                           G['%s_A_indptr' % tag]), shape=tuple(G['%s_A_shape' % tag]))


def rel_err(a, b):
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def elem_err(a, b):
    """max over elements of |a - b| / max(1, |b|)."""
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b))))


@pytest.mark.parametrize('tag', ['bbs', 'bbc'])
def test_bb_trajectory_vs_reference(cuda, golden, tag, parity):
    from device import BBEngine
    G = golden('solvers.npz')
    A = _csr(G, tag)
    iters = list(G['%s_iters' % tag])
    eng = BBEngine(A, G['%s_b' % tag], G['%s_block_sizes' % tag],
                   options={'max_iter': int(iters[-1]), 'opt_tol': 1e-30})
    rec = {}

    def log(i, s, dt):
        rec[i] = s
        return 0.0
    eng.solve(log=log, record_every=1, poll=1)
    assert sorted(rec) == iters
    worst = max(rel_err(rec[i], G['%s_states' % tag][k]) for k, i in enumerate(iters))
    parity('bb_golden_%s' % tag, worst, 1e-12)


def test_bb_main_problems_converge(cuda, golden):
    """tests/fast/test_main.py criterion on the same three problems."""
    import torch
    from device import BBEngine
    G = golden('solvers.npz')
    for vi in range(3):
        A = _csr(G, 'main%d' % vi)
        b, bs = G['main%d_b' % vi], G['main%d_block_sizes' % vi]
        eng = BBEngine(A, b, bs, options={'max_iter': 300000, 'opt_tol': 1e-30})
        z = eng.solve(poll=25)
        x = torch.empty(eng.n, dtype=torch.float64, device='cuda')
        # x = x0 + N z via the device z2x
        from c_extensions.c_extensions import z2x_c
        xs = np.zeros(eng.n)
        z2x_c(xs, z.cpu().numpy().copy(), eng.layout.xstarts_h)
        err = 0.5 * np.linalg.norm(A.dot(xs) - b) ** 2
        assert err < 1e-16, (vi, err)
        # the exit fires on an exact-zero sum(delta_g) (BB.py:22), which depends on
        # the last bits of the trajectory: only the order of magnitude is pinned
        ref_last = int(G['main%d_iters' % vi][-1])
        assert abs(eng.iterations - ref_last) <= max(10, ref_last // 4), (eng.iterations, ref_last)


@pytest.fixture(scope='module')
def shard100k(orc):
    from synthetic import make_shard, add_noise
    sh = make_shard(100_000, 5_000, 10_000, per_col=16, seed=11)
    b = add_noise(sh['Ax'], 0.02, seed=11)
    ref = orc.bb_trace(sh['A'], b, sh['block_sizes'], 50, record_every=1)
    return sh, b, ref


# SpMV formats: the panels (dense row blocks); the streamed tiles as the
# engine picks them (dealt images for K1 and K2: column-sorted gathers, LDS
# atomic sums); the thread-stream tiles (deterministic=True: every row in CSR
# order); the tiles with several column groups (partials + last-arriver
# sums); K1 dealt with K2 on thread streams
FORMATS = {'panels': dict(fmt='panels'),
           'tiles': dict(fmt='tiles'),
           'tiles-det': dict(fmt='tiles', deterministic=True),
           'tiles-groups': dict(fmt='tiles', tile_plans=((1024, 4, 0), (1536, 2, 0))),
           'tiles-mixed': dict(fmt='tiles', tile_layouts=(1, 0)),
           'tiles-dealt16': dict(fmt='tiles', tile_layouts=(1, 1)),
           'tiles-dealt12': dict(fmt='tiles', tile_layouts=(2, 2)),
           'tiles-dealt12-groups': dict(fmt='tiles', tile_layouts=(2, 2),
                                        tile_plans=((1024, 4, 0), (1536, 2, 0)))}
# formats whose K2 sums each row in CSR order (one group, thread streams)
K2_EXACT = ('panels', 'tiles-det', 'tiles-mixed')
# formats with a fixed summation order everywhere (bit-reproducible runs)
DETERMINISTIC = ('panels', 'tiles-det')


@pytest.mark.parametrize('fmt', sorted(FORMATS))
@pytest.mark.parametrize('general', [False, True])
def test_bb_fixed_iterations_match_oracle_at_scale(cuda, shard100k, general, fmt, parity):
    """A 100k-route synthetic problem, iterates at 1, 10, 50 vs the oracle, with
    the scaled-incidence images (no values) and with stored values, on every
    SpMV format."""
    from device import BBEngine
    sh, b, ref = shard100k
    eng = BBEngine(sh['A'], b, sh['block_sizes'], options={'max_iter': 50, 'opt_tol': 1e-30},
                   general=general, **FORMATS[fmt])
    assert eng.scaled == (not general)
    assert eng.fmt_A == eng.fmt_AT == FORMATS[fmt]['fmt']
    rec = {}

    def log(i, s, dt):
        rec[i] = s
        return 0.0
    eng.solve(log=log, record_every=1, poll=1)
    # per element, every format -- the fixed-order ones and the run-dependent
    # ones (LDS / global atomics) -- at 1e-12 (measured <= ~1e-15)
    for i in (1, 10, 50):
        parity('bb_100k_%s_%s_%d' % (fmt, 'general' if general else 'scaled', i),
               elem_err(rec[i], ref[i]), 1e-12)


@pytest.mark.parametrize('fmt', sorted(FORMATS))
@pytest.mark.parametrize('general', [False, True])
def test_k2_gradient_bit_exact_vs_scipy(cuda, shard100k, general, fmt):
    """K2 alone (stage 3): w = A'r is summed in CSR order (panels: in a register
    per row; tiles: in LDS, each thread's stream in column order), so with one
    column group g = N'(A'r) equals SciPy's N.T.dot(A.T.dot(r)) bit for bit;
    with several groups to rounding."""
    import torch
    from device import BBEngine
    from oracle import oracle as orc
    sh, b, _ = shard100k
    eng = BBEngine(sh['A'], b, sh['block_sizes'], options={'max_iter': 5, 'opt_tol': 1e-30},
                   general=general, **FORMATS[fmt])
    r = np.random.RandomState(5).randn(eng.m)
    eng.r.copy_(torch.from_numpy(r))
    eng.stage(3, 0)
    got = eng.g[0][:eng.nz].cpu().numpy()
    N = orc.block_sizes_to_N(sh['block_sizes'])
    want = N.T.tocsr().dot(sh['AT'].dot(r))
    if fmt not in K2_EXACT:
        assert np.max(np.abs(got - want)) <= 1e-12 * np.max(np.abs(want))
    else:
        assert np.array_equal(got, want)


@pytest.mark.parametrize('fmt', sorted(FORMATS))
def test_k1_residual_vs_scipy(cuda, shard100k, fmt):
    """K1 alone (stage 7 at iteration 0): r = A x + target with chunk-group
    partials; equal to SciPy to rounding (1e-12 relative)."""
    import torch
    from device import BBEngine
    sh, b, _ = shard100k
    eng = BBEngine(sh['A'], b, sh['block_sizes'], options={'max_iter': 5, 'opt_tol': 1e-30},
                   **FORMATS[fmt])
    x = np.random.RandomState(6).rand(eng.n)
    xin = torch.from_numpy(eng.colv.cpu().numpy() * x if eng.scaled else x).cuda()
    eng.x.copy_(xin)
    eng.stage(7, 0)
    got = eng.r.cpu().numpy()
    want = sh['A'].dot(x) + eng.target.cpu().numpy()
    assert np.max(np.abs(got - want)) <= 1e-12 * np.max(np.abs(want))


@pytest.mark.parametrize('fmt', DETERMINISTIC)
def test_bb_deterministic(cuda, fmt):
    """Two runs, same inputs -> bit-identical iterates (fixed reduction order)."""
    from device import BBEngine
    from synthetic import make_shard, add_noise
    sh = make_shard(50_000, 2_500, 5_000, per_col=16, seed=3)
    b = add_noise(sh['Ax'], 0.02, seed=3)
    outs = []
    for _ in range(2):
        eng = BBEngine(sh['A'], b, sh['block_sizes'], options={'max_iter': 30, 'opt_tol': 1e-30},
                       **FORMATS[fmt])
        outs.append(eng.solve(poll=30).cpu().numpy().copy())
    assert np.array_equal(outs[0].view(np.int64), outs[1].view(np.int64))


@pytest.mark.parametrize('merge', ['1', '0'])
def test_k3_wave_pava_bit_exact(cuda, orc, monkeypatch, merge):
    """K3 alone (stage 4): z_new = clip01(PAVA_v1(z - t g)) and x = N z_new, bit for
    bit against the oracle, on blocks of 2..150 routes (wave packs -- two per
    wave sharing their later passes, or one -- and the paths for z-blocks
    longer than 64)."""
    import torch
    monkeypatch.setenv('BSLS_K3_MERGE', merge)
    monkeypatch.setenv('BSLS_K3_WARM', '0')      # the reference passes always
    import _native
    from device import BBEngine
    rs = np.random.RandomState(7)
    sizes = np.concatenate([rs.randint(2, 40, size=300), [66, 65, 130, 2, 150, 64, 3]])
    rs.shuffle(sizes)
    n = int(sizes.sum())
    m = 200
    A = sps.random(m, n, density=0.02, random_state=rs, format='csr')
    eng = BBEngine(A, rs.randn(m), sizes, options={'max_iter': 10, 'opt_tol': 1e-30})
    nz = eng.nz
    for trial in range(5):
        zc = np.cumsum(rs.rand(nz)) * 0.01 if trial == 0 else rs.randn(nz)
        g = rs.randn(nz) * (0.5 if trial < 2 else 50.0)
        if trial >= 3:
            # ties: runs of equal values (equal-valued chains must not pool,
            # and pooled runs meet equal neighbours), and signed zeros
            zc = np.round(rs.randn(nz), 0 if trial == 3 else 1)
            zc[rs.rand(nz) < 0.1] = -0.0
            g = np.zeros(nz)
        t = [1.0, 0.37, 3.0, 1.0, 1.0][trial]
        eng.z[0][:nz].copy_(torch.from_numpy(zc))
        eng.g[1][:nz].copy_(torch.from_numpy(g))
        sc = np.zeros(_native.S_COUNT)
        sc[_native.S_SUMDG] = 1.0
        sc[_native.S_DZDG] = t
        sc[_native.S_DGDG] = 1.0
        eng.scal.copy_(torch.from_numpy(sc))
        eng.stage(4, 1)
        got = eng.z[1][:nz].cpu().numpy()
        ref = zc - t * g
        zst = eng.layout.zstarts_h
        orc.isotonic_regression_multi_c(ref, zst)
        ref = np.maximum(np.minimum(ref, 1.0), 0.0)
        assert np.array_equal(got.view(np.int64), ref.view(np.int64)), trial
        xr = orc.block_sizes_to_N(sizes).dot(ref)
        assert np.array_equal(eng.x.cpu().numpy(), xr), trial
        # the dz = z - z_prev hand-off K3 writes for the next K2 (every block,
        # the serial > 64 path too)
        off = _native.load().bsls_bb_dz_offset(eng.m, eng.n, nz)
        dz = eng.work[off:off + 8 * nz].view(torch.float64).cpu().numpy()
        assert np.array_equal(dz.view(np.int64), (got - zc).view(np.int64)), trial


@pytest.mark.parametrize('merge', ['1', '0'])
def test_k3_warm_start_within_ulps(cuda, orc, monkeypatch, merge):
    """K3 with the warm start (pava_warm): blocks of 2..150 routes, both pack
    forms; repeated and slightly moved inputs (the kept partitions hold),
    then a moved and an unrelated input (they fail: repaired, the reference
    passes run from the runs that still hold, pava_warm_repair) -- every
    result within 1e-12 of the oracle's PAVA, x = N z exact on the kernel's z."""
    import torch
    monkeypatch.setenv('BSLS_K3_MERGE', merge)
    monkeypatch.setenv('BSLS_K3_WARM', '1')
    import _native
    from device import BBEngine
    rs = np.random.RandomState(11)
    sizes = np.concatenate([rs.randint(2, 40, size=300), [66, 65, 130, 2, 150, 64, 3]])
    rs.shuffle(sizes)
    n = int(sizes.sum())
    A = sps.random(200, n, density=0.02, random_state=rs, format='csr')
    eng = BBEngine(A, rs.randn(200), sizes, options={'max_iter': 10, 'opt_tol': 1e-30})
    assert eng.P.pava_warm == 1
    nz = eng.nz
    base, g = rs.randn(nz), rs.randn(nz) * 0.5
    res = []
    # (the last two with g = 0: coarse inputs with many exact ties, then a
    # few of them moved -- tied runs through the repair)
    coarse = np.round(base * 4) / 4
    g0 = np.zeros(nz)
    cases = [(base, g), (base, g), (base + 1e-7 * rs.randn(nz), g), (base + 0.05 * rs.randn(nz), g),
             (rs.randn(nz), g), (base, g), (coarse, g0), (coarse + 0.25 * (rs.rand(nz) < 0.1), g0)]
    for k, (zc, g) in enumerate(cases):
        eng.z[0][:nz].copy_(torch.from_numpy(zc))
        eng.g[1][:nz].copy_(torch.from_numpy(g))
        sc = np.zeros(_native.S_COUNT)
        sc[_native.S_SUMDG], sc[_native.S_DZDG], sc[_native.S_DGDG] = 1.0, 0.37, 1.0
        eng.scal.copy_(torch.from_numpy(sc))
        eng.stage(4, 1)
        got = eng.z[1][:nz].cpu().numpy()
        ref = zc - 0.37 * g
        orc.isotonic_regression_multi_c(ref, eng.layout.zstarts_h)
        ref = np.maximum(np.minimum(ref, 1.0), 0.0)
        assert np.max(np.abs(got - ref)) <= 1e-12, (k, np.max(np.abs(got - ref)))
        assert np.array_equal(eng.x.cpu().numpy(), orc.block_sizes_to_N(sizes).dot(got)), k
        res.append(np.array_equal(got, ref))
    assert res[0] and not res[1]          # cold: the reference passes; repeated: warm


@pytest.mark.parametrize('merge', ['0', '1'])
def test_k3_warm_repair_near_ties_many_iterations(cuda, orc, monkeypatch, merge):
    """the repair keeps a run pooled when its floating-point prefix
    test says it cannot be split, so a run splittable only by a rounding
    margin stays pooled.  K3 fed 40 inputs in a row on a coarse grid (exact
    ties) perturbed by ~1e-15 relative, each warm-started from the partition
    the previous call kept: every result within 1e-12 of the oracle's PAVA."""
    import torch
    monkeypatch.setenv('BSLS_K3_MERGE', merge)
    monkeypatch.setenv('BSLS_K3_WARM', '1')
    import _native
    from device import BBEngine
    rs = np.random.RandomState(17)
    sizes = np.concatenate([rs.randint(2, 40, size=300), [66, 130, 2, 64]])
    rs.shuffle(sizes)
    n = int(sizes.sum())
    A = sps.random(200, n, density=0.02, random_state=rs, format='csr')
    eng = BBEngine(A, rs.randn(200), sizes, options={'max_iter': 10, 'opt_tol': 1e-30})
    nz = eng.nz
    grid = np.round(rs.randn(nz) * 4) / 4
    g = np.zeros(nz)
    worst = 0.0
    for k in range(40):
        zc = grid * (1.0 + 1e-15 * rs.randn(nz)) + (1e-15 * rs.randn(nz) if k % 4 == 0 else 0.0)
        eng.z[0][:nz].copy_(torch.from_numpy(zc))
        eng.g[1][:nz].copy_(torch.from_numpy(g))
        sc = np.zeros(_native.S_COUNT)
        sc[_native.S_SUMDG], sc[_native.S_DZDG], sc[_native.S_DGDG] = 1.0, 0.37, 1.0
        eng.scal.copy_(torch.from_numpy(sc))
        eng.stage(4, 1)
        got = eng.z[1][:nz].cpu().numpy()
        ref = zc.copy()
        orc.isotonic_regression_multi_c(ref, eng.layout.zstarts_h)
        ref = np.maximum(np.minimum(ref, 1.0), 0.0)
        err = float(np.max(np.abs(got - ref)))
        worst = max(worst, err)
        assert err <= 1e-12, (k, err)
    assert worst < 1e-13, worst


def test_dense_row_network_falls_back_to_tiles(cuda, orc, monkeypatch, parity):
    """A 100k-route network with 8 links every route crosses: the panel image
    overflows, the engine takes the streamed tiles for A, and the iterates
    still follow the oracle; the x-space operator's residual walks its
    fixed-point tile image (f, g as SciPy's to 1e-12), and on the panels
    (BSLS_LSQ_K1=panels) it falls back to the CSR kernels."""
    from device import BBEngine
    from algorithm_utils import SparseLSQ
    from test_host import _dense_row_matrix
    A = _dense_row_matrix()
    rs = np.random.RandomState(4)
    sizes = rs.multinomial(A.shape[1] - 5000, np.ones(5000) / 5000) + 1
    x = np.concatenate([rs.dirichlet(np.ones(k)) for k in sizes])
    b = A.dot(x) * (1 + 0.02 * rs.randn(A.shape[0]))
    eng = BBEngine(A, b, sizes, options={'max_iter': 10, 'opt_tol': 1e-30})
    assert eng.fmt_A == 'tiles'
    rec = {}

    def log(i, s, dt):
        rec[i] = s
        return 0.0
    eng.solve(log=log, record_every=1, poll=1)
    ref = orc.bb_trace(A, b, sizes, 10, record_every=1)
    for i in (1, 5, 10):
        parity('bb_dense_row_%d' % i, rel_err(rec[i], ref[i]), 1e-12)
    op = SparseLSQ(A, b, panels=True)
    assert op.lsq is not None and op.lsq.k1 == 'tiles_fixed'
    xt = rs.rand(A.shape[1])
    gh = np.zeros(A.shape[1])
    f = op(xt, gh)                           # g written in place, as np.copyto
    tmp = A.dot(xt) - b
    assert abs(float(f) - 0.5 * tmp.dot(tmp)) <= 1e-12 * 0.5 * tmp.dot(tmp)
    gref = A.T.dot(tmp)
    assert np.max(np.abs(gh - gref)) <= 1e-10 * np.max(np.abs(gref))
    monkeypatch.setenv('BSLS_LSQ_K1', 'panels')
    assert SparseLSQ(A, b, panels=True).lsq is None


def test_bb_iterates_with_long_blocks_vs_oracle(cuda, orc, parity):
    """BB iterates over blocks of 66..300 routes (K3's serial path, and the dz it
    hands to the next K2 on that path) next to short ones, vs the oracle."""
    from device import BBEngine
    from synthetic import make_shard, add_noise
    rs = np.random.RandomState(12)
    sizes = np.concatenate([rs.randint(66, 300, 40), rs.randint(2, 20, 400)])
    rs.shuffle(sizes)
    n = int(sizes.sum())
    sh = make_shard(n + 1000, 100, 3_000, per_col=16, seed=12)
    A = sh['A'][:, :n].tocsr()
    b = add_noise(A.dot(rs.rand(n)), 0.02, seed=12)
    eng = BBEngine(A, b, sizes, options={'max_iter': 15, 'opt_tol': 1e-30})
    rec = {}

    def log(i, s, dt):
        rec[i] = s
        return 0.0
    eng.solve(log=log, record_every=1, poll=1)
    ref = orc.bb_trace(A, b, sizes, 15, record_every=1)
    for i in (1, 2, 5, 15):
        parity('bb_long_blocks_%d' % i, rel_err(rec[i], ref[i]), 1e-12)


@pytest.mark.parametrize('codec', ['f16', 'f32', 'f64'])
def test_stored_value_codecs_vs_oracle(cuda, orc, codec, parity):
    """Stored-value (general) dealt images: values that convert to _Float16 /
    float exactly travel as such (BSLS_TILE_VAL16 / VAL32: 2 / 4 bytes instead
    of 8, widened back to the same doubles in the walk), any other as doubles.
    The three codecs on the same pattern: BB iterates at 1, 5, 20 against the
    oracle (SciPy over the same doubles) within 1e-12, and K2 to 1e-12."""
    import torch
    from device import BBEngine
    from synthetic import make_shard, add_noise
    sh = make_shard(60_000, 3_000, 6_000, per_col=16, seed=19)
    A = sh['A'].copy()
    if codec == 'f32':
        A.data = A.data * (1.0 + 2.0 ** -12)          # <= 22 bits: exact in float, not in _Float16
    elif codec == 'f64':
        A.data = A.data * (1.0 + np.random.RandomState(3).rand(A.nnz) * 1e-3)
    A = sps.csr_matrix(A)
    b = add_noise(A.dot(sh['x_true']), 0.02, seed=19)
    ref = orc.bb_trace(A, b, sh['block_sizes'], 20, record_every=1)
    eng = BBEngine(A, b, sh['block_sizes'], options={'max_iter': 20, 'opt_tol': 1e-30},
                   general=True, fmt='tiles')
    assert eng.A_til.val_codec == codec and eng.AT_til.val_codec == codec
    rec = {}

    def log(i, s, dt):
        rec[i] = s
        return 0.0
    eng.solve(log=log, record_every=1, poll=1)
    for i in (1, 5, 20):
        parity('bb_codec_%s_%d' % (codec, i), rel_err(rec[i], ref[i]), 1e-12)
    r = np.random.RandomState(5).randn(eng.m)
    eng.r.copy_(torch.from_numpy(r))
    eng.stage(3, 0)
    got = eng.g[0][:eng.nz].cpu().numpy()
    N = orc.block_sizes_to_N(sh['block_sizes'])
    want = N.T.tocsr().dot(A.T.tocsr().dot(r))
    assert np.max(np.abs(got - want)) <= 1e-12 * np.max(np.abs(want))


def test_sy_dr_retired(cuda, shard100k):
    """bsls_bb_problem.sy_dr is reserved since round 6 (dz . dg from the
    residuals moved the reference's exact-zero exit, BB.py:22): a nonzero
    value is refused (BSLS_E_ARG) before anything is launched."""
    from device import BBEngine
    sh, b, _ = shard100k
    eng = BBEngine(sh['A'], b, sh['block_sizes'], options={'max_iter': 3, 'opt_tol': 1e-30})
    eng.set_z0(np.zeros(eng.nz))
    eng.P.sy_dr = 1
    with pytest.raises(ValueError):
        eng.prologue()
    eng.P.sy_dr = 0
    eng.prologue()
    eng.iterate(1, 3)
