"""Column-sharded BB orchestration (distributed.ShardedBB) on 2 gloo ranks (CPU).

The GPU stages are replaced by a NumPy test double that implements each stage's
contract from include/bsls_hip.h (bsls_bb_stage) with the oracle's PAVA, so
what is tested is the sharding: block-aligned column split, the r all-reduce,
the four-sum all-reduce and the stage order.  The sharded run must reproduce
the unsharded run and the oracle's BB trajectory (python/BB.py semantics).
"""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, 'block-simplex-least-squares_amd')


class FakeStages:
    """NumPy model of bsls_bb_stage for one column shard."""

    def __init__(self, A, AT, sizes, target, orc, max_iter, fold=True):
        self.A, self.AT, self.sizes, self.target = A, AT, np.asarray(sizes), target
        # fold: K1 adds its column groups' sums by atomics into an r that
        # stage 15 (the K3 before it) initialised -- a column shard's dealt K1
        # with several groups (csrc/bb.hip k1_init_folded); else stage 15 / 14
        # are stages 13 / 1
        self.fold = fold
        self.orc, self.max_iter = orc, max_iter
        self.n = int(self.sizes.sum())
        self.nz = self.n - len(self.sizes)
        self.xst = np.concatenate(([0], np.cumsum(self.sizes)[:-1]))
        self.zst = self.xst - np.arange(len(self.sizes))
        self.z = [np.zeros(self.nz), np.zeros(self.nz)]
        self.g = [np.zeros(self.nz), np.zeros(self.nz)]
        self.x = np.zeros(self.n)
        self.r = torch.zeros(A.shape[0], dtype=torch.float64)
        self.scal = torch.zeros(16, dtype=torch.float64)
        self.role = 0

    def set_shard_role(self, role):
        self.role = role

    rr_lo = rr_hi = 0

    def set_rr_slice(self, lo, hi):
        self.rr_lo, self.rr_hi = lo, hi

    def Nz(self, z):
        out = np.empty(self.n)
        for b, (xs, k) in enumerate(zip(self.xst, self.sizes)):
            zb = z[self.zst[b]:self.zst[b] + k - 1]
            prev = np.concatenate(([0.0], zb))
            out[xs:xs + k] = np.concatenate((zb, [0.0])) - prev
        return out

    def Ntw(self, w):
        g = np.empty(self.nz)
        for b, (xs, k) in enumerate(zip(self.xst, self.sizes)):
            g[self.zst[b]:self.zst[b] + k - 1] = w[xs:xs + k - 1] - w[xs + 1:xs + k]
        return g

    ROWS = 97   # rows per K1 row block (residual_rows granule)

    def row_blocks(self):
        return -(-self.A.shape[0] // self.ROWS), self.ROWS

    def _partial(self, it, r0, r1):
        """stage 1 on rows [r0, r1): A_g x_g (+ target with role 1); once
        stopped, role 2 writes 0 and role 1 keeps r (bsls_bb_problem.shard_role)."""
        if it > 0 and float(self.scal[0]) != 0:
            if self.role == 2:
                self.r[r0:r1] = 0.0
            return
        v = self.A[r0:r1].dot(self.x)
        if self.role == 1:
            v = v + self.target[r0:r1]
        self.r[r0:r1] = torch.from_numpy(v)

    def _init_r(self):
        """stage 15's r initialisation (bb_k3 kinit): target on role 1, 0 on
        role 2; once stopped role 1 keeps r and role 2 writes 0."""
        if float(self.scal[0]) != 0:
            if self.role == 2:
                self.r.zero_()
            return
        self.r[:] = torch.from_numpy(self.target.copy()) if self.role == 1 else 0.0

    def _add_partial(self, it):
        """stage 14 after a folding stage 15: the groups' sums add into r
        (nothing once stopped: stage 15 already left r as it must be)."""
        if float(self.scal[0]) != 0:
            return
        self.r += torch.from_numpy(self.A.dot(self.x))

    # link parts (bsls_bb_k2_part / bsls_bb_k1_rows): K2 by column groups over
    # K1's row-block parts; set by _run(link=True)
    k1_part_bounds = None

    def _rows_of(self, q):
        lb = self.k1_part_bounds
        return lb[q] * self.ROWS, min(lb[q + 1] * self.ROWS, self.A.shape[0])

    def k2_part(self, it, q):
        """stage 10 on link part q: its partial route sums A_q' r_q and its
        slice of ||r||^2 (only ITS rows of r are read); the last part adds the
        earlier ones and runs N' and the sums."""
        s = self.scal
        last = q == len(self.k1_part_bounds) - 2
        if it > 0 and float(s[0]) != 0:
            if last:
                self._stopped_sums(10)
            return
        r0, r1 = self._rows_of(q)
        rq = self.r.numpy()[r0:r1]
        wq = self.AT[:, r0:r1].dot(rq)
        lo, hi = (self.rr_lo, self.rr_hi) if self.rr_hi > self.rr_lo else (0, self.A.shape[0])
        a, b = max(lo, r0), min(hi, r1)
        rrq = float(np.dot(self.r.numpy()[a:b], self.r.numpy()[a:b])) if b > a else 0.0
        self._w = wq if q == 0 else self._w + wq
        self._rr = rrq if q == 0 else self._rr + rrq
        if not last:
            return
        zc, zn = (it - 1) & 1, it & 1
        g = self.Ntw(self._w)
        self.g[zn][:] = g
        dg = g - self.g[zc]
        dz = self.z[zc] - self.z[zn]
        s[11:15] = s[5:9].clone()
        s[9] = self._rr
        s[5], s[6], s[7], s[8] = dg.sum(), dz.dot(dg), dg.dot(dg), g.dot(g)

    def k1_rows(self, it, rb0, rb1):
        """stage 14 on row blocks [rb0, rb1)."""
        r0, r1 = rb0 * self.ROWS, min(rb1 * self.ROWS, self.A.shape[0])
        if not self.fold:
            self._partial(it, r0, r1)
            return
        if float(self.scal[0]) != 0:
            return
        self.r[r0:r1] += torch.from_numpy(self.A[r0:r1].dot(self.x))

    def _stopped_sums(self, k):
        """K2 of a stopped run (k2_stopped_sums): role 2 zeroes the sums the
        driver all-reduces next, so the sum keeps role 1's."""
        if self.role == 2:
            self.scal[5:10 if k == 10 else 9] = 0.0

    def residual_rows(self, it, rb0, rb1):
        self._partial(it, rb0 * self.ROWS, min(rb1 * self.ROWS, self.A.shape[0]))

    def _record(self, it):
        """||r||^2, f and the stopping test of iteration it (stage 9)."""
        s = self.scal
        if it > 0 and float(s[0]) != 0:
            return
        rr = float(self.r.dot(self.r))
        s[4], s[9] = 0.5 * np.sqrt(rr) ** 2, rr
        if it > 0:
            s[1], s[2] = it, it & 1
            if it >= self.max_iter:
                s[0] = 2

    def stage(self, k, it):
        s = self.scal
        zc, zn = (it - 1) & 1, it & 1
        if k == 0:
            s.zero_()
        elif k == 1:
            self._partial(it, 0, self.A.shape[0])
        elif k == 9:
            self._record(it)
        elif k == 14:
            if self.fold:
                self._add_partial(it)
            else:
                self._partial(it, 0, self.A.shape[0])
        elif k == 15:             # stage 13 with stage 14's r initialisation
            self.stage(12, it)
            if self.fold:
                self._init_r()
            self.stage(4, it)
        elif k in (3, 8, 10):
            if it > 0 and float(s[0]) != 0:
                self._stopped_sums(k)
                return
            g = self.Ntw(self.AT.dot(self.r.numpy()))
            if it == 0:
                self.g[0][:] = g
                return
            self.g[zn][:] = g
            dg = g - self.g[zc]
            dz = self.z[zc] - self.z[zn]
            if k == 8:
                self._record(it - 1)     # before this iteration's sums land
                if float(s[0]) != 0:     # stopped at it - 1: its sums stay
                    self._stopped_sums(k)
                    return
            if k == 10:
                s[11:15] = s[5:9].clone()            # iteration it - 1's sums, for stage 12
                rs = self.r[self.rr_lo:self.rr_hi] if self.rr_hi > self.rr_lo else self.r
                s[9] = float(rs.dot(rs))             # this rank's slice of ||r||^2
            s[5], s[6], s[7], s[8] = dg.sum(), dz.dot(dg), dg.dot(dg), g.dot(g)
        elif k == 13:             # stage 12 then stage 4 (K3 with the record folded in)
            self.stage(12, it)
            self.stage(4, it)
        elif k == 12:
            # f / stopping test of it - 1 from the all-reduced ||r||^2 (s[9])
            p = it - 1
            if p > 0 and float(s[0]) != 0:
                return
            rr = float(s[9])
            s[4] = 0.5 * np.sqrt(rr) ** 2
            if p > 0:
                s[1], s[2] = p, p & 1
                if p >= self.max_iter:
                    s[0] = 2
                    s[5:9] = s[11:15].clone()
        elif k == 4:
            if float(s[0]) != 0:
                return
            t = float(s[6]) / float(s[7])
            y = self.z[zc] - t * self.g[zn]
            self.orc.isotonic_regression_multi_c(y, self.zst)
            self.z[zn][:] = np.maximum(np.minimum(y, 1.0), 0.0)
            self.x = self.Nz(self.z[zn])
        elif k == 5:
            self.z[1][:] = self.z[0] + 1
            self.x = self.Nz(self.z[1])
        elif k == 6:
            self.x = self.Nz(self.z[0])


def _problem():
    sys.path.insert(0, PKG)
    from synthetic import make_shard, add_noise
    sh = make_shard(6_000, 300, 800, per_col=8, seed=21)
    b = add_noise(sh['Ax'], 0.02, seed=21)
    return sh, b


class _Done:
    def wait(self):
        pass


def _run(rank, world, iters, out_q, parts=1, stop_at=None, fold=True, link=False):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, PKG)
    from oracle import oracle as orc
    from distributed import ShardedBB, partition_blocks
    if world > 1:
        dist.init_process_group('gloo', rank=rank, world_size=world)
        red = lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM)
        red_async = lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)
    else:
        red = lambda t: None
        red_async = lambda t: _Done()
    sh, b = _problem()
    sizes = sh['block_sizes']
    bounds = partition_blocks(sizes, sizes * 8.0, world)
    xst = np.concatenate(([0], np.cumsum(sizes)))
    c0, c1 = xst[bounds[rank]], xst[bounds[rank + 1]]
    A_g = sh['A'][:, c0:c1].tocsr()
    sz_g = sizes[bounds[rank]:bounds[rank + 1]]
    x0 = np.zeros(c1 - c0)
    x0[np.cumsum(sz_g) - 1] = 1.0
    part = torch.from_numpy(A_g.dot(x0))
    red(part)
    target = part.numpy() - b
    eng = FakeStages(A_g, A_g.T.tocsr(), sz_g, target, orc, stop_at or iters, fold=fold)
    if link:
        from distributed import row_parts
        eng.k1_part_bounds = np.array(row_parts(eng.row_blocks()[0], parts))
    drv = ShardedBB(eng, red, parts=parts, all_reduce_async=red_async, rank=rank)
    assert drv.link == link
    drv.prologue()
    traj = {}
    for i in range(1, iters + 1):
        drv.iterate(i, 1)
        traj[i] = eng.z[i & 1].copy()
    res = {k: v for k, v in traj.items() if k in (1, 5, iters)}
    if stop_at:
        res['r'] = eng.r.numpy().copy()
        res['scal'] = eng.scal.numpy().copy()
    out_q.put((rank, res))
    if world > 1:
        dist.destroy_process_group()


def _spawn(world, iters, parts=1, stop_at=None, fold=True, link=False):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(29500 + (os.getpid() % 1000) + 7 * parts + (stop_at or 0)
                                    + 3 * int(fold) + 41 * int(link))
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_run, args=(r, world, iters, q, parts, stop_at, fold, link))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if stop_at:
        return res
    return {i: np.concatenate([res[r][i] for r in range(world)]) for i in res[0]}


@pytest.mark.timeout(600)
@pytest.mark.parametrize('fold', [True, False])
def test_two_rank_sharded_bb_matches_single_and_oracle(orc, fold):
    iters = 20
    one = _spawn(1, iters, fold=fold)
    two = _spawn(2, iters, fold=fold)
    for i in one:
        d = np.max(np.abs(one[i] - two[i])) / max(1.0, np.max(np.abs(one[i])))
        assert d < 1e-10, (i, d)
    sh, b = _problem()
    ref = orc.bb_trace(sh['A'], b, sh['block_sizes'], iters, record_every=1)
    for i in one:
        d = np.max(np.abs(two[i] - ref[i])) / max(1.0, np.max(np.abs(ref[i])))
        assert d < 1e-8, (i, d)


@pytest.mark.timeout(600)
def test_two_rank_overlapped_residual_matches_single(orc):
    """The residual all-reduced in 3 row parts, asynchronously, behind K1's
    row parts (ShardedBB parts > 1): same trajectory as the single rank."""
    iters = 12
    one = _spawn(1, iters)
    three = _spawn(2, iters, parts=3)
    for i in one:
        d = np.max(np.abs(one[i] - three[i])) / max(1.0, np.max(np.abs(one[i])))
        assert d < 1e-10, (i, d)


@pytest.mark.timeout(600)
@pytest.mark.parametrize('fold', [True, False])
def test_two_rank_stop_keeps_final_residual(orc, fold):
    """Iterations enqueued past the stop (max_iter 5, 9 enqueued) leave r the
    final residual on both ranks -- rank 0 keeps its r, rank 1 writes 0 before
    each all-reduce (in stage 15's r initialisation where it folds, fold=True,
    the library's choice for a dealt K1 with several column groups; in stage
    1 / 14 otherwise) -- the stop is reported at iteration 5 on both, and the
    BB sums stay iteration 5's (rank 1 zeroes its copy before each five-sum
    all-reduce past the stop, k2_stopped_sums, instead of doubling them)."""
    one = _spawn(1, 9, stop_at=5, fold=fold)
    two = _spawn(2, 9, stop_at=5, fold=fold)
    r1 = one[0]['r']
    for rank in (0, 1):
        assert two[rank]['scal'][0] == 2 and two[rank]['scal'][1] == 5
        d = np.max(np.abs(two[rank]['r'] - r1)) / max(1.0, np.max(np.abs(r1)))
        assert d < 1e-10, (rank, d)
        s1, s2 = one[0]['scal'][5:9], two[rank]['scal'][5:9]
        assert np.max(np.abs(s2 - s1)) <= 1e-9 * max(1.0, np.max(np.abs(s1))), (rank, s1, s2)


@pytest.mark.timeout(600)
@pytest.mark.parametrize('fold', [True, False])
def test_two_rank_link_parts_match_single(orc, fold):
    """The exchange pipelined behind both walks (link parts: K1 by 3 row-block
    parts, each part's rows of r all-reduced asynchronously, the next K2 by the
    matching column groups, part q waiting only for its own exchange and
    reading only its rows of r): the single rank's trajectory, and the stop
    (max_iter 5 of 9 enqueued) with the stop iteration's r and sums."""
    iters = 12
    one = _spawn(1, iters, fold=fold)
    three = _spawn(2, iters, parts=3, fold=fold, link=True)
    for i in one:
        d = np.max(np.abs(one[i] - three[i])) / max(1.0, np.max(np.abs(one[i])))
        assert d < 1e-10, (i, d)
    ref = _spawn(1, 9, stop_at=5, fold=fold)
    two = _spawn(2, 9, parts=3, stop_at=5, fold=fold, link=True)
    r1, s1 = ref[0]['r'], ref[0]['scal'][5:9]
    for rank in (0, 1):
        assert two[rank]['scal'][0] == 2 and two[rank]['scal'][1] == 5
        assert np.max(np.abs(two[rank]['r'] - r1)) <= 1e-10 * max(1.0, np.max(np.abs(r1)))
        assert np.max(np.abs(two[rank]['scal'][5:9] - s1)) <= 1e-9 * max(1.0, np.max(np.abs(s1)))


@pytest.mark.timeout(600)
def test_two_rank_unfused_schedule(orc, monkeypatch):
    """The three schedules (BSLS_SHARD_FUSE=2, the default: stage 10's sliced
    ||r||^2 all-reduced with the sums and stage 12's stop test; 1: stage 8's
    fused test; 0: stage 3 and a stage-9 test after every exchange): the same
    trajectory, and the same stop."""
    iters = 10
    fused = _spawn(2, iters)                    # the sliced schedule (fuse 2, default)
    base = _spawn(2, 9, stop_at=5)
    for rank in (0, 1):
        assert base[rank]['scal'][0] == 2 and base[rank]['scal'][1] == 5
    s5 = base[0]['scal'][5:9]
    for mode in ('0', '1'):
        monkeypatch.setenv('BSLS_SHARD_FUSE', mode)
        plain = _spawn(2, iters)
        for i in fused:
            d = np.max(np.abs(fused[i] - plain[i])) / max(1.0, np.max(np.abs(fused[i])))
            assert d < 1e-12, (mode, i, d)
        two = _spawn(2, 9, stop_at=5)
        for rank in (0, 1):
            assert two[rank]['scal'][0] == 2 and two[rank]['scal'][1] == 5, mode
            # the stopping iteration's sums stay in scal whatever the schedule
            d = np.max(np.abs(two[rank]['scal'][5:9] - s5)) / max(1.0, np.max(np.abs(s5)))
            assert d < 1e-9, (mode, rank, d)
        monkeypatch.delenv('BSLS_SHARD_FUSE')


def test_row_parts():
    sys.path.insert(0, PKG)
    from distributed import row_parts
    assert row_parts(10, 3) == [0, 3, 7, 10]
    assert row_parts(2, 5) == [0, 1, 2]
    assert row_parts(7, 1) == [0, 7]


def test_partitioned_problem_is_world_independent():
    """synthetic.make_partitioned (config C5's generator): the shards of every
    world size concatenate to the same matrix, x_true and block sizes, and the
    partial products sum to the same b."""
    sys.path.insert(0, PKG)
    import scipy.sparse as sps
    from synthetic import make_partitioned
    full = make_partitioned(60_000, 3_000, 5_000, gen_chunks=8)
    for world in (2, 3):
        sh = [make_partitioned(60_000, 3_000, 5_000, rank=r, world=world, gen_chunks=8)
              for r in range(world)]
        A = sps.hstack([q['A'] for q in sh]).tocsr()
        A.sort_indices()
        assert (A != full['A']).nnz == 0
        assert np.array_equal(np.concatenate([q['x_true'] for q in sh]), full['x_true'])
        assert np.array_equal(np.concatenate([q['block_sizes'] for q in sh]),
                              full['block_sizes'])
        assert [q['col0'] for q in sh] == list(np.cumsum([0] + [q['n'] for q in sh])[:-1])
        b = sum(q['Ax'] for q in sh)
        assert np.max(np.abs(b - full['Ax'])) <= 1e-12 * np.max(np.abs(full['Ax']))
        # scaled incidence: every stored entry of column j is colv[j]
        for q in sh:
            C = q['A'].tocsc()
            assert np.array_equal(C.data, np.repeat(q['colv'], np.diff(C.indptr)))


class _FxEngine:
    """Just what ShardedBB._fix_r reads: whether this rank's engine can keep r
    in fixed point, and the bound's inputs."""

    def __init__(self, rank, ok):
        import scipy.sparse as sps
        self._ok = ok
        self._A_host = sps.csr_matrix(np.array([[1.0, 2.0], [0.0, 3.0 + rank]]))
        self.r = torch.zeros(2, dtype=torch.float64)
        self.target = torch.tensor([0.5, -4.0], dtype=torch.float64)
        self.z0 = torch.zeros(3, dtype=torch.float64)
        self.scale = None

    def fixed_r_ok(self):
        return self._ok

    def set_r_fixed(self, s):
        self.scale = s


def _fx_run(rank, world, port, q, oks):
    sys.path.insert(0, PKG)
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from distributed import ShardedBB
    e = _FxEngine(rank, oks[rank])
    drv = ShardedBB.__new__(ShardedBB)        # only the fixed-point decision
    drv.e, drv._rank = e, rank
    drv.all_reduce = lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM)
    drv._fix_r()
    # the ranks still agree on every later collective
    t = torch.ones(1, dtype=torch.float64)
    dist.all_reduce(t)
    q.put((rank, e.scale, float(t.item())))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize('oks', [(True, False), (False, True), (True, True)])
def test_fixed_point_r_is_a_collective_choice(oks):
    """fixed_r_ok depends on each rank's own shard, so the choice
    is all-reduced -- fixed point only when every rank can take it, the same
    scale on every rank; otherwise every rank keeps doubles (no rank skips
    the others' all-reduces, no int64 words summed into doubles)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 31000 + (os.getpid() % 900) + 11 * (oks[0] + 2 * oks[1])
    ps = [ctx.Process(target=_fx_run, args=(r, 2, port, q, oks)) for r in range(2)]
    for p in ps:
        p.start()
    res = {item[0]: item[1:] for item in (q.get(timeout=120) for _ in ps)}
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] == res[1][1] == 2.0
    if all(oks):
        # B = max(|target| + 2 (max|z0| + 1) sum over ranks of |A| row sums)
        #   = max(0.5 + 2 * 6, 4 + 2 * 7) = 18 -> 2^(61 - 5)
        assert res[0][0] == res[1][0] == 2.0 ** 56
    else:
        assert res[0][0] is None and res[1][0] is None
