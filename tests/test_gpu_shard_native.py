"""The native sharded driver at world 2 (bsls_bb_shard_iterate, csrc/shard.hip),
i.e. the schedule bench.py ships at N > 1, on one MI355X.

RCCL refuses two ranks on one device, so the two ranks share the GPU and
their all-reduces go through gloo: distributed.CallbackComm hands the C++
loop a host callback (bsls_comm_create_callback) in place of RCCL.  That
runs the driver's world > 1 branch as shipped -- stage 10, the five-sum
all-reduce, stage 15 (K3 + the atomic K1's r initialisation: target on
shard_role 1, 0 on shard_role 2), stage 14 (the atomic K1), the r
all-reduce -- with both shard roles.  The reference has no parallel code
(SURVEY.md §2); the split is blockify's contiguous blocks
(python/bsls_matrices.py:109-126) and the oracle is the
one-process BB trajectory (python/BB.py:7-45 over main.py:53-65).

* iterates at 1 / 5 / 20 on make_partitioned's C5-density 2-way split
  (1.2M routes, 120k links: the entries-per-link density of an 8-way C5
  shard) against the oracle;
* the stop: iterations enqueued past max_iter change nothing, r stays the
  final residual and the BB sums stay the stop iteration's on both ranks;
* convergence (python/BB.py:21-24, tests/fast/test_main.py:31-47): the three
  tests/fast problems run to their own exit on the sharded driver (atomic
  K1: run-dependent summation order) -- 0.5||Ax - b||^2 < 1e-16 and the exit
  iteration within the band the one-GPU test holds around the reference's
  454 / 569 / 745.

The atomic K1 keeps r in 64-bit fixed point on a shard (bsls_bb_problem.r_fx,
distributed.ShardedBB._fix_r): its groups' sums add as integers and the r
exchange sums int64 words, so neither the order the groups land in nor the
rank count changes r's bits -- what lets a converged run reach BB.py:22's
exact-zero sum(delta_g) where the one-GPU run does (float atomics moved one
problem's exit from ~770 to 874 iterations, gpurun_out/r5a_shard.log).
Tolerance: 1e-12 per element (|d| <= 1e-12 max(1, |ref|)) at these
iteration counts -- what the runs measure (~1e-15, profiles/
r06_parity_errors.jsonl) with room for the dealt tiles' LDS atomics, which
still sum each tile's rows in a run-dependent order; the north star allows
1e-6.
"""
import argparse
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, 'block-simplex-least-squares_amd')
SEED = 237423433

N5, P5, M5 = 1_200_000, 60_000, 120_000
CHECK5 = (1, 5, 20)
TOL = 1e-12


def elem_err(a, b):
    """max over elements of |a - b| / max(1, |b|)."""
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b))))


def _setup(rank, world, port):
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)


def _engine(A_g, sizes_g, b, x0_g, max_iter, early_exit, **kw):
    """The rank's BBEngine with target = sum over ranks of A_g x0_g - b."""
    import torch
    import torch.distributed as dist
    from device import BBEngine
    part = torch.from_numpy(A_g.dot(x0_g))
    dist.all_reduce(part)
    target = torch.from_numpy(part.numpy() - b).cuda()
    eng = BBEngine(A_g, None, sizes_g, options={'max_iter': max_iter, 'opt_tol': 1e-30},
                   early_exit=early_exit, target=target, **kw)
    return eng


def _driver(eng, rank):
    from distributed import ShardedBB, CallbackComm, torch_all_reduce
    comm = CallbackComm(torch_all_reduce(), rank=rank, engine=eng)
    drv = ShardedBB(eng, torch_all_reduce(), rank=rank, native=comm)
    assert drv.native is comm and drv.fuse == 2
    return drv, comm


def _finish(comm):
    import torch
    import torch.distributed as dist
    torch.cuda.synchronize()
    comm.close()
    dist.barrier()
    dist.destroy_process_group()


def _run_c5(rank, world, port, out_q):
    _setup(rank, world, port)
    import torch
    from synthetic import make_partitioned
    full = make_partitioned(N5, P5, M5)
    sh = make_partitioned(N5, P5, M5, rank=rank, world=world)
    x0 = np.zeros(sh['n'])
    x0[np.cumsum(sh['block_sizes']) - 1] = 1.0
    eng = _engine(sh['A'], sh['block_sizes'], full['Ax'], x0, 10 ** 9, False,
                  AT=sh['AT'], colv=sh['colv'])
    eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))
    drv, comm = _driver(eng, rank)
    drv.prologue()
    traj = {}
    done = 0
    for i in CHECK5:
        drv.iterate(done + 1, i - done)          # several iterations per C++ call
        done = i
        traj[i] = eng.current_z(i & 1).cpu().numpy().copy()
    info = dict(role=int(eng.P.shard_role), groups=int(eng.A_til.img['ngroups']),
                fmt=(eng.fmt_A, eng.fmt_AT), r_fx=float(eng.P.r_fx))
    out_q.put((rank, traj, info))
    _finish(comm)


def _spawn(target, world, *args, timeout=600):
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 32100 + (os.getpid() % 700) + 7 * len(target.__name__)
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time
    res = {}
    t_end = time.time() + timeout
    while len(res) < len(procs):
        # a rank that died (an exception before its put) fails the test now,
        # instead of after the whole timeout on the queue
        try:
            item = q.get(timeout=5)
            res[item[0]] = item[1:]
            continue
        except queue.Empty:
            pass
        dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
        if dead or time.time() > t_end:
            for p in procs:
                if p.is_alive():
                    p.kill()
            raise AssertionError('rank processes failed (exit codes %s) or timed out'
                                 % [p.exitcode for p in procs])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


@pytest.mark.timeout(900)
def test_native_driver_two_ranks_c5_density_vs_oracle(cuda, orc, parity):
    from synthetic import make_partitioned
    res = _spawn(_run_c5, 2)
    for r in (0, 1):
        traj, info = res[r]
        # both shard roles, the C5 kernels, a K1 with several column groups
        # (so K1 adds by atomics into the r stage 15 initialised)
        assert info['role'] == (1 if r == 0 else 2)
        assert info['fmt'] == ('tiles', 'tiles') and info['groups'] > 1, info
        assert info['r_fx'] > 0, info          # r in fixed point (bsls_bb_problem.r_fx)
    full = make_partitioned(N5, P5, M5)
    ref = orc.bb_trace(full['A'], full['Ax'], full['block_sizes'], max(CHECK5), record_every=1)
    for i in CHECK5:
        got = np.concatenate([res[0][0][i], res[1][0][i]])
        parity('shard_native_c5dens_%d' % i, elem_err(got, ref[i]), TOL)


# ---- the stop ---------------------------------------------------------------

def _small():
    from synthetic import make_partitioned, add_noise
    kw = dict(per_col=8, seed=33, gen_chunks=8)
    full = make_partitioned(40_000, 2_000, 3_000, **kw)
    return full, add_noise(full['Ax'], 0.02, seed=33), kw


def _run_stop(rank, world, port, out_q, max_iter, enq):
    _setup(rank, world, port)
    import torch
    from synthetic import make_partitioned
    full, b, kw = _small()
    sh = make_partitioned(40_000, 2_000, 3_000, rank=rank, world=world, **kw)
    x0 = np.zeros(sh['n'])
    x0[np.cumsum(sh['block_sizes']) - 1] = 1.0
    eng = _engine(sh['A'], sh['block_sizes'], b, x0, max_iter, True, fmt='tiles')
    eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))
    drv, comm = _driver(eng, rank)
    drv.prologue()
    drv.iterate(1, enq)
    s = eng.scalars()
    zb = int(s[2])
    out_q.put((rank, dict(z=eng.current_z(zb).cpu().numpy().copy(),
                          r=eng.residual_value().cpu().numpy().copy(),
                          scal=s.copy(), groups=int(eng.A_til.img['ngroups']))))
    _finish(comm)


@pytest.mark.timeout(600)
def test_native_driver_two_ranks_stop(cuda, orc, parity):
    """max_iter 7, 30 iterations enqueued in one C++ call: both ranks report the
    stop at 7 with iteration 7's z, r = the residual of z_7 on both (role 1
    keeps its r, role 2 writes 0 in stage 15), and the BB sums of iteration 7
    on both (role 2 zeroes its copy before each all-reduce past the stop)."""
    res = _spawn(_run_stop, 2, 7, 30)
    full, b, _ = _small()
    sizes = full['block_sizes']
    ref = orc.bb_trace(full['A'], b, sizes, 7, record_every=1)
    z = np.concatenate([res[0][0]['z'], res[1][0]['z']])
    parity('shard_native_stop_7', elem_err(z, ref[7]), TOL)
    from bsls_utils import particular_x0, block_sizes_to_N
    r7 = full['A'].dot(particular_x0(sizes) + block_sizes_to_N(sizes).dot(ref[7])) - b
    s0 = res[0][0]['scal']
    for r in (0, 1):
        d = res[r][0]
        assert d['groups'] > 1
        assert d['scal'][0] == 2 and d['scal'][1] == 7, d['scal'][:3]
        assert np.max(np.abs(d['r'] - r7)) <= 1e-9 * max(1.0, np.max(np.abs(r7)))
        # every rank holds the same summed sums -- not world^k times them
        assert np.array_equal(d['scal'][5:9], s0[5:9]), (d['scal'][5:9], s0[5:9])
    # ... and they are iteration 7's: the one-GPU engine's sums at its stop
    from device import BBEngine
    one = BBEngine(full['A'], b, sizes, options={'max_iter': 7, 'opt_tol': 1e-30}, fmt='tiles')
    one.solve(poll=30)
    s1 = one.scalars()
    assert s1[0] == 2 and s1[1] == 7
    assert elem_err(s0[5:9], s1[5:9]) < 1e-8, (s0[5:9], s1[5:9])


# ---- convergence to the reference's own exit ---------------------------------

def _run_exit(rank, world, port, out_q, path):
    _setup(rank, world, port)
    import torch
    from distributed import partition_blocks
    P = np.load(path)
    import scipy.sparse as sps
    A = sps.csr_matrix((P['data'], P['indices'], P['indptr']), shape=tuple(P['shape']))
    b, sizes, x0 = P['b'], P['sizes'], P['x0']
    bounds = partition_blocks(sizes, sizes.astype(np.float64), world)
    xst = np.concatenate(([0], np.cumsum(sizes)))
    c0, c1 = xst[bounds[rank]], xst[bounds[rank + 1]]
    A_g = A[:, c0:c1].tocsr()
    sz_g = sizes[bounds[rank]:bounds[rank + 1]]
    # main.py's options (gradient_descent.py:29-31); early exits on
    eng = _engine(A_g, sz_g, b, x0[c0:c1], 300000, True, fmt='tiles')
    eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))   # x2z(particular_x0) = 0
    drv, comm = _driver(eng, rank)
    drv.prologue()
    i = 0
    while True:
        drv.iterate(i + 1, 25)
        i += 25
        s = eng.scalars()
        if s[0] != 0 or i >= 300000:
            break
    out_q.put((rank, dict(z=eng.current_z(int(s[2])).cpu().numpy().copy(), scal=s.copy(),
                          groups=int(eng.A_til.img['ngroups']), role=int(eng.P.shard_role),
                          r_fx=float(eng.P.r_fx))))
    _finish(comm)


@pytest.mark.timeout(900)
@pytest.mark.parametrize('vi', [0, 1, 2])
def test_native_driver_two_ranks_runs_to_exit(cuda, golden, tmp_path, vi):
    import bsls_utils
    from bsls_matrices import BSLSMatrices
    from bsls_utils import particular_x0, block_sizes_to_N
    G = golden('solvers.npz')
    kw = [{}, {'alpha': 0.5}, {'A_sparse': 0.05}][vi]
    np.random.seed(SEED)
    fname = os.path.join(str(tmp_path), 'test_main.mat')
    bsls_utils.generate_data(fname=fname, **kw)
    bm = BSLSMatrices(fname=fname, full=True, L=True, OD=True, CP=True, LP=True, eq='CP',
                      init=False)
    bm.degree_reduced_form()
    AA, bb, N, sizes, x_split, nz, scaling, rsort_index, x0 = bm.get_LS()
    sizes = np.asarray(sizes, dtype=np.int64)
    assert np.array_equal(x0, particular_x0(sizes))
    import scipy.sparse as sps
    A = sps.csr_matrix(AA)
    path = os.path.join(str(tmp_path), 'prob.npz')
    np.savez(path, data=A.data, indices=A.indices, indptr=A.indptr, shape=np.array(A.shape),
             b=np.asarray(bb, dtype=np.float64), sizes=sizes, x0=np.asarray(x0, dtype=np.float64))
    res = _spawn(_run_exit, 2, path)
    s0, s1 = res[0][0]['scal'], res[1][0]['scal']
    for r in (0, 1):
        assert res[r][0]['groups'] > 1 and res[r][0]['role'] == (1 if r == 0 else 2)
        assert res[r][0]['r_fx'] > 0          # order-free fixed-point r
    # both ranks decide alike: same reason, same iteration
    assert s0[0] != 0 and s0[0] == s1[0] and s0[1] == s1[1], (s0[:3], s1[:3])
    it = int(s0[1])
    z = np.concatenate([res[0][0]['z'], res[1][0]['z']])
    x = x0 + block_sizes_to_N(sizes).dot(z)
    err = 0.5 * float(np.sum((A.dot(x) - bb) ** 2))
    assert err < 1e-16, err                                # tests/fast/test_main.py:31-47
    ref_it = int(G['main%d_iters' % vi][-1])               # 454 / 569 / 745
    assert abs(it - ref_it) <= max(10, ref_it // 16), (it, ref_it)


# ---- the exchange pipelined behind both walks (link parts) --------------------

def _run_link(rank, world, port, out_q, parts, native):
    _setup(rank, world, port)
    import torch
    from synthetic import make_partitioned
    from distributed import ShardedBB, CallbackComm, torch_all_reduce, torch_all_reduce_async
    full, b, kw = _small()
    sh = make_partitioned(40_000, 2_000, 3_000, rank=rank, world=world, **kw)
    x0 = np.zeros(sh['n'])
    x0[np.cumsum(sh['block_sizes']) - 1] = 1.0
    eng = _engine(sh['A'], sh['block_sizes'], b, x0, 10 ** 9, False, fmt='tiles',
                  link_parts=parts)
    eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))
    comm = CallbackComm(torch_all_reduce(), rank=rank, engine=eng) if native else None
    drv = ShardedBB(eng, torch_all_reduce(), parts=parts, rank=rank, native=comm,
                    all_reduce_async=None if native else torch_all_reduce_async())
    assert drv.link and (drv.native is comm)
    drv.prologue()
    traj, done = {}, 0
    for i in CHECK5:
        drv.iterate(done + 1, i - done)
        done = i
        traj[i] = eng.current_z(i & 1).cpu().numpy().copy()
    info = dict(k2_groups=int(eng.AT_til.img['ngroups']), bounds=list(eng.k1_part_bounds),
                r_fx=float(eng.P.r_fx))
    out_q.put((rank, traj, info))
    if comm is not None:
        _finish(comm)
    else:
        import torch.distributed as dist
        torch.cuda.synchronize()
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize('native', [True, False])
def test_link_parts_two_ranks_vs_oracle(cuda, orc, native, parity):
    """K1 by 3 row-block parts, each part's rows of r all-reduced as it
    finishes, the next K2 by the 3 matching column groups (bsls_bb_k2_part:
    part q reads only its rows of r; the last adds the earlier parts' route
    sums) -- the C++ driver (bsls_bb_shard_iterate_parts, the exchanges on a
    second stream ordered by events) and the Python loop -- follows the
    oracle at 1 / 5 / 20."""
    res = _spawn(_run_link, 2, 3, native)
    for r in (0, 1):
        info = res[r][1]
        assert info['k2_groups'] == 3 and len(info['bounds']) == 4, info
    full, b, _ = _small()
    ref = orc.bb_trace(full['A'], b, full['block_sizes'], max(CHECK5), record_every=1)
    for i in CHECK5:
        got = np.concatenate([res[0][0][i], res[1][0][i]])
        parity('shard_link_parts_%s_%d' % ('native' if native else 'python', i),
               elem_err(got, ref[i]), TOL)


# ---- RCCL itself, forced through its collectives on one rank ------------------

def _run_rccl_forced(rank, world, port, out_q, parts):
    """One nccl rank: RcclComm(force=True), so bsls_bb_shard_iterate[_parts]
    issue every ncclAllReduce of the shipped loop -- the five-sum (f64), the r
    exchange (int64 under the fixed-point r), and with parts the per-part
    exchanges on the comm stream -- on a one-rank communicator, where the sum
    is the identity and the oracle's trajectory is the reference."""
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=rank, world_size=world,
                            device_id=torch.device('cuda', 0))
    from device import BBEngine
    from distributed import ShardedBB, RcclComm, torch_all_reduce
    full, b, kw = _small()
    x0 = np.zeros(full['n'])
    x0[np.cumsum(full['block_sizes']) - 1] = 1.0
    # (one rank: target = A x0 - b directly; _engine's host all-reduce is gloo's)
    target = torch.from_numpy(full['A'].dot(x0) - b).cuda()
    eng = BBEngine(full['A'], None, full['block_sizes'],
                   options={'max_iter': 10 ** 9, 'opt_tol': 1e-30}, early_exit=False,
                   target=target, fmt='tiles', link_parts=parts if parts > 1 else None)
    eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))
    comm = RcclComm(force=True)
    drv = ShardedBB(eng, torch_all_reduce(), parts=parts, rank=rank, native=comm)
    assert drv.native is comm and drv.link == (parts > 1)
    drv.prologue()
    traj, done = {}, 0
    for i in CHECK5:
        drv.iterate(done + 1, i - done)
        done = i
        traj[i] = eng.current_z(i & 1).cpu().numpy().copy()
    # a direct f64 all-reduce through the same communicator: the identity
    t = torch.arange(1000, dtype=torch.float64, device='cuda') * 0.1
    ref = t.clone()
    comm.all_reduce(t)
    torch.cuda.synchronize()
    info = dict(r_fx=float(eng.P.r_fx), ranks=comm.count(),
                direct_ok=bool(torch.equal(t, ref)), groups=int(eng.A_til.img['ngroups']))
    out_q.put((rank, traj, info))
    torch.cuda.synchronize()
    comm.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize('parts', [1, 3])
def test_rccl_collectives_forced_one_rank_vs_oracle(cuda, orc, parts, parity):
    """VERDICT r05 Missing #3: the RCCL transport's calls had only run where a
    one-rank communicator skips them.  Forced on (bsls_comm_force_collectives),
    the shipped loop -- and at parts = 3 the link-part pipeline with its
    exchanges on a second stream -- runs every ncclAllReduce against the real
    library (int64 words of the fixed-point r, doubles of the sums) and still
    follows the oracle at 1 / 5 / 20."""
    res = _spawn(_run_rccl_forced, 1, parts)
    traj, info = res[0]
    assert info['ranks'] == 1 and info['direct_ok'], info
    assert info['r_fx'] > 0, info           # the r exchange summed int64 words
    full, b, _ = _small()
    ref = orc.bb_trace(full['A'], b, full['block_sizes'], max(CHECK5), record_every=1)
    for i in CHECK5:
        parity('rccl_forced_parts%d_%d' % (parts, i), elem_err(traj[i], ref[i]), TOL)


def test_link_parts_reject_bounds_unlike_the_k2_groups(cuda):
    """K2 part q waits only for exchange q, so the C entry point
    refuses row-block bounds whose rows are not the K2 image's column groups
    (BSLS_E_ARG) instead of racing the all-reduce on the comm stream."""
    import ctypes
    import torch
    import _native
    from device import BBEngine
    from distributed import ModelComm
    full, b, _ = _small()
    eng = BBEngine(full['A'], b, full['block_sizes'], options={'max_iter': 10, 'opt_tol': 1e-30},
                   early_exit=False, fmt='tiles', link_parts=3)
    eng.set_shard_role(1)
    comm = ModelComm(1, 0)
    cs = torch.cuda.Stream()
    lb = [int(v) for v in eng.k1_part_bounds]
    L = _native.lib()

    def call(bounds):
        arr = (ctypes.c_int64 * 4)(*bounds)
        return L.bsls_bb_shard_iterate_parts(eng.P, comm.handle, 1, 0, 3, arr,
                                             ctypes.c_void_p(cs.cuda_stream),
                                             _native.stream_handle())
    try:
        assert call(lb) == 0
        moved = list(lb)
        moved[1] += 1 if moved[2] - moved[1] > 1 else -1
        assert moved[1] > 0 and moved[1] < moved[2]
        assert call(moved) == _native.BSLS_E_ARG
        assert call(lb) == 0                   # the right bounds still pass after a refusal
    finally:
        torch.cuda.synchronize()
        comm.close()


def _run_uneven(rank, world, port, out_q, scale):
    _setup(rank, world, port)
    import torch
    from synthetic import make_partitioned
    full, b = _uneven(scale)
    kw = dict(per_col=8, seed=33, gen_chunks=8)
    sh = make_partitioned(40_000, 2_000, 3_000, rank=rank, world=world, **kw)
    x0 = np.zeros(sh['n'])
    x0[np.cumsum(sh['block_sizes']) - 1] = 1.0
    eng = _engine(sh['A'], sh['block_sizes'], b, x0, 10 ** 9, False, fmt='tiles')
    eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))
    drv, comm = _driver(eng, rank)
    drv.prologue()
    traj, done = {}, 0
    for i in CHECK5:
        drv.iterate(done + 1, i - done)
        done = i
        traj[i] = eng.current_z(i & 1).cpu().numpy().copy()
    out_q.put((rank, traj, dict(r_fx=float(eng.P.r_fx))))
    _finish(comm)


def _uneven(scale):
    """The _small problem with b's first 30 links `scale` times the rest: the
    fixed-point r's one scale is set by them, so every other
    row is resolved more coarsely than it would be alone.  Row-bound spread
    (max B_i / min B_i): 65 at 1e3, 6.3e4 at 1e6 (2.6 unscaled)."""
    from synthetic import make_partitioned, add_noise
    full = make_partitioned(40_000, 2_000, 3_000, per_col=8, seed=33, gen_chunks=8)
    b = add_noise(full['Ax'], 0.02, seed=33)
    b[:30] *= scale
    return full, b


@pytest.mark.timeout(600)
@pytest.mark.parametrize('scale,rfx', [(1e3, '1'), (1e6, '1'), (1e6, '0')])
def test_native_driver_fixed_point_r_uneven_rows_vs_oracle(cuda, orc, parity, monkeypatch,
                                                          scale, rfx):
    """one fixed-point scale for rows of very different bounds.
    A spread of 65 (scale 1e3) stays within 1e-12 (measured 1e-14 .. 4e-14).
    At 6.3e4 (scale 1e6: b spans six orders) the iterates measure ~1e-11
    from the oracle with the fixed point (BSLS_SHARD_RFX=1) and ~5e-12 with
    doubles (=0) at iteration 1: the conditioning, not the representation,
    sets it; both are held to 1e-10 there, far inside the north star's 1e-6."""
    monkeypatch.setenv('BSLS_SHARD_RFX', rfx)
    res = _spawn(_run_uneven, 2, scale)
    for r in (0, 1):
        assert (res[r][1]['r_fx'] > 0) == (rfx == '1'), (scale, rfx, res[r][1])
    full, b = _uneven(scale)
    ref = orc.bb_trace(full['A'], b, full['block_sizes'], max(CHECK5), record_every=1)
    tol = TOL if scale < 1e4 else 1e-10
    for i in CHECK5:
        got = np.concatenate([res[0][0][i], res[1][0][i]])
        parity('shard_native_uneven_rows_%g_rfx%s_%d' % (scale, rfx, i), elem_err(got, ref[i]),
               tol)
