"""Column-sharded BB (distributed.ShardedBB) over the real HIP stages.

Two ranks share the one GPU of the test box (gloo moves the all-reduces through
host memory: RCCL refuses two ranks on one device), plus one rank over RCCL
(backend "nccl") so the collective path bench.py uses at N > 1 runs too.  Each
rank builds a device BBEngine on its block-aligned column shard and drives the
stages bsls_bb_stage(0..6) with the all-reduces between them; the concatenated
iterates must follow the oracle's BB trajectory (python/BB.py semantics) to the
north star's 1e-6 relative.
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, 'block-simplex-least-squares_amd')

ITERS = 30
CHECK = (1, 2, 7, 30)


def _problem():
    from synthetic import make_shard, add_noise
    sh = make_shard(40_000, 2_000, 3_000, per_col=8, seed=33)
    b = add_noise(sh['Ax'], 0.02, seed=33)
    return sh, b


def _partitioned(rank, world):
    """A small world-independent problem (synthetic.make_partitioned, config
    C5's generator): rank's shard, full b."""
    from synthetic import make_partitioned, add_noise
    kw = dict(per_col=8, seed=33, gen_chunks=8)
    full = make_partitioned(40_000, 2_000, 3_000, **kw)
    sh = make_partitioned(40_000, 2_000, 3_000, rank=rank, world=world, **kw)
    return sh, add_noise(full['Ax'], 0.02, seed=33), full


def _run(rank, world, backend, port, out_q, fmt=None, parts=1, max_iter=10 ** 9, native=False):
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    from device import BBEngine
    from distributed import (ShardedBB, partition_blocks, torch_all_reduce,
                             torch_all_reduce_async)
    if backend == 'nccl':
        dist.init_process_group('nccl', rank=rank, world_size=world,
                                device_id=torch.device('cuda', 0))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    if fmt:
        sh, b, _ = _partitioned(rank, world)
        A_g, sz_g = sh['A'], sh['block_sizes']
        x0 = np.zeros(sh['n'])
    else:
        sh, b = _problem()
        sizes = sh['block_sizes']
        bounds = partition_blocks(sizes, sizes.astype(np.float64), world)
        xst = np.concatenate(([0], np.cumsum(sizes)))
        c0, c1 = xst[bounds[rank]], xst[bounds[rank + 1]]
        A_g = sh['A'][:, c0:c1].tocsr()
        sz_g = sizes[bounds[rank]:bounds[rank + 1]]
        x0 = np.zeros(c1 - c0)
    x0[np.cumsum(sz_g) - 1] = 1.0
    part = torch.from_numpy(A_g.dot(x0)).cuda()
    dist.all_reduce(part)
    target = part - torch.from_numpy(b).cuda()
    eng = BBEngine(A_g, None, sz_g, options={'max_iter': max_iter, 'opt_tol': 1e-30},
                   early_exit=max_iter < 10 ** 9, target=target, fmt=fmt)
    eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))
    comm = None
    if native:
        from distributed import RcclComm
        comm = RcclComm()
    drv = ShardedBB(eng, torch_all_reduce(), parts=parts,
                    all_reduce_async=torch_all_reduce_async(), rank=rank, native=comm)
    drv.prologue()
    traj = {}
    for i in range(1, ITERS + 1):
        drv.iterate(i, 1)
        if i in CHECK:
            zb = int(eng.scalars()[2]) if max_iter < 10 ** 9 else (i & 1)
            traj[i] = eng.current_z(zb).cpu().numpy().copy()
    if max_iter < 10 ** 9:
        traj["r"] = eng.residual_value().cpu().numpy().copy()
        traj['scal'] = eng.scalars().copy()
    out_q.put((rank, traj))
    if comm is not None:
        torch.cuda.synchronize()
        comm.close()
    dist.barrier()
    dist.destroy_process_group()


def _spawn(world, backend, fmt=None, parts=1, max_iter=10 ** 9, raw=False, native=False):
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29700 + (os.getpid() % 500) + world + 3 * parts + (max_iter % 7) + 11 * int(native)
    procs = [ctx.Process(target=_run, args=(r, world, backend, port, q, fmt, parts, max_iter,
                                            native))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if raw:
        return res
    return {i: np.concatenate([res[r][i] for r in range(world)]) for i in CHECK}


def _check(got, orc, partitioned=False):
    if partitioned:
        full, b = _partitioned(0, 1)[2], _partitioned(0, 1)[1]
        sh = dict(A=full['A'], block_sizes=full['block_sizes'])
    else:
        sh, b = _problem()
    ref = orc.bb_trace(sh['A'], b, sh['block_sizes'], ITERS, record_every=1)
    for i in CHECK:
        d = np.max(np.abs(got[i] - ref[i])) / max(1.0, np.max(np.abs(ref[i])))
        assert d < 1e-6, (i, d)


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_sharded_bb_two_ranks_on_device(cuda, orc):
    _check(_spawn(2, 'gloo'), orc)


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_sharded_bb_rccl_one_rank(cuda, orc):
    _check(_spawn(1, 'nccl'), orc)


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_sharded_bb_tiles_overlapped_two_ranks(cuda, orc):
    """C5's path at small size: world-independent shards (make_partitioned), the
    streamed-tile kernels, the residual all-reduced in 3 row parts behind K1
    (bsls_bb_residual_rows + async all-reduce)."""
    _check(_spawn(2, 'gloo', fmt='tiles', parts=3), orc, partitioned=True)


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_sharded_bb_tiles_overlapped_rccl(cuda, orc):
    _check(_spawn(1, 'nccl', fmt='tiles', parts=3), orc, partitioned=True)


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_sharded_stop_keeps_final_residual(cuda, orc):
    """max_iter = 7 with early exits on: iterations 8..30 enqueued past the stop
    change nothing -- every rank reports the stop at iteration 7 with the z of
    iteration 7, and r stays the residual of iteration 7 on every rank (rank 0
    keeps its r, the others write 0 before each all-reduce), not world x r."""
    res = _spawn(2, 'gloo', max_iter=7, raw=True)
    sh, b = _problem()
    ref = orc.bb_trace(sh['A'], b, sh['block_sizes'], 7, record_every=1)
    z = np.concatenate([res[r][30] for r in range(2)])
    assert np.max(np.abs(z - ref[7])) <= 1e-6 * max(1.0, np.max(np.abs(ref[7])))
    for r in range(2):
        s = res[r]['scal']
        assert s[0] == 2 and s[1] == 7, s[:3]          # STOP_MAXITER at iteration 7
    # the residual of z_7: A (x0 + N z_7) - b
    from bsls_utils import particular_x0, block_sizes_to_N
    sizes = sh['block_sizes']
    r7 = sh['A'].dot(particular_x0(sizes) + block_sizes_to_N(sizes).dot(ref[7])) - b
    for r in range(2):
        assert np.max(np.abs(res[r]['r'] - r7)) <= 1e-9 * max(1.0, np.max(np.abs(r7)))


@pytest.mark.gpu
@pytest.mark.timeout(400)
@pytest.mark.parametrize('fmt', [None, 'tiles'])
def test_native_shard_driver_rccl(cuda, orc, fmt):
    """The C++ driver (bsls_bb_shard_iterate: the stages and both RCCL
    all-reduces of an iteration enqueued from C++, its own communicator made
    through RcclComm) follows the oracle, on the panels and on the tiles."""
    _check(_spawn(1, 'nccl', fmt=fmt, native=True), orc, partitioned=fmt == 'tiles')


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_native_shard_driver_equals_python_loop(cuda):
    """Same kernels, same order, the same one-rank collectives: on the
    fixed-order (panel) images the C++ loop gives the Python loop's iterates
    bit for bit, and the same stop."""
    # (the fixed-order images: the default dealt tiles' LDS atomics vary run
    # to run in the last bits, whichever loop enqueues them)
    a = _spawn(1, 'nccl', fmt='panels', native=True, raw=True)[0]
    b = _spawn(1, 'nccl', fmt='panels', native=False, raw=True)[0]
    for i in CHECK:
        assert np.array_equal(a[i], b[i]), i
    a = _spawn(1, 'nccl', max_iter=7, native=True, raw=True)[0]
    assert a['scal'][0] == 2 and a['scal'][1] == 7
