"""bench.py's measurement helpers on the CPU (no GPU, no kernels): which PMC
traffic file a line reads, the (workload, world) keys it looks kernels up
by, traffic null where a key was never profiled, and the windowed timing
the headline takes its median from."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))

import bench  # noqa: E402
import traffic  # noqa: E402


def _kern(us):
    return {'K2_spmvT_Nt_dots': {'avg_us': us, 'alg_bytes': 227e6, 'GB_s': 227e3 / us, 'frac': 0.8,
                                 'format_bytes': 87e6, 'format_frac': 0.3,
                                 'rocprof_kernels': ['bb_k2t']},
            'K1_spmv_A': {'avg_us': us / 2, 'alg_bytes': 202e6, 'GB_s': 1.0, 'frac': 0.8,
                          'format_bytes': 1.0, 'format_frac': 0.1},
            'formats': None}


def test_traffic_file_is_the_default_builds():
    f = bench.traffic_file()
    assert f is not None and os.path.basename(f) == 'traffic_r06.json'   # the newest round's


def test_traffic_keys_cover_every_line_the_driver_prints():
    d = json.load(open(bench.traffic_file()))
    for key in ('C3', 'C5', 'C3_x2', 'C3_x4', 'C3_x8', 'C5_x2', 'C5_x4', 'C5_x8'):
        assert key in traffic.KERNELS, key
        assert 'K2_spmvT_Nt_dots' in d[key], key
        assert d[key]['K2_spmvT_Nt_dots']['hbm_bytes_per_launch'] > 0


def test_roofline_traffic_keyed_and_null_when_unprofiled(tmp_path):
    p = tmp_path / 'traffic_r99.json'
    p.write_text(json.dumps({'C3': {'K2_spmvT_Nt_dots': {'hbm_bytes_per_launch': 88e6}}}))
    r = bench.roofline_of(_kern(34.0), str(p), 'C3')
    assert r['kernel'] == 'K2_spmvT_Nt_dots' and r['traffic'] == 88e6
    assert abs(r['physical_frac'] - 88e6 / 34e-6 / 8e12) < 1e-12
    r = bench.roofline_of(_kern(34.0), str(p), 'C3_x8')   # a shard never profiled
    assert r['traffic'] is None and r['physical_frac'] is None


def test_time_run_windows_exact_steps():
    calls = []

    def run(first, count):
        calls.append((first, count))

    class _Cuda:
        @staticmethod
        def synchronize():
            pass

    import torch
    real = torch.cuda.synchronize
    torch.cuda.synchronize = _Cuda.synchronize
    try:
        els = bench.time_run(run, 20, 5, None, windows=4)
    finally:
        torch.cuda.synchronize = real
    assert len(els) == 4 and all(e >= 0 for e in els)
    # warmup first, then four windows of exactly K iterations, consecutive
    assert calls == [(1, 5), (6, 20), (26, 20), (46, 20), (66, 20)]
    assert np.median(els) >= min(els)


# ---- the N > 1 self-check ---------------------------------

def test_selfcheck_verdict():
    ref = np.linspace(-2.0, 3.0, 101)
    assert bench.selfcheck_verdict(ref.copy(), ref, 1e-6) == (0.0, True)
    got = ref.copy()
    got[7] += 2e-6 * max(1.0, abs(ref[7]))
    err, ok = bench.selfcheck_verdict(got, ref, 1e-6)
    assert not ok and abs(err - 2e-6) < 1e-12
    assert bench.selfcheck_verdict(ref[:-1], ref, 1e-6) == (float('inf'), False)
    got = ref.copy()
    got[3] = np.nan
    assert not bench.selfcheck_verdict(got, ref, 1e-6)[1]


def _gather_rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    z = torch.arange(10 * rank, 10 * rank + 3 + 4 * rank, dtype=torch.float64)
    q.put((rank, bench.gather_z(z, dist, world)))
    dist.destroy_process_group()


def test_gather_z_ragged_two_ranks():
    """The ranks' z slices (different lengths) in rank order, on every rank."""
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 33000 + os.getpid() % 900
    ps = [ctx.Process(target=_gather_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = np.concatenate([np.arange(0, 3), np.arange(10, 17)]).astype(np.float64)
    for r in (0, 1):
        assert np.array_equal(res[r], want)


def _main_rank(rank, world, port, q, fail):
    """bench.main() at N = 2 over gloo with the GPU legs replaced: the order of
    the legs and the line's self-check fields."""
    import io
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), BSLS_DIST_BACKEND='gloo')
    calls = []

    def fake_check(world_, rank_, dist, parts=1, problem=None):
        calls.append('selfcheck')
        return {'err': 3e-16 if not fail else 1e-3, 'ok': not fail, 'rccl_ranks': world_,
                'tol': 1e-6, 'transport': 'fake'}

    def fake_workload(wl, args, world_, rank_, dist, tfile, steps, shard_of=None):
        calls.append('timed:' + wl)
        return {'value': 1.0, 'unit': 'it/s'} if rank_ == 0 else None

    bench.selfcheck_sharded = fake_check
    bench.bench_workload = fake_workload
    sys.argv = ['bench.py', '--gpus', str(world), '--steps', '2', '--warmup', '1']
    buf, real = io.StringIO(), sys.stdout
    sys.stdout = buf
    code = 0
    try:
        bench.main()
    except SystemExit as e:
        code = e.code
    finally:
        sys.stdout = real
    q.put((rank, code, calls, buf.getvalue()))


def _run_main(fail):
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 34000 + os.getpid() % 900 + 3 * int(fail)
    ps = [ctx.Process(target=_main_rank, args=(r, 2, port, q, fail)) for r in range(2)]
    for p in ps:
        p.start()
    res = {item[0]: item[1:] for item in (q.get(timeout=180) for _ in ps)}
    for p in ps:
        p.join(timeout=60)
    return res


def test_main_n2_selfcheck_before_timing_and_in_the_line():
    res = _run_main(False)
    for r in (0, 1):
        code, calls, _ = res[r]
        assert code in (0, None)
        # the check runs first, then the headline and the strong-scaling leg
        assert calls == ['selfcheck', 'timed:C3', 'timed:C5'], calls
    line = json.loads(res[0][2].strip().splitlines()[-1])
    assert line['selfcheck_err'] == 3e-16 and line['rccl_ranks'] == 2
    assert line['selfcheck']['ok'] and line['value'] == 1.0
    assert res[1][2] == ''                      # one line, on rank 0 only


def test_main_n2_selfcheck_mismatch_exits_nonzero_untimed():
    res = _run_main(True)
    for r in (0, 1):
        code, calls, _ = res[r]
        assert code == 3 and calls == ['selfcheck'], (code, calls)
    line = json.loads(res[0][2].strip().splitlines()[-1])
    assert line['value'] is None and line['selfcheck_err'] == 1e-3 and 'error' in line
