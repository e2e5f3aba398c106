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
    assert f is not None and os.path.basename(f) == 'traffic_r05.json'   # not traffic_r05_sydr.json


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
