"""Host cost of the sharded BB driver (distributed.ShardedBB) on one GPU: rank 0
of a W-way C5 partition through a one-rank RCCL group (bench.py
--rehearse-shard W).  Prints the host time to enqueue K iterations (no sync)
and the wall time of the same K iterations with the final synchronize: when
the first is close to the second, the Python launch path, not the GPU, sets
the per-rank iteration rate.

    python tools/host_cost.py --world 8 --iters 200
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--world', type=int, default=8)
    ap.add_argument('--iters', type=int, default=200)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    for k, v in (('MASTER_ADDR', '127.0.0.1'), ('MASTER_PORT', '29541'), ('RANK', '0'),
                 ('WORLD_SIZE', '1')):
        os.environ.setdefault(k, v)
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', device_id=torch.device('cuda', 0))
    import bench
    sh, b = bench.build_problem('C5', 1, 0, dist, shard_of=args.world)
    eng, run = bench.build_engine(sh, b, 1, dist, 1, sharded=True)
    run(1, 20)
    torch.cuda.synchronize()
    K = args.iters
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(21 + rep * K, K)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print('W=%d rep %d: enqueue %.1f us/it, wall %.1f us/it'
              % (args.world, rep, (t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6), flush=True)
    # the same stages without the collectives (a one-rank group sums nothing)
    t0 = time.perf_counter()
    for i in range(K):
        for s in (3, 4, 1, 2):
            eng.stage(s, 1000 + i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print('stages only: enqueue %.1f us/it, wall %.1f us/it' % ((t1 - t0) / K * 1e6,
                                                                (t2 - t0) / K * 1e6), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
