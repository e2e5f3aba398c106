"""Probe: the native shard driver's RCCL calls forced on a one-rank
communicator (bsls_comm_force_collectives), step by step with a line after
each, and which librccl copies the process has mapped.  One process, nccl
world 1; run under `timeout`.  Usage: python tools/rccl_forced_probe.py [step]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'block-simplex-least-squares_amd')]

import numpy as np


def say(*a):
    print('[%.2fs]' % (time.perf_counter() - T0), *a, flush=True)


def rccl_maps():
    out = set()
    with open('/proc/self/maps') as f:
        for line in f:
            if 'rccl' in line or 'nccl' in line:
                out.add(line.split()[-1])
    return sorted(out)


T0 = time.perf_counter()
os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
os.environ.setdefault('MASTER_PORT', '29611')
import torch
import torch.distributed as dist
import ctypes
torch.cuda.set_device(0)
dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
say('pg up; rccl maps:', rccl_maps())
import _native
from _native import check, ptr, stream_handle
from distributed import RcclComm
L = _native.lib()
comm = RcclComm(force=False)
say('RcclComm up; count', comm.count(), 'maps:', rccl_maps())
t = torch.arange(8, dtype=torch.float64, device='cuda')
comm.all_reduce(t)
torch.cuda.synchronize()
say('direct f64 all-reduce ok', t[:3].tolist())
ti = torch.arange(8, dtype=torch.int64, device='cuda')
check(L.bsls_comm_all_reduce(comm.handle, ptr(ti), 8, stream_handle()), 'ar')
torch.cuda.synchronize()
say('direct all-reduce of int64 words (as doubles) ok')
# the driver's forced loop on the small partitioned problem
from synthetic import make_partitioned, add_noise
from device import BBEngine
from distributed import ShardedBB, torch_all_reduce
kw = dict(per_col=8, seed=33, gen_chunks=8)
full = make_partitioned(40_000, 2_000, 3_000, **kw)
b = add_noise(full['Ax'], 0.02, seed=33)
x0 = np.zeros(full['n'])
x0[np.cumsum(full['block_sizes']) - 1] = 1.0
target = torch.from_numpy(full['A'].dot(x0) - b).cuda()
eng = BBEngine(full['A'], None, full['block_sizes'], options={'max_iter': 10 ** 9, 'opt_tol': 1e-30},
               early_exit=False, target=target, fmt='tiles')
eng.set_z0(torch.zeros(eng.nz, dtype=torch.float64))
drv = ShardedBB(eng, torch_all_reduce(), rank=0, native=comm)
drv.prologue()
torch.cuda.synchronize()
say('prologue ok, r_fx', float(eng.P.r_fx))
drv.iterate(1, 1)
torch.cuda.synchronize()
say('1 iteration unforced ok')
check(L.bsls_comm_force_collectives(comm.handle, 1), 'force')
for i in range(2, 6):
    drv.iterate(i, 1)
    say('forced iteration %d enqueued' % i)
    torch.cuda.synchronize()
    say('forced iteration %d done' % i)
comm.close()
dist.destroy_process_group()
say('done')
