"""Where a short timed window's extra time goes (C3, one GPU): for windows of
K iterations after W warmup, the host wall time (as bench.time_run takes it)
against HIP events recorded on the engine's stream at the window's two ends
(device time of the K iterations), per window.

    python tools/window_probe.py [--steps 20] [--warmup 400] [--windows 10]
        [--prime]

--prime: before each window's barrier/synchronize, a short untimed spin on the
stream (the GPU busy right up to the window) -- whether an idle gap before
the window costs device time.
--preheat: ~100 ms of full-chip elementwise work before the warmup (diagnostic:
whether the walks' slow first iterations are the chip's clocks settling).
--stage K: instead of the windows, stage K (3 = K2, 7 = K1) relaunched 300
times on one state right after the engine's prologue (diagnostic, under a
kernel trace: whether the walks' early-iteration trend needs the iterate).
--hold: a ~0.5-ms spin enqueued before the window's first event, so the host
has enqueued the whole window before the device reaches it (diagnostic: the
device time without any wait on the host's launches)."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=400)
    ap.add_argument('--windows', type=int, default=10)
    ap.add_argument('--prime', action='store_true')
    ap.add_argument('--hold', action='store_true')
    ap.add_argument('--preheat', action='store_true')
    ap.add_argument('--stage', type=int, default=0)
    a = ap.parse_args()
    import torch
    import bench
    torch.cuda.set_device(0)
    sh, b = bench.build_problem('C3', 1, 0, None)
    eng, run = bench.build_engine(sh, b, 1, None, 1)
    if a.preheat:
        t = torch.empty(1 << 27, dtype=torch.float64, device='cuda')
        for _ in range(250):
            t.mul_(1.0000001)
        torch.cuda.synchronize()
        del t
    if a.stage:
        for _ in range(300):
            eng.stage(a.stage, 1)
        torch.cuda.synchronize()
        print('stage %d relaunched 300 times' % a.stage)
        return
    run(1, a.warmup)
    torch.cuda.synchronize()
    first = 1 + a.warmup
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    wall, dev, enq = [], [], []
    for _ in range(a.windows):
        if a.prime:
            torch.cuda._sleep(20000)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if a.hold:
            torch.cuda._sleep(500000)
        e0.record()
        run(first, a.steps)
        enq.append((time.perf_counter() - t0) * 1e6)
        e1.record()
        torch.cuda.synchronize()
        wall.append((time.perf_counter() - t0) * 1e6)
        dev.append(e0.elapsed_time(e1) * 1e3)
        first += a.steps
    wall, dev = np.array(wall), np.array(dev)
    print('steps %d warmup %d prime %s hold %s: wall median %.1f us (%.2f per it), device median '
          '%.1f us (%.2f per it), wall - device median %.1f us, enqueue median %.1f us'
          % (a.steps, a.warmup, a.prime, a.hold, np.median(wall), np.median(wall) / a.steps,
             np.median(dev), np.median(dev) / a.steps, np.median(wall - dev), np.median(enq)),
          flush=True)


if __name__ == '__main__':
    main()
