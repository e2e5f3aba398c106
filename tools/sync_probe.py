"""What a bench window's two ends cost on the host: wall time from a
synchronized idle stream through one launch to torch.cuda.synchronize()
returning, for a tiny kernel and two spins -- the fixed part
of every timed window (bench.time_run), against the device time.

    python tools/sync_probe.py [--spin-flag]

--spin-flag: hipSetDeviceFlags(hipDeviceScheduleSpin) before the first HIP
call (the host spins on completion instead of waiting for an interrupt)."""
import ctypes
import sys
import time

import numpy as np


def main():
    if '--spin-flag' in sys.argv:
        hip = ctypes.CDLL('libamdhip64.so')
        print('hipSetDeviceFlags(spin) ->', hip.hipSetDeviceFlags(ctypes.c_uint(1)))
    import torch
    x = torch.zeros(1024, device='cuda')
    torch.cuda.synchronize()
    # cycles of torch's spin kernel per us (~100 MHz shader-clock counter)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(int(1e6))
    e1.record()
    torch.cuda.synchronize()
    per_us = 1e6 / (e0.elapsed_time(e1) * 1e3)
    for name, work in (('tiny add', lambda: x.add_(1.0)),
                       ('spin short', lambda: torch.cuda._sleep(int(100 * per_us))),
                       ('spin long', lambda: torch.cuda._sleep(int(1500 * per_us)))):
        wall, dev = [], []
        for _ in range(200):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            work()
            e1.record()
            torch.cuda.synchronize()
            wall.append((time.perf_counter() - t0) * 1e6)
            dev.append(e0.elapsed_time(e1) * 1e3)
        w, d = np.median(wall), np.median(dev)
        print('%-14s wall %8.1f us  device %8.1f us  overhead %6.1f us' % (name, w, d, w - d),
              flush=True)


if __name__ == '__main__':
    main()
