"""Projected Barzilai-Borwein (reference: python/BB.py:7-45).

`solve` keeps the reference's signature and loop, over caller closures
f / nabla_f / proj operating on NumPy arrays or HIP-resident torch tensors.
The production path for the z-space problem is `solve_engine`: the whole
iteration runs fused on the device (device.BBEngine, kernels in csrc/bb.hip),
with identical logging points and stopping rule.
"""
import time

from _arr import builtin_sum, dot


def solve(x0, f, nabla_f, stopping, record_every=500, proj=None, log=None, options=None):
    # Save initial state
    start = log(0, x0, 0)
    i, stop = 0, False
    x = x0
    x_prev = x + 1
    g_prev = nabla_f(x_prev)
    while not stop:
        i += 1
        g = nabla_f(x)
        delta_g = g - g_prev
        if builtin_sum(delta_g) == 0:
            print('Exiting... no change in gradient')
            break
        delta_x = x - x_prev
        t = dot(delta_x, delta_g) / dot(delta_g, delta_g)   # BB2 step
        if abs(t) <= 1e-10 or abs(t) > 1e10:
            print('BB update is having some trouble, implement fix! t=%8.5e' % t)
        x_next = x - t * g
        x_prev, x = x, x_next
        g_prev = g
        if proj:
            x = proj(x)
        fx = f(x)
        stop = stopping(g, fx, i, t, delta_g=delta_g, options=options)
        if i % record_every == 0:
            start = log(i, x, time.time() - start)
    log(i, x, time.time() - start)
    return x


def solve_engine(engine, z0=None, record_every=500, log=None, poll=50, to_host=True):
    """BB.solve semantics on the fused device engine; returns the final z."""
    return engine.solve(z0=z0, log=log, record_every=record_every, poll=poll, to_host=to_host)
