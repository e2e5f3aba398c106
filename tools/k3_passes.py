"""PAVA pass statistics of K3's input (CPU): runs the oracle BB loop on a
C3-shaped problem (scaled down) and, at chosen iterations, replays the
reference PAVA v1 (isotonic_regression.h:13-58) on z - t g per K3 pack,
recording passes per pack and runs alive after each pass.  Sizes the design
of the K3 PAVA (how many runs a wave carries after pass 1).
python tools/k3_passes.py [--n 200000] [--at 2,5,20,50]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))


def pava_passes(y):
    """Run counts after every pass of the reference PAVA v1 on one block
    (unit weights); the last entry is the converged run count."""
    Y = list(y)
    W = [1] * len(Y)
    counts = [len(Y)]
    while True:
        nY, nW = [], []
        i, pooled = 0, False
        while i < len(Y):
            j = i
            while j + 1 < len(Y) and Y[j + 1] <= Y[j]:
                j += 1
            if Y[i] != Y[j]:
                num, den = 0.0, 0
                for r in range(i, j + 1):
                    num += Y[r] * W[r]
                    den += W[r]
                nY.append(num / den)
                nW.append(den)
                pooled = True
            else:
                nY.extend(Y[i:j + 1])
                nW.extend(W[i:j + 1])
            i = j + 1
        if not pooled:
            break
        Y, W = nY, nW
        counts.append(len(Y))
    return counts


def packs_of(kz):
    out, b, p = [], 0, kz.size
    while b < p:
        if kz[b] > 64:
            out.append([b])
            b += 1
            continue
        tot, e = 0, b
        while e < p and kz[e] <= 64 and tot + kz[e] <= 64:
            tot += int(kz[e])
            e += 1
        out.append(list(range(b, e)))
        b = e
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=200_000)
    ap.add_argument('--at', default='2,5,20,50,100')
    args = ap.parse_args()
    import synthetic
    from oracle import oracle as orc
    n = args.n
    sh = synthetic.make_shard(n, n // 20, n // 10, 16)
    b = synthetic.add_noise(sh['Ax'], 0.02)
    sizes = sh['block_sizes']
    P = orc.solve_in_z_parts(sh['A'], b, sizes)
    kz = sizes - 1
    zst = P['zstarts']
    packs = packs_of(kz)
    at = set(int(a) for a in args.at.split(','))
    it = [0]
    proj0 = P['proj']

    def proj(x):
        it[0] += 1
        if it[0] in at:
            passes, runs1, runs_end, lens = [], [], [], []
            for pk in packs:
                cnt = [pava_passes(x[zst[bb]:zst[bb] + kz[bb]]) for bb in pk]
                np_ = max(len(c) for c in cnt)          # pooling passes of the slowest block
                passes.append(np_)
                runs1.append(sum(c[1] if len(c) > 1 else c[0] for c in cnt))
                runs_end.append(sum(c[-1] for c in cnt))
                lens.append(sum(kz[bb] for bb in pk))
            # lane-per-block: groups of 64 consecutive blocks, lockstep steps =
            # sum over passes of the longest run list among unconverged blocks
            allc = [pava_passes(x[zst[bb]:zst[bb] + kz[bb]]) for bb in range(kz.size)]
            steps = []
            for g0 in range(0, kz.size, 64):
                cs = allc[g0:g0 + 64]
                npass = max(len(c) for c in cs)
                steps.append(sum(max(c[q] for c in cs if len(c) > q) for q in range(npass)))
            print('  lane-per-block groups %d: steps mean %.1f max %d; entries/group %.0f'
                  % (len(steps), np.mean(steps), max(steps), kz.sum() / len(steps)))
            passes, runs1 = np.array(passes), np.array(runs1)
            print('iter %d: packs %d, mean len %.1f, passes mean %.2f max %d '
                  '(hist %s), runs after pass 1 mean %.1f (p90 %d), converged runs %.1f'
                  % (it[0], len(packs), np.mean(lens), passes.mean(), passes.max(),
                     np.bincount(passes).tolist(), runs1.mean(), np.percentile(runs1, 90),
                     np.mean(runs_end)), flush=True)
        return proj0(x)
    orc.bb_solve(P['z0'], P['f'], P['nabla_f'], orc.stopping, record_every=10 ** 9, proj=proj,
                 log=lambda i, s, dt: 0.0,
                 options={'max_iter': max(at), 'verbose': 0, 'opt_tol': 1e-30})


if __name__ == '__main__':
    main()
