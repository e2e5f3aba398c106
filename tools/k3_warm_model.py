"""numpy model of K3's warm-start test (pava_wave.hpp pava_warm): the same
segmented scan (row_shr 1/2/4/8, row_bcast 15/31 with the per-step segment
test), split and order conditions, on random packs: every true PAVA partition
must pass, and no partition may pass with a fit further than 1e-12 from PAVA's."""
import numpy as np
rs = np.random.RandomState(1)

def pava_blocks(y, starts, L):
    out = y.copy(); heads = np.zeros(L, bool)
    bounds = list(starts) + [L]
    for a, b in zip(bounds[:-1], bounds[1:]):
        st = []
        for i in range(a, b):
            st.append([i, y[i], 1])
            while len(st) > 1 and st[-2][1] / st[-2][2] >= st[-1][1] / st[-1][2]:
                s_, sm, c = st.pop(); st[-1][1] += sm; st[-1][2] += c
        for k, (s0, sm, c) in enumerate(st):
            e0 = st[k + 1][0] if k + 1 < len(st) else b
            out[s0:e0] = sm / c; heads[s0] = True
    return out, heads

def warm(y, L, B, H):
    l = np.arange(64)
    act = l < L
    h = np.array([max(j for j in range(i + 1) if H[j]) for i in range(64)])
    e = np.array([(min([j for j in range(i + 1, 64) if H[j]] or [64]) - 1) for i in range(64)])
    e = np.minimum(e, L - 1)
    s = np.where(act, np.pad(y, (0, 64 - L)), 0.0)
    for k in (1, 2, 4, 8):
        u = np.array([s[i - k] if (i % 16) >= k else 0.0 for i in range(64)])
        s = s + np.where(l - k >= h, u, 0.0)
    u = np.array([s[(i & ~15) - 1] if (i // 16) in (1, 3) else 0.0 for i in range(64)])
    s = s + np.where(((l & 16) != 0) & (h <= (l & ~15) - 1), u, 0.0)
    u = np.array([s[31] if i >= 32 else 0.0 for i in range(64)])
    s = s + np.where((l >= 32) & (h <= 31), u, 0.0)
    S = s[e]
    m = S / (e - h + 1)
    mp = np.concatenate([[0.0], m[:-1]])
    split_ok = (l == e) | (s >= (l - h + 1) * m)
    order_ok = (l != h) | B[:64] | (mp <= m)
    ok = ~act | (split_ok & order_ok)
    return ok.all(), m[:L], s[:L]

npass = nfail = bad = 0
for trial in range(3000):
    sizes = []
    L = 0
    while True:
        k = rs.randint(1, 40)
        if L + k > 64: break
        sizes.append(k); L += k
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    B = np.zeros(64, bool); B[starts] = True
    y = rs.randn(L) * (0.5 if trial % 2 else 1.0) + np.linspace(0, 1, L) * (trial % 3)
    fit, heads = pava_blocks(y, starts, L)
    Hm = np.zeros(64, bool); Hm[:L] = heads
    # segmented scan check
    ok, m, s = warm(y, L, B, Hm)
    if ok:
        npass += 1
        if np.max(np.abs(m - fit)) > 1e-12 * max(1, np.abs(fit).max()): bad += 1
    else:
        nfail += 1
    # a perturbed partition must not pass unless it yields the same fit
    H2 = Hm.copy(); j = rs.randint(1, L) if L > 1 else 0
    if not B[j]: H2[j] = not H2[j]
    ok2, m2, _ = warm(y, L, B, H2)
    if ok2 and np.max(np.abs(m2 - fit)) > 1e-12 * max(1, np.abs(fit).max()): bad += 1
print('true partition: pass', npass, 'fail', nfail, 'bad', bad)
