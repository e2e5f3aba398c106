#!/usr/bin/env python
"""Per-launch HBM traffic of the fused BB kernels from rocprofv3 PMC passes
(tools/gpu_round.sh step `pmc`: FETCH_SIZE and WRITE_SIZE in separate passes
over tools/kprof.py).  MI355X_MICROARCH.md "HBM / rocprofv3": FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide
coalesced reads, so traffic = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes).
Usage: python tools/traffic.py CONFIG OUT.json pmc_dir... -- adds CONFIG's kernels
(dealt tiles; K1 = the walk + its finish launch) to OUT.json (keyed by config, read by bench.py)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# bench.py kernel names -> device kernels (demangled prefixes) in one launch of the stage
KERNELS = {
    'C3': {'K2_spmvT_Nt_dots': ['bsls::bb_k2t<3, true, 0, 2>'],
           'K3_pava_clip_z2x': ['bsls::bb_k3<1, false, 2>'],
           'K1_spmv_A': ['bsls::bb_k1t<0, true, true, true,', 'bsls::bb_k1_sum<true, true, true>'],
           'proj_simplex_C2': ['bsls::proj_lds_kernel<false, 2, false>'],   # the exact path
           'proj_simplex_fast_C2': ['bsls::proj_pipe_lds_kernel<false, false>'],
           'isotonic_C4': ['bsls::iso_packs_kernel<1, false>']},
    'C5': {'K2_spmvT_Nt_dots': ['bsls::bb_k2t<3, true, 0, 2>'],
           'K3_pava_clip_z2x': ['bsls::bb_k3<2, true, 2>'],
           'K1_spmv_A': ['bsls::bb_k1t<0, true, true, true,', 'bsls::bb_k1_sum<true, true, true>']},
}
# rank 0 of an N-way split (stages 10 / 15 / 14: atomic K1, r initialised in
# K3; bench.py --rehearse-shard N [--rehearse-workload C3]), keyed as bench.py
# looks them up at N GPUs: '<workload>_x<N>'.  A '|' separates alternatives
# (K3's pack form depends on the shard's pack count).
SHARD = {'K2_spmvT_Nt_dots': ['bsls::bb_k2t<3, true, 2, 2>'],
         'K3_pava_clip_z2x': ['bsls::bb_k3<1, false, 2>|bsls::bb_k3<2, true, 2>'],
         'K1_spmv_A': ['bsls::bb_k1t<0, true, true, false,']}
for _wl in ('C3', 'C5'):
    for _n in (2, 4, 8):
        KERNELS['%s_x%d' % (_wl, _n)] = SHARD


def load(dirs):
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
            per = defaultdict(float)
            for r in csv.DictReader(open(f)):
                per[(r['Dispatch_Id'], r['Kernel_Name'], r['Counter_Name'])] += float(r['Counter_Value'])
            for (_, kn, cn), v in per.items():
                vals[kn][cn].append(v)
    return vals


def main():
    cfg, path = sys.argv[1], sys.argv[2]
    vals = load(sys.argv[3:])
    out = {}
    for name, parts in KERNELS[cfg].items():
        fetch = write = 0.0
        ok = True
        for alts in parts:
            hits = [k for pfx in alts.split('|') for k in vals if pfx in k]
            if not hits:
                ok = False
                break
            k = hits[0]
            f, w = vals[k].get('FETCH_SIZE', []), vals[k].get('WRITE_SIZE', [])
            if not f or not w:
                ok = False
                break
            fetch += sum(f) / len(f)
            write += sum(w) / len(w)
        if ok:
            out[name] = {'fetch_kib': fetch, 'write_kib': write,
                         'hbm_bytes_per_launch': (2 * fetch + write) * 1024,
                         'formula': '(2*FETCH_SIZE + WRITE_SIZE) KiB, gfx950 FETCH correction'}
    allc = json.load(open(path)) if os.path.exists(path) else {}
    allc[cfg] = out
    json.dump(allc, open(path, 'w'), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
