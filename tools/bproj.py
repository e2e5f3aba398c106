"""C2 projection timing as bench.py measures it (cold input, batched launches):
python tools/bproj.py  (GPU box; BSLS_LIB selects a variant build)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))

import bench  # noqa: E402

if __name__ == '__main__':
    for _ in range(2):
        r = bench.bench_proj()
        print(json.dumps({k: r[k] for k in ('avg_us', 'GB_s', 'isolated_median_us',
                                            'bit_exact_vs_oracle')}), flush=True)
