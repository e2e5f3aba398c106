"""bench.py's x-space BB leg alone on the C3 problem (GPU box)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))
import bench  # noqa: E402
from synthetic import make_shard, add_noise, SEED  # noqa: E402

sh = make_shard(1_000_000, 50_000, 100_000, 16, seed=SEED)
b = add_noise(sh['Ax'], 0.02, seed=SEED)
print(json.dumps(bench.bench_xspace(sh, b)), flush=True)
