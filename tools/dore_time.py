"""DORE on the device (bsls_dore_iterate) on the C3 problem: bench.py's dore
leg alone.  python tools/dore_time.py [iterations]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'block-simplex-least-squares_amd'))


def main():
    import bench
    sh, b = bench.build_problem('C3', 1, 0, None)
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    print(json.dumps(bench.bench_dore(sh, b, iters=iters)), flush=True)


if __name__ == '__main__':
    main()
