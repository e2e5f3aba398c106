set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_plugins.py > gpurun_out/dore_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "
import sys, json; sys.path.insert(0, '.'); sys.path.insert(0, 'block-simplex-least-squares_amd')
import bench
sh, b = bench.build_problem('C3', 1, 0, None)
print(json.dumps(bench.bench_dore(sh, b)))
" > gpurun_out/dore_bench.log 2>&1
echo "bench rc=$?"
