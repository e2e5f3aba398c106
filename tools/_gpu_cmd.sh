set -u
mkdir -p gpurun_out
{
for V in "" _nt; do
  echo "== variant '$V' C5"; BSLS_LIB=block-simplex-least-squares_amd/lib/libbsls_hip$V.so timeout -k 10 200 python tools/stage_time.py --iters 50 --reps 10 --shape C5 | grep -E "K1|K2|iteration" || exit 1
  echo "== variant '$V' shard"; BSLS_LIB=block-simplex-least-squares_amd/lib/libbsls_hip$V.so timeout -k 10 200 python tools/stage_time.py --iters 50 --reps 10 --shape C5 --world 8 | grep -E "K1|K2|iteration" || exit 1
done
} > gpurun_out/st18.log 2>&1
echo "stage rc=$?"
