set -u
mkdir -p gpurun_out
B=build/tile4_ubench
run() { echo "== $*"; timeout -k 5 120 $B "$@" || { echo "rc=$?"; exit 1; }; }
{
run 100000 1000000 16 8000 16
run 100000 1000000 16 4000 8
run 1000000 100000 -16 4000 1
run 1000000 100000 -16 8000 2
run 1000000 1250000 16 16000 4
run 1000000 1250000 16 20000 5
run 1000000 1250000 16 8000 2
run 1250000 1000000 -16 20000 4
} > gpurun_out/tile7.log 2>&1
