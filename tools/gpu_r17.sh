set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r17
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r17/pl -o run --output-format csv -- python3 bench.py --mode phaselift --batch 512 --iters 20 --steps 1 --warmup 0 --no-prof > gpurun_out/r17/pl.log 2>&1
echo rc=$?
