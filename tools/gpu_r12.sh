set -o pipefail
mkdir -p gpurun_out/r12
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/r12/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --mode phaselift --batch 64 --iters 200 --steps 1 --warmup 0 > gpurun_out/r12/pl64.json 2> gpurun_out/r12/pl64.err &&
timeout -k 10 600 python bench.py --mode phaselift --batch 512 --iters 200 --steps 1 --warmup 0 > gpurun_out/r12/pl512.json 2> gpurun_out/r12/pl512.err
echo rc=$?
