set -o pipefail
mkdir -p gpurun_out/r14
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/r14/tests.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r14/bench_unit.json 2> gpurun_out/r14/bench_unit.err &&
timeout -k 10 300 python bench.py --mode pipeline --batch 4096 --steps 1 --warmup 0 > gpurun_out/r14/pipe.json 2> gpurun_out/r14/pipe.err &&
timeout -k 10 300 python bench.py --mode phaselift --batch 512 --steps 1 --warmup 0 > gpurun_out/r14/pl.json 2> gpurun_out/r14/pl.err
echo rc=$?
