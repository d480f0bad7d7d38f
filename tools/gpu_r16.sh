set -o pipefail
mkdir -p gpurun_out/r16
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "phaselift or pipeline or driver" > gpurun_out/r16/tests.log 2>&1 &&
timeout -k 10 600 python bench.py --mode phaselift --batch 512 --steps 1 --warmup 0 > gpurun_out/r16/pl.json 2> gpurun_out/r16/pl.err &&
timeout -k 10 300 python bench.py --mode pipeline --batch 4096 --steps 1 --warmup 0 > gpurun_out/r16/pipe.json 2> gpurun_out/r16/pipe.err
echo rc=$?
