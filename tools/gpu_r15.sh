set -o pipefail
mkdir -p gpurun_out/r15
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -x -q -p no:cacheprovider > gpurun_out/r15/tests.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r15/bench_unit.json 2> gpurun_out/r15/bench_unit.err
echo rc=$?
