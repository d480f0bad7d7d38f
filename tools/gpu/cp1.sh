set -o pipefail
timeout -k 10 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msr.py tests/test_gpu_refine.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_tkeig.py tests/test_gpu_private.py tests/test_gpu_driver.py > gpurun_out/cp1_test.log 2>&1 && \
timeout -k 10 200 python bench.py --no-regime-p --no-refine-input --no-cpu-baseline > gpurun_out/cp1_unit.json 2>/dev/null && \
timeout -k 10 300 python bench.py --mode refine --no-cpu-baseline > gpurun_out/cp1_refine.json 2>/dev/null && \
timeout -k 10 300 python bench.py --mode pipeline --no-cpu-baseline > gpurun_out/cp1_pipe.json 2>/dev/null
echo rc=$?
