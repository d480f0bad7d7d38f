set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tkeig.py tests/test_gpu_parity.py tests/test_gpu_msr.py tests/test_gpu_pipeline.py tests/test_gpu_refine.py > gpurun_out/tk3_test.log 2>&1 && \
ACE_LIB=tools/libace_tkdbg.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-regime-p --no-refine-input --steps 1 --warmup 0 > gpurun_out/tkdbg.log 2>&1 && \
ACE_TK_EIG=6 timeout -k 10 200 python bench.py --no-regime-p --no-refine-input --no-cpu-baseline > gpurun_out/tk3_b6.json 2>/dev/null && \
ACE_TK_EIG=100000 timeout -k 10 200 python bench.py --no-regime-p --no-refine-input --no-cpu-baseline > gpurun_out/tk3_ball.json 2>/dev/null && \
ACE_TK_EIG=0 timeout -k 10 300 python bench.py --mode pipeline --no-cpu-baseline > gpurun_out/tk3_p0.json 2>/dev/null && \
ACE_TK_EIG=6 timeout -k 10 300 python bench.py --mode pipeline --no-cpu-baseline > gpurun_out/tk3_p6.json 2>/dev/null && \
ACE_TK_EIG=100000 timeout -k 10 300 python bench.py --mode pipeline --no-cpu-baseline > gpurun_out/tk3_pall.json 2>/dev/null
echo rc=$?
