set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tkeig.py tests/test_gpu_parity.py tests/test_gpu_msr.py > gpurun_out/tk3_test.log 2>&1 && \
ACE_LIB=tools/libace_tkdbg.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-regime-p --no-refine-input --steps 1 --warmup 0 > gpurun_out/tkdbg.log 2>&1 && \
ACE_TK_EIG=6 timeout -k 10 200 python bench.py --no-regime-p --no-refine-input --no-cpu-baseline > gpurun_out/tk3_b6.json 2>/dev/null && \
ACE_TK_EIG=100000 timeout -k 10 200 python bench.py --no-regime-p --no-refine-input --no-cpu-baseline > gpurun_out/tk3_ball.json 2>/dev/null && \
ACE_TK_EIG=30 timeout -k 10 200 python bench.py --no-regime-p --no-refine-input --no-cpu-baseline > gpurun_out/tk3_b30.json 2>/dev/null
echo rc=$?
