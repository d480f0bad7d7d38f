set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tkeig.py tests/test_gpu_parity.py > gpurun_out/tk1_test.log 2>&1 && \
ACE_TK_EIG=0 timeout -k 10 200 python bench.py --no-regime-p --no-refine-input --no-cpu-baseline > gpurun_out/tk1_b0.json 2>/dev/null && \
ACE_TK_EIG=6 ACE_TK_TRACE=1 timeout -k 10 200 python bench.py --no-regime-p --no-refine-input --no-cpu-baseline > gpurun_out/tk1_b6.json 2>gpurun_out/tk1_b6.err && \
ACE_TK_EIG=20 timeout -k 10 200 python bench.py --no-regime-p --no-refine-input --no-cpu-baseline > gpurun_out/tk1_b20.json 2>/dev/null && \
ACE_TK_EIG=100000 timeout -k 10 200 python bench.py --no-regime-p --no-refine-input --no-cpu-baseline > gpurun_out/tk1_ball.json 2>/dev/null
echo rc=$?
