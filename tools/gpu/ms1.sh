set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msr.py tests/test_gpu_refine.py tests/test_gpu_tkeig.py > gpurun_out/ms1_test.log 2>&1 && \
ACE_MSR_PARTIAL=0 ACE_MSR_START=56 timeout -k 10 200 python bench.py --no-regime-p --no-refine-input --no-cpu-baseline > gpurun_out/ms1_base.json 2>/dev/null && \
ACE_MSR_PARTIAL=50 ACE_MSR_START=56 timeout -k 10 200 python bench.py --no-regime-p --no-refine-input --no-cpu-baseline > gpurun_out/ms1_p50s56.json 2>/dev/null && \
ACE_MSR_PARTIAL=50 ACE_MSR_START=40 ACE_MSR_TRACE=1 timeout -k 10 200 python bench.py --no-regime-p --no-refine-input --no-cpu-baseline > gpurun_out/ms1_p50s40.json 2>gpurun_out/ms1_p50s40.err && \
ACE_MSR_PARTIAL=150 ACE_MSR_START=32 timeout -k 10 200 python bench.py --no-regime-p --no-refine-input --no-cpu-baseline > gpurun_out/ms1_p150s32.json 2>/dev/null && \
ACE_MSR_PARTIAL=150 ACE_MSR_START=32 ACE_MSR_RETRY=4 timeout -k 10 200 python bench.py --no-regime-p --no-refine-input --no-cpu-baseline > gpurun_out/ms1_p150s32r4.json 2>/dev/null && \
ACE_TK_EIG=2 timeout -k 10 200 python bench.py --no-regime-p --no-refine-input --no-cpu-baseline > gpurun_out/ms1_tk2.json 2>/dev/null && \
ACE_MSR_PARTIAL=50 ACE_MSR_START=40 timeout -k 10 300 python bench.py --mode refine --no-cpu-baseline > gpurun_out/ms1_refine.json 2>/dev/null
echo rc=$?
