set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_phaselift.py tests/test_gpu_spectral.py > gpurun_out/hb1_test.log 2>&1; echo test rc=$?
ACE_HETRD_BLK=0 timeout -k 10 300 python bench.py --mode phaselift --no-cpu-baseline > gpurun_out/hb1_pl0.json 2>/dev/null && \
timeout -k 10 300 python bench.py --mode phaselift --no-cpu-baseline > gpurun_out/hb1_pl1.json 2>/dev/null
echo rc=$?
