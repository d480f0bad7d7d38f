# trieig with 2 inverse-iteration solves (default): the suites that run it, then the 16-row prefetch and the
# dstebz absolute tolerance A/B, then the suites on the absolute-tolerance build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_te2
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py tests/test_gpu_pipeline.py tests/test_gpu_driver.py > gpurun_out/ab_te2/tests.log 2>&1 || { tail -30 gpurun_out/ab_te2/tests.log; exit 1; }
tail -2 gpurun_out/ab_te2/tests.log
bash tools/gpu/envab.sh ab_te2 "--mode phaselift --steps 1 --no-cpu-baseline" - ACE_LIB=ablib/libace_te_pf16.so ACE_LIB=ablib/libace_te_abstol.so || exit 1
ACE_LIB=ablib/libace_te_abstol.so timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py tests/test_gpu_pipeline.py > gpurun_out/ab_te2/tests_abstol.log 2>&1 || { tail -30 gpurun_out/ab_te2/tests_abstol.log; exit 1; }
tail -2 gpurun_out/ab_te2/tests_abstol.log
