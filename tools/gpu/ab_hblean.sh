# hetrd_blk with single-barrier DPP block sums (default now): the suites; then zlarfg in every thread and no
# correction barriers at the panel's first column (ACE_HB_LEAN)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_hblean; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py tests/test_gpu_pipeline.py tests/test_gpu_driver.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ACE_LIB=ablib/libace_hblean.so timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py tests/test_gpu_pipeline.py > $O/tests_lean.log 2>&1 || { tail -30 $O/tests_lean.log; exit 1; }
tail -1 $O/tests_lean.log
bash tools/gpu/envab.sh ab_hblean "--mode phaselift --steps 1 --no-cpu-baseline" - ACE_LIB=ablib/libace_hblean.so
