# hetrd_blk on DPP sums (default now): the suites; then its block sums with one barrier (ACE_HB_SYNC1)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_hbsync; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py tests/test_gpu_pipeline.py tests/test_gpu_driver.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ACE_LIB=ablib/libace_hbsync1.so timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py > $O/tests_s1.log 2>&1 || { tail -30 $O/tests_s1.log; exit 1; }
tail -1 $O/tests_s1.log
bash tools/gpu/envab.sh ab_hbsync "--mode phaselift --steps 1 --no-cpu-baseline" - ACE_LIB=ablib/libace_hbsync1.so
