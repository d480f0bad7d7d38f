# lower-triangle hetrd_blk (default now): the suites that run it; panel width 8 / 2 against 4; the trailing
# update with 4 / 6 / 8 rows per round trip, and by balanced column pairs (2 / 4 rows per round trip)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_hbl_nb; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py tests/test_gpu_pipeline.py tests/test_gpu_driver.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ACE_LIB=ablib/libace_hbtp1_tb4.so timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py > $O/tests_tp.log 2>&1 || { tail -30 $O/tests_tp.log; exit 1; }
tail -1 $O/tests_tp.log
bash tools/gpu/envab.sh ab_hbl_nb "--mode phaselift --steps 1 --no-cpu-baseline" - ACE_LIB=ablib/libace_hbl_nb8.so ACE_LIB=ablib/libace_hbl_nb2.so ACE_LIB=ablib/libace_hbtb4.so ACE_LIB=ablib/libace_hbtb6.so ACE_LIB=ablib/libace_hbtb8.so ACE_LIB=ablib/libace_hbtp1_tb2.so ACE_LIB=ablib/libace_hbtp1_tb4.so
