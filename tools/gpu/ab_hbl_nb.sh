# lower-triangle hetrd_blk (default now): the suites that run it; its panel width 8 / 2 against 4
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_hbl_nb; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py tests/test_gpu_pipeline.py tests/test_gpu_driver.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu/envab.sh ab_hbl_nb "--mode phaselift --steps 1 --no-cpu-baseline" - ACE_LIB=ablib/libace_hbl_nb8.so ACE_LIB=ablib/libace_hbl_nb2.so
