# hetrd_blk at 512 threads per matrix (two work-groups per CU) on the lower-triangle / pair / DPP form
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_hb512n; mkdir -p $O
ACE_LIB=ablib/libace_hb512n.so timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu/envab.sh ab_hb512n "--mode phaselift --steps 1 --no-cpu-baseline" - ACE_LIB=ablib/libace_hb512n.so
