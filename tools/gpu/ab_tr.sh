# hetrd_blk lower-triangle product with 2 rows per lane and task (8 loads per round trip; ACE_HB_TR=2)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_tr; mkdir -p $O
ACE_LIB=ablib/libace_tr2.so timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu/envab.sh ab_tr "--mode phaselift --steps 1 --no-cpu-baseline" - ACE_LIB=ablib/libace_tr2.so
