set -o pipefail
O=gpurun_out/r3g; mkdir -p $O
export TMPDIR=/tmp
echo "== ns"; ACE_LIB=tools/libace_dbg.so timeout -k 10 200 python -u tools/dbg/ns_972.py 2>&1 | tail -8 || exit 1
echo "== refcb"; timeout -k 10 200 python -u tools/dbg/refcb_1024.py || exit 1
echo "== tests"; timeout -k 10 900 python -u -m pytest tests/test_gpu_driver.py tests/test_svt_kat.py tests/test_gpu_config5.py tests/test_gpu_parity.py tests/test_gpu_phaselift.py tests/test_gpu_private.py -m gpu -x -v --timeout 300 --timeout-method thread -k "driver or svt or prox or config5 or config3 or config4 or four_wave or nuclear" > $O/tests.log 2>&1; rc=$?; tail -25 $O/tests.log; exit $rc
