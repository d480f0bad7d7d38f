set -o pipefail
O=gpurun_out/r3g; mkdir -p $O
export TMPDIR=/tmp
echo "== ns skipped"
echo "== refcb skipped"
echo "== tests"; timeout -k 10 900 python -u -m pytest tests/test_gpu_driver.py tests/test_svt_kat.py tests/test_gpu_config5.py tests/test_gpu_parity.py tests/test_gpu_phaselift.py tests/test_gpu_private.py -m gpu -x -v --timeout 300 --timeout-method thread -k "config5 or config3 or config4 or four_wave or nuclear" > $O/tests.log 2>&1; rc=$?; tail -25 $O/tests.log; exit $rc
