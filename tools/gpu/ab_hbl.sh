set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/hbl
ACE_LIB=ablib/libace_hblower.so timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py > gpurun_out/hbl/tests.log 2>&1 || { tail -30 gpurun_out/hbl/tests.log; exit 1; }
tail -3 gpurun_out/hbl/tests.log
bash tools/gpu/envab.sh ab_hbl "--mode phaselift --steps 1 --no-cpu-baseline" - ACE_LIB=ablib/libace_hblower.so ACE_LIB=ablib/libace_hb512_8.so ACE_LIB=ablib/libace_hb1024_4.so
