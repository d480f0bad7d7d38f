# hetrd_blk: panel width 4 against 2 on the DPP / pair form, with the panel corrections' wave sums for all q side
# by side (ACE_HB_CPAR); tests on the CPAR builds
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_hbcp; mkdir -p $O
for L in nb4_cp1 nb2_cp1; do
ACE_LIB=ablib/libace_hb$L.so timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py > $O/tests_$L.log 2>&1 || { tail -30 $O/tests_$L.log; exit 1; }
tail -1 $O/tests_$L.log
done
bash tools/gpu/envab.sh ab_hbcp "--mode phaselift --steps 1 --no-cpu-baseline" - ACE_LIB=ablib/libace_hbnb4_cp0.so ACE_LIB=ablib/libace_hbnb4_cp1.so ACE_LIB=ablib/libace_hbnb2_cp1.so
