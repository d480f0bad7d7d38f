# hetrd_blk combinations: balanced column-pair trailing update with 4 rows per round trip (R = at NB 4), at panel
# width 2 (A) / 3 (D), with the product's task prefetch (B: NB 2, C: NB 4); E: A with the next panel's columns
# kept in LDS by the trailing update (ACE_HB_PCOL); tests on A, B and E
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_hbc; mkdir -p $O
for L in A B E; do
ACE_LIB=ablib/libace_hbc$L.so timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py > $O/tests_$L.log 2>&1 || { tail -30 $O/tests_$L.log; exit 1; }
tail -1 $O/tests_$L.log
done
bash tools/gpu/envab.sh ab_hbc "--mode phaselift --steps 1 --no-cpu-baseline" ACE_LIB=ablib/libace_hbcR.so ACE_LIB=ablib/libace_hbcA.so ACE_LIB=ablib/libace_hbcB.so ACE_LIB=ablib/libace_hbcC.so ACE_LIB=ablib/libace_hbcD.so ACE_LIB=ablib/libace_hbcE.so
