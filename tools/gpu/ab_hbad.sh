# hetrd_blk with the thread map following the trailing order (ACE_HB_ADAPT) and trieig from a shared grid of
# Sturm counts (ACE_TE_GRID): tests on each build, then the PhaseLift line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_hbad
for L in hbadapt tegrid; do
ACE_LIB=ablib/libace_$L.so timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py > gpurun_out/ab_hbad/tests_$L.log 2>&1 || { tail -30 gpurun_out/ab_hbad/tests_$L.log; exit 1; }
tail -1 gpurun_out/ab_hbad/tests_$L.log
done
bash tools/gpu/envab.sh ab_hbad "--mode phaselift --steps 1 --no-cpu-baseline" - ACE_LIB=ablib/libace_hbadapt.so ACE_LIB=ablib/libace_hbadapt_nb8.so ACE_LIB=ablib/libace_hbadapt_nb3.so ACE_LIB=ablib/libace_tegrid.so
