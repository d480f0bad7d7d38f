# trieig: Newton-accelerated eigenvalues and 2 inverse-iteration solves, tests then the PhaseLift line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_te
ACE_LIB=ablib/libace_te_both.so timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py > gpurun_out/ab_te/tests.log 2>&1 || { tail -30 gpurun_out/ab_te/tests.log; exit 1; }
tail -2 gpurun_out/ab_te/tests.log
ACE_LIB=ablib/libace_te_bothst.so timeout -k 10 300 python3 -u bench.py --mode phaselift --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/ab_te/st.out 2> gpurun_out/ab_te/st.err || { tail -20 gpurun_out/ab_te/st.err; exit 1; }
bash tools/gpu/envab.sh ab_te "--mode phaselift --steps 1 --no-cpu-baseline" - ACE_LIB=ablib/libace_te_newton.so ACE_LIB=ablib/libace_te_sw2.so ACE_LIB=ablib/libace_te_both.so
