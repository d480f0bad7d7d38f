# PhaseLift elementwise kernels: x_old / z_old copy with 16-B accesses, take_z and assemble by LDS tiles, wy_larft's
# G row / tau loaded a step ahead (all the same values): tests, then the line A/B against the previous build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_pl; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu/envab.sh ab_pl "--mode phaselift --steps 1 --no-cpu-baseline" ACE_LIB=ablib/libace_prev.so -
