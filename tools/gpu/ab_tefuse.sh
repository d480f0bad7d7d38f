# trieig with the inverse iteration's normalisation folded into the next solve's loads and the vector written out
# 32 rows per round trip (ACE_TE_FUSE): tests, then the PhaseLift line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_tefuse; mkdir -p $O
ACE_LIB=ablib/libace_tefuse.so timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py tests/test_gpu_pipeline.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu/envab.sh ab_tefuse "--mode phaselift --steps 1 --no-cpu-baseline" - ACE_LIB=ablib/libace_tefuse.so
