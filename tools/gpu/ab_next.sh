# trieig phase stamps on the PhaseLift line; m-space run start / retry on the unit and refine lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/testamps
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py tests/test_gpu_pipeline.py > gpurun_out/testamps/tests.log 2>&1 || { tail -30 gpurun_out/testamps/tests.log; exit 1; }
tail -2 gpurun_out/testamps/tests.log
ACE_LIB=ablib/libace_testamps.so timeout -k 10 300 python3 -u bench.py --mode phaselift --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/testamps/pl.json 2> gpurun_out/testamps/pl.err || { tail -20 gpurun_out/testamps/pl.err; exit 1; }
grep "trieig b" gpurun_out/testamps/pl.err | head -12
bash tools/gpu/envab.sh ab_msrstart "--no-cpu-baseline --no-regime-p --no-refine-input --steps 5" - "ACE_MSR_START=64 ACE_MSR_RETRY=4" "ACE_MSR_START=70 ACE_MSR_RETRY=2" && \
bash tools/gpu/envab.sh ab_msrstart_ref "--mode refine --steps 3 --no-cpu-baseline" - "ACE_MSR_START=64 ACE_MSR_RETRY=4" "ACE_MSR_START=70 ACE_MSR_RETRY=2"
