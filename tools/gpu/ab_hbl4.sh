# hetrd_blk from the lower triangle only (ACE_HB_LOWER, DPP row sums) at panel width 4: tests, A/B, HBM PMC
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_hbl4; mkdir -p $O
ACE_LIB=ablib/libace_hblower4.so timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_spectral.py tests/test_gpu_pipeline.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu/envab.sh ab_hbl4 "--mode phaselift --steps 1 --no-cpu-baseline" - ACE_LIB=ablib/libace_hblower4.so || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  ACE_LIB=ablib/libace_hblower4.so timeout -k 10 -s KILL 300 rocprofv3 --pmc $c -d $O/$c -o run --output-format csv -- python3 bench.py --mode phaselift --iters 20 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
done
python3 tools/pmc_summary.py $O/FETCH_SIZE/run_counter_collection.csv $O/WRITE_SIZE/run_counter_collection.csv $O/pmc.json 512 phaselift > $O/pmc.txt; head -4 $O/pmc.txt; rm -rf $O/FETCH_SIZE $O/WRITE_SIZE
bash tools/gpu/ab_tefuse.sh
