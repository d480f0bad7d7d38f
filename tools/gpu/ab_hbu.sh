# trieig grid start (default now): pipeline / driver suites; SQ counters of the PhaseLift kernels; hetrd_blk
# Hermitian-product unroll 8 / 16 on the PhaseLift line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_hbu; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pipeline.py tests/test_gpu_driver.py tests/test_gpu_phaselift.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY -d $O/sq -o run --output-format csv -- python3 bench.py --mode phaselift --iters 20 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
python3 tools/sq_summary.py $O/sq/run_counter_collection.csv > $O/sq_summary.txt; cat $O/sq_summary.txt; rm -rf $O/sq
bash tools/gpu/envab.sh ab_hbu "--mode phaselift --steps 1 --no-cpu-baseline" - ACE_LIB=ablib/libace_hb_u8.so ACE_LIB=ablib/libace_hb_u16.so
