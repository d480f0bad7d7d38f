set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/h2b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_heev2.py -x -v --timeout 120 --timeout-method thread > $O/t1.log 2>&1; rc=$?
tail -14 $O/t1.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pl -o run --output-format csv -- python3 bench.py --mode phaselift --iters 20 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pl.log 2>&1 || { tail -20 $O/pl.log; exit 1; }
cp $O/pl/run_kernel_stats.csv $O/pl_kernel_stats.csv; head -8 $O/pl_kernel_stats.csv | cut -c1-160
rm -rf $O/pl
