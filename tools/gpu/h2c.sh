set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/h2c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_heev2.py tests/test_gpu_phaselift.py -k "heev2 or two_stage or reduction_paths or config4_geometry" -x -q --timeout 120 --timeout-method thread > $O/t1.log 2>&1; rc=$?
tail -3 $O/t1.log
[ $rc -eq 0 ] || exit 1
ACE_LIB=$PWD/ablib/libace_h2s.so timeout -k 10 120 python bench.py --mode phaselift --iters 2 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/s.json 2> $O/s.err || { tail -5 $O/s.err; exit 1; }
grep -E "he2hb|hb2st" $O/s.err | head -12
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pl -o run --output-format csv -- python3 bench.py --mode phaselift --iters 20 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pl.log 2>&1 || { tail -20 $O/pl.log; exit 1; }
cp $O/pl/run_kernel_stats.csv $O/pl_kernel_stats.csv
rm -rf $O/pl
python3 -c "
import csv
for r in csv.DictReader(open('$O/pl_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3), r['Percentage'])
" | head -10 || true
