set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/h2d; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_heev2.py tests/test_gpu_phaselift.py -x -q --timeout 300 --timeout-method thread > $O/t1.log 2>&1; rc=$?
tail -3 $O/t1.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/t1.log | head -20; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pl -o run --output-format csv -- python3 bench.py --mode phaselift --iters 20 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pl.log 2>&1 || { tail -20 $O/pl.log; exit 1; }
cp $O/pl/run_kernel_stats.csv $O/pl_kernel_stats.csv
rm -rf $O/pl
python3 tools/kstats.py $O/pl_kernel_stats.csv 12
timeout -k 10 300 python bench.py --mode phaselift --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_pl.json 2> $O/bench_pl.err || { tail -20 $O/bench_pl.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_pl.json').read().strip().splitlines()[-1]); print('phaselift', d['value'], d['ms_per_step'])"
