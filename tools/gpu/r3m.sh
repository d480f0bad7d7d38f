# r02 v9 measurement round: default bench line (both regimes, CPU baseline), A2nuclear, rocprof
# kernel stats + timeline, PMC FETCH_SIZE / WRITE_SIZE over a full solve (regime S)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3m
mkdir -p $O
echo "tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1 || { echo gpu tests failed; tail -30 $O/tests_gpu.log; exit 1; }
tail -1 $O/tests_gpu.log
echo "bench $(date +%T)"
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('value', d['value'], d['kernels_ms'], d['roofline']['kernel'], d['roofline']['frac'], d.get('regime_P',{}).get('value'))"
echo "nuclear $(date +%T)"
timeout -k 10 600 python3 bench.py --variant A2nuclear --no-cpu-baseline --no-regime-p > $O/bench_nuc.json 2>> $O/bench.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_nuc.json'));print('nuclear', d['value'])"
echo "rocprof $(date +%T)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-prof --no-regime-p > $O/prof.log 2>&1 || { echo rocprof failed; tail -20 $O/prof.log; exit 1; }
python3 tools/timeline.py $O/prof/run_kernel_trace.csv > $O/timeline.txt
head -8 $O/timeline.txt
echo "pmc $(date +%T)"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-prof --no-regime-p > $O/pmc_fetch.log 2>&1 || { echo pmc fetch failed; tail -20 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-prof --no-regime-p > $O/pmc_write.log 2>&1 || { echo pmc write failed; tail -20 $O/pmc_write.log; exit 1; }
python3 tools/pmc_summary.py $(ls $O/pmc_fetch/*counter_collection.csv | head -1) $(ls $O/pmc_write/*counter_collection.csv | head -1) $O/pmc_hbm.json > $O/pmc_hbm.txt
head -8 $O/pmc_hbm.txt
echo "pipeline $(date +%T)"
timeout -k 10 600 python3 bench.py --mode pipeline --no-cpu-baseline > $O/bench_pipe.json 2>> $O/bench.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_pipe.json'));print('pipeline', d['value'])"
echo "done $(date +%T)"
