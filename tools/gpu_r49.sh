# T formed inside gyk for avok realisations: GPU suite + unit bench + trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r49
mkdir -p $O
echo "tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1 || { echo gpu tests failed; tail -40 $O/tests_gpu.log; exit 1; }
tail -2 $O/tests_gpu.log
echo "bench $(date +%T)"
timeout -k 10 600 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 python3 bench.py --variant A2nuclear --no-cpu-baseline > $O/bench_nuc.json 2>> $O/bench.err || exit 1; cat $O/bench_nuc.json
echo "rocprof $(date +%T)"
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-prof > $O/prof.log 2>&1 || { echo rocprof failed; tail -20 $O/prof.log; exit 1; }
python3 tools/timeline.py $O/prof/run_kernel_trace.csv | head -8
echo "done $(date +%T)"
