# Measurement round: smoke, full GPU suite, unit bench (default), rocprof kernel stats, PMC FETCH/WRITE passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r25
mkdir -p $O
echo "smoke $(date +%T)"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "tests $(date +%T)"
timeout -k 10 900 python3 -m pytest tests -q -m gpu > $O/tests_gpu.log 2>&1 || { echo gpu tests failed; tail -30 $O/tests_gpu.log; exit 1; }
tail -1 $O/tests_gpu.log
echo "bench $(date +%T)"
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo "rocprof $(date +%T)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-prof > $O/prof.log 2>&1 || { echo rocprof failed; tail -20 $O/prof.log; exit 1; }
echo "pmc $(date +%T)"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 30 --no-cpu-baseline --no-prof > $O/pmc_fetch.log 2>&1 || { echo pmc fetch failed; tail -20 $O/pmc_fetch.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 30 --no-cpu-baseline --no-prof > $O/pmc_write.log 2>&1 || { echo pmc write failed; tail -20 $O/pmc_write.log; exit 1; }
echo "done $(date +%T)"
