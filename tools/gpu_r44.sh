# Measurement round: unit bench, rocprof kernel stats, PMC FETCH/WRITE passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r44
mkdir -p $O
echo "bench $(date +%T)"
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo "rocprof $(date +%T)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/prof.log 2>&1 || { echo rocprof failed; tail -20 $O/prof.log; exit 1; }
echo "pmc $(date +%T)"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 30 --no-cpu-baseline --no-prof > $O/pmc_fetch.log 2>&1 || { echo pmc fetch failed; tail -20 $O/pmc_fetch.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 30 --no-cpu-baseline --no-prof > $O/pmc_write.log 2>&1 || { echo pmc write failed; tail -20 $O/pmc_write.log; exit 1; }
timeout -k 10 600 python3 bench.py --variant A2nuclear --no-cpu-baseline > $O/bench_nuc.json 2>> $O/bench.err && cat $O/bench_nuc.json && timeout -k 10 600 python3 bench.py --mode pipeline --no-cpu-baseline > $O/bench_pipe.json 2>> $O/bench.err && cat $O/bench_pipe.json || exit 1
echo "done $(date +%T)"
