# v18 measurement round: unit bench (+ CPU baseline), A2nuclear, pipeline, PhaseLift, rocprof kernel stats + trace, PMC over a full solve
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r58
mkdir -p $O
echo "bench $(date +%T)"
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 python3 bench.py --variant A2nuclear --no-cpu-baseline > $O/bench_nuc.json 2>> $O/bench.err || exit 1
echo "pipeline $(date +%T)"
timeout -k 10 600 python3 bench.py --mode pipeline --no-cpu-baseline > $O/bench_pipe.json 2>> $O/bench.err || exit 1
echo "phaselift $(date +%T)"
timeout -k 10 600 python3 bench.py --mode phaselift --batch 512 --steps 1 --warmup 0 --no-cpu-baseline > $O/bench_pl.json 2>> $O/bench.err || exit 1
echo "rocprof $(date +%T)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-prof > $O/prof.log 2>&1 || { echo rocprof failed; tail -20 $O/prof.log; exit 1; }
python3 tools/timeline.py $O/prof/run_kernel_trace.csv > $O/timeline.txt
echo "pmc $(date +%T)"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pmc_fetch.log 2>&1 || { echo pmc fetch failed; tail -20 $O/pmc_fetch.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pmc_write.log 2>&1 || { echo pmc write failed; tail -20 $O/pmc_write.log; exit 1; }
echo "done $(date +%T)"
