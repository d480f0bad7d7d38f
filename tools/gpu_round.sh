#!/bin/bash
# One GPU measurement round: smoke, GPU tests, bench lines, rocprof summaries, PMC passes.
# Usage (on the GPU box, from the repo root): bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
step tests && timeout -k 10 900 python -m pytest tests -q -m gpu > $OUT/tests_gpu.log 2>&1 || { echo gpu tests failed; tail -30 $OUT/tests_gpu.log; exit 1; }
tail -2 $OUT/tests_gpu.log
step bench && timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
step bench_nuclear && timeout -k 10 600 python bench.py --variant A2nuclear --no-cpu-baseline > $OUT/bench_nuclear.json 2>> $OUT/bench.err || exit 1
step bench_private && timeout -k 10 600 python bench.py --private --batch 1024 --no-cpu-baseline > $OUT/bench_private.json 2>> $OUT/bench.err || exit 1
step rocprof && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-prof > $OUT/prof.log 2>&1 || { echo rocprof failed; tail -20 $OUT/prof.log; exit 1; }
step pmc_fetch && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 6 --no-cpu-baseline --no-prof > $OUT/pmc_fetch.log 2>&1 || { echo pmc fetch failed; tail -20 $OUT/pmc_fetch.log; exit 1; }
step pmc_write && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 6 --no-cpu-baseline --no-prof > $OUT/pmc_write.log 2>&1 || { echo pmc write failed; tail -20 $OUT/pmc_write.log; exit 1; }
step done
