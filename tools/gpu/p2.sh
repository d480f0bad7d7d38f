# regime P measurement: GPU suite, private bench (+ CPU baseline), rocprof kernel stats, PMC HBM passes
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/p2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --private > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --private --no-cpu-baseline --no-prof > $O/prof.log 2>&1 || { echo rocprof failed; tail -20 $O/prof.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --private --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pmc_fetch.log 2>&1 || { echo pmc fetch failed; tail -20 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --private --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pmc_write.log 2>&1 || { echo pmc write failed; tail -20 $O/pmc_write.log; exit 1; }
echo done
