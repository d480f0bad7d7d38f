#!/bin/bash
# Generic GPU-box step runner: bash tools/gpu/run.sh <tag> <step>...
# steps: smoke | tests[:<pytest -k expr or file>] | bench[:<bench args, comma-separated>] | trace:<bench args>
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
i=0
for s in "$@"; do
  i=$((i+1))
  echo "== $i $s $(date +%T)"
  case $s in
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/$i.smoke.log 2>&1 || { tail -30 $O/$i.smoke.log; exit 1; } ; tail -3 $O/$i.smoke.log ;;
    tests) timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/$i.tests.log 2>&1 || { tail -40 $O/$i.tests.log; exit 1; } ; tail -3 $O/$i.tests.log ;;
    testsall) timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/$i.tests.log 2>&1; rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/$i.tests.log | tail -30; [ $rc -eq 0 ] || exit 1 ;;
    tests:*) t=${s#tests:}; t=${t//,/ }; timeout -k 10 1000 python -u -m pytest $t -m gpu -x -v --timeout 300 --timeout-method thread > $O/$i.tests.log 2>&1 || { tail -40 $O/$i.tests.log; exit 1; } ; tail -3 $O/$i.tests.log ;;
    bench:*) a=${s#bench:}; a=${a//,/ }; timeout -k 10 600 python -u bench.py $a > $O/$i.bench.json 2> $O/$i.bench.err || { tail -30 $O/$i.bench.err; exit 1; } ; cat $O/$i.bench.json ;;
    trace:*) a=${s#trace:}; a=${a//,/ }; timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-regime-p --no-refine-input --no-configs --no-prof $a > $O/$i.trace.log 2>&1 || { tail -30 $O/$i.trace.log; exit 1; } ; python3 tools/iter_buckets.py $O/trace$i/run_kernel_trace.csv > $O/$i.buckets.txt; cat $O/$i.buckets.txt ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
