# round-2 re-entry check: GPU suite + unit bench (both regimes)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2a
mkdir -p $O
echo "tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1 || { echo gpu tests failed; tail -30 $O/tests_gpu.log; exit 1; }
tail -2 $O/tests_gpu.log
echo "bench $(date +%T)"
timeout -k 10 600 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('value', d['value'], d['kernels_ms'], d.get('regime_P',{}).get('value'))"
echo "done $(date +%T)"
