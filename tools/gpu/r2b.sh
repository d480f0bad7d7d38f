# lean Z-step: parity tests, then unit bench with and without it
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2b
mkdir -p $O
echo "tests $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1 || { echo gpu tests failed; tail -30 $O/tests_gpu.log; exit 1; }
tail -2 $O/tests_gpu.log
for L in 1 0 1; do
echo "bench lean=$L $(date +%T)"
ACE_LEAN=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-regime-p > $O/bench_l$L.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_l$L.json'));print('value', d['value'], d['kernels_ms'])"
done
echo "done $(date +%T)"
