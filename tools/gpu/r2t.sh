# gyk T-phase batching: GPU parity file, bench, stamps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2t
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1 || { echo gpu tests failed; tail -30 $O/tests_gpu.log; exit 1; }
tail -1 $O/tests_gpu.log
for r in 1 2; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-regime-p > $O/bench_$r.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_$r.json'));print('value', d['value'], d['kernels_ms'])"
done
ACE_LIB=tools/libace_stamps.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-regime-p --steps 1 --warmup 1 > $O/stamps.txt 2> $O/err.txt || { echo failed; tail $O/err.txt; exit 1; }
grep "gyk-lazy\|i8ah-fused" $O/stamps.txt | awk 'NR>250 && NR<=400' | head -8
