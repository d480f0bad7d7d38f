set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r20
mkdir -p $O
echo "tests $(date +%T)"
timeout -k 10 900 python3 -m pytest tests -q -m gpu > $O/tests_gpu.log 2>&1 || { echo gpu tests failed; tail -40 $O/tests_gpu.log; exit 1; }
tail -2 $O/tests_gpu.log
echo "bench $(date +%T)"
timeout -k 10 600 python3 bench.py > $O/bench_unit.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
cat $O/bench_unit.json
timeout -k 10 600 python3 bench.py --mode pipeline --steps 1 --warmup 0 --no-cpu-baseline > $O/pipe.json 2>> $O/bench.err || { echo pipe failed; tail -20 $O/bench.err; exit 1; }
cat $O/pipe.json
timeout -k 10 600 python3 bench.py --mode phaselift --batch 512 --steps 1 --warmup 0 --no-cpu-baseline > $O/pl.json 2>> $O/bench.err || { echo pl failed; tail -20 $O/bench.err; exit 1; }
cat $O/pl.json
echo "done $(date +%T)"
