set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r22
mkdir -p $O
timeout -k 10 900 python3 -m pytest tests -q -m gpu > $O/tests_gpu.log 2>&1 || { echo gpu tests failed; tail -40 $O/tests_gpu.log; exit 1; }
tail -1 $O/tests_gpu.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_unit.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_unit.json')); print(d['value'], d['kernels_ms'])"
timeout -k 10 600 python3 bench.py --mode pipeline --steps 1 --warmup 0 --no-cpu-baseline > $O/pipe.json 2>> $O/bench.err || { echo pipe failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/pipe.json')); print(d['value'], d['kernels_total_ms'])"
