# round 2 re-entry check: GPU suite, unit bench (regime S, with CPU baseline), regime P bench, batch sweep
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-q1}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('S', d['value'], d['kernels_ms'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --private > $O/bench_p.json 2> $O/bench_p.err || { tail $O/bench_p.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_p.json'));print('P', d['value'], d['kernels_ms'], d['roofline']['frac'], d['cpu_baseline']['value'])"
for b in 256 512 1024; do
timeout -k 10 300 python bench.py --private --batch $b --steps 3 --no-cpu-baseline > $O/bench_p$b.json 2>> $O/bench_p.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_p$b.json'));print('P batch $b', d['value'], d['kernels_ms'])"
done
for b in 1024 2048; do
timeout -k 10 300 python bench.py --batch $b --steps 3 --no-cpu-baseline > $O/bench_s$b.json 2>> $O/bench.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_s$b.json'));print('S batch $b', d['value'], d['kernels_ms'])"
done
