# sub-batch stagger sweep on the current build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2s
mkdir -p $O
for S in 0 1 2 0 1 2; do
ACE_STAGGER=$S timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-regime-p > $O/bench_$S.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_$S.json'));print('stagger $S value', d['value'], d['kernels_ms'])"
done
ACE_STAGGER=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-prof --no-regime-p > $O/prof.log 2>&1 || { echo rocprof failed; tail -20 $O/prof.log; exit 1; }
python3 tools/timeline.py $O/prof/run_kernel_trace.csv | head -14
