# stream stagger sweep (ACE_STAGGER = 0..3) on the unit bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r47
mkdir -p $O
for s in 0 1 2 3; do
  ACE_STAGGER=$s timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_s$s.json 2>> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_s$s.json'));print('stagger $s', d['value'], d['kernels_ms'])"
done
ACE_STAGGER=2 timeout -k 10 600 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-prof > $O/prof.log 2>&1 || { echo rocprof failed; tail -20 $O/prof.log; exit 1; }
python3 tools/timeline.py $O/prof/run_kernel_trace.csv
