# gyf (gyk + fused apply_AH in one launch): parity file, bench A/B, trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "gyf_ragged or lean or compact or fused" -m gpu --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1 || { echo gpu tests failed; tail -30 $O/tests_gpu.log; exit 1; }
tail -1 $O/tests_gpu.log
for L in 1; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-regime-p > $O/bench_$L.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_$L.json'));print('run $L value', d['value'], d['kernels_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-prof --no-regime-p > $O/prof.log 2>&1 || { echo rocprof failed; tail -20 $O/prof.log; exit 1; }
python3 tools/timeline.py $O/prof/run_kernel_trace.csv > $O/timeline.txt
head -14 $O/timeline.txt
