# fused apply_AH v3 (control in the Z-step): GPU suite, bench A/B, trace, stamps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2n
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1 || { echo gpu tests failed; tail -30 $O/tests_gpu.log; exit 1; }
tail -1 $O/tests_gpu.log
for L in 1 0; do
ACE_FUSE=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-regime-p > $O/bench_$L.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_$L.json'));print('fuse $L value', d['value'], d['kernels_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-prof --no-regime-p > $O/prof.log 2>&1 || { echo rocprof failed; tail -20 $O/prof.log; exit 1; }
python3 tools/timeline.py $O/prof/run_kernel_trace.csv > $O/timeline.txt
head -14 $O/timeline.txt
ACE_LIB=tools/libace_stamps.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-regime-p --steps 1 --warmup 1 > $O/stamps.txt 2> $O/err.txt || { echo failed; tail $O/err.txt; exit 1; }
grep "i8ah-fused" $O/stamps.txt | awk 'NR>250 && NR<=400' | head -12
