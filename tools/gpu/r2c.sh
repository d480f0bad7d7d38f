# kernel trace of the unit bench (lean Z-step)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2c
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-prof --no-regime-p > $O/prof.log 2>&1 || { echo rocprof failed; tail -20 $O/prof.log; exit 1; }
python3 tools/timeline.py $O/prof/run_kernel_trace.csv > $O/timeline.txt
head -40 $O/timeline.txt
