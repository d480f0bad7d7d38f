set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-p6}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --private --steps 1 --warmup 1 --no-cpu-baseline --no-prof > $O/prof.log 2>&1 || { echo rocprof failed; tail -20 $O/prof.log; exit 1; }
head -14 $O/prof/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
