# Kernel traces of the unit bench (one timed step) under variant env settings: trace_unit.sh <tag> [ENV=VAL ...]
set -o pipefail
T=$1; shift
O=gpurun_out/tr_$T; mkdir -p $O; export TMPDIR=/tmp
export "$@"; timeout -k 10 300 rocprofv3 --kernel-trace -d $O/raw -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-regime-p --no-refine-input --no-configs --no-prof --steps 1 --warmup 1 > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
cp $O/raw/run_kernel_trace.csv $O/trace.csv && rm -rf $O/raw
