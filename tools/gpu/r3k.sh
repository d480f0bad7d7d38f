set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3k
mkdir -p $O
ACE_LIB=tools/libace_stamps.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-regime-p --steps 1 --warmup 0 > $O/stamps.txt 2> $O/err.txt || { echo failed; tail $O/err.txt; exit 1; }
grep -c "" $O/stamps.txt
