# phase stamps of gyk (lazy) and the fused apply_AH (work-group 5)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2p
mkdir -p $O
ACE_LIB=tools/libace_stamps.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-regime-p --steps 1 --warmup 1 > $O/stamps.txt 2> $O/err.txt || { echo failed; tail $O/err.txt; exit 1; }
grep "gyk-lazy\|i8ah-fused" $O/stamps.txt | awk 'NR>250 && NR<=400' | head -20
