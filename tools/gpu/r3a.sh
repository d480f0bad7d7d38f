# cold-start Z-step diagnostics: Jacobi sweep counts and phase times per wave
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
ACE_LIB=tools/libace_dbg.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-regime-p --steps 1 --warmup 0 > $O/dbg.txt 2> $O/err.txt || { echo failed; tail $O/err.txt; exit 1; }
grep "^1w b" $O/dbg.txt | head -60
grep "^cold" $O/dbg.txt | sort | uniq -c | sort -rn | head -20
