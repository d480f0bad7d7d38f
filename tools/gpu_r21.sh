set -o pipefail
O=gpurun_out/r21
mkdir -p $O
ACE_LIB=$PWD/tools/libace_dbg.so timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/dbg_bench4.log 2>&1
echo rc=$?
grep -c "^wave" $O/dbg_bench4.log
