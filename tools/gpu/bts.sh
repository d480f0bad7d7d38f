set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/bts; mkdir -p $O
ACE_LIB=$PWD/ablib/libace_bts.so timeout -k 10 300 python bench.py --mode phaselift --iters 3 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/b.json 2> $O/b.err; rc=$?
grep bt2 $O/b.err | head -40
exit $rc
