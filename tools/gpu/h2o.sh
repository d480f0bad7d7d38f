set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/h2o; mkdir -p $O
ACE_LIB=ablib/libace_h2s.so timeout -k 10 300 python bench.py --mode phaselift --batch 512 --iters 4 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
grep "^hb2st" $O/stamps.log | head -12
grep "^he2hb" $O/stamps.log | head -4
