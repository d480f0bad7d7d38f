# Phase timestamps of hb2st_kernel / he2hb_kernel / trieig_kernel from the stamped build:
#   make -C 2ace-mmwave-channel-estimation_amd/csrc OUT=../../ablib/libace_h2s.so BLD=build_h2s EXTRA=-DACE_H2_STAMPS
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/heev2_stamps; mkdir -p $O
ACE_LIB=ablib/libace_h2s.so timeout -k 10 300 python bench.py --mode phaselift --batch 512 --iters 4 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
grep "^hb2st" $O/stamps.log | head -12
grep "^he2hb" $O/stamps.log | head -4
