set -o pipefail
export TMPDIR=/tmp
ACE_LIB=$PWD/tools/libace_dbg.so timeout -k 10 300 python3 tools/dbg_msp1.py 4096 256 32 12 1 > gpurun_out/sweeps.log 2>&1 || { tail gpurun_out/sweeps.log; exit 1; }
grep -c cold gpurun_out/sweeps.log
