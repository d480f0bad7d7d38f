set -o pipefail
export TMPDIR=/tmp
echo "cfg 1024 256 32 200 fixed"; timeout -k 10 300 python3 tools/dbg_msp.py 1024 256 32 200 1 || exit 1
echo "cfg 1024 256 32 500 conv"; timeout -k 10 300 python3 tools/dbg_msp.py 1024 256 32 500 0 || exit 1
echo "cfg 600 121 16 200 fixed"; timeout -k 10 300 python3 tools/dbg_msp.py 600 121 16 200 1 || exit 1
echo "cfg 64 256 32 300 conv"; timeout -k 10 300 python3 tools/dbg_msp.py 64 256 32 300 0 || exit 1
mkdir -p gpurun_out/p1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p1 -o p1 --output-format csv -- python3 tools/dbg_msp1.py 4096 256 32 200 1 > /dev/null 2>&1 || exit 1
cut -d, -f1-5 gpurun_out/p1/p1_kernel_stats.csv | head -9 | cut -c1-60,200-
