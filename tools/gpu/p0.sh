set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --private --batch 4096 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/p0_bench.json 2> gpurun_out/p0_bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p0_prof -o p0 -- python3 bench.py --private --batch 4096 --steps 1 --warmup 1 --no-cpu-baseline --no-prof > gpurun_out/p0_prof.log 2>&1
