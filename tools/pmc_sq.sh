set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/gemmpmc
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $O/p1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 6 --no-cpu-baseline --no-prof > $O/p1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS -d $O/p2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 6 --no-cpu-baseline --no-prof > $O/p2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d $O/p3 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 6 --no-cpu-baseline --no-prof > $O/p3.log 2>&1
