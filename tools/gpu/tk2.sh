set -o pipefail
ACE_LIB=tools/libace_tkdbg.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-regime-p --no-refine-input --steps 1 --warmup 0 > gpurun_out/tkdbg.log 2>&1 && \
ACE_LIB=tools/libace_tkdbg.so timeout -k 10 300 python bench.py --mode pipeline --batch 1024 --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/zs4dbg.log 2>&1 && \
ACE_MSR_TRACE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-regime-p --no-refine-input --steps 1 --warmup 1 > gpurun_out/msrw.json 2> gpurun_out/msrw.err && \
bash tools/gpu/trace_unit.sh tk6 ACE_TK_EIG=6 && bash tools/gpu/trace_unit.sh tk0 ACE_TK_EIG=0
