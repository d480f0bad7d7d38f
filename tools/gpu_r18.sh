set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r18
timeout -k 10 300 python3 tools/bf_parity_count.py > gpurun_out/r18/parity_count.log 2>&1 && \
timeout -k 10 300 python3 bench.py --mode beamformer --steps 5 --warmup 2 > gpurun_out/r18/bench_bf.json 2> gpurun_out/r18/bench_bf.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r18/prof -o run --output-format csv -- python3 bench.py --mode beamformer --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r18/bench_bf_prof.log 2>&1
echo rc=$?
cat gpurun_out/r18/parity_count.log; cat gpurun_out/r18/bench_bf.json; tail -3 gpurun_out/r18/bench_bf.err
