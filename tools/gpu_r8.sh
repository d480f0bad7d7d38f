set -o pipefail
mkdir -p gpurun_out/r8
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r8/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r8/bench_unit.json 2> gpurun_out/r8/bench_unit.err &&
timeout -k 10 300 python bench.py --mode pipeline --batch 1024 --steps 1 --warmup 0 > gpurun_out/r8/pipe1024.json 2> gpurun_out/r8/pipe1024.err &&
timeout -k 10 500 python bench.py --mode pipeline --batch 4096 --steps 1 --warmup 0 > gpurun_out/r8/pipe4096.json 2> gpurun_out/r8/pipe4096.err
echo rc=$?
