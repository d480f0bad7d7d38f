set -o pipefail
O=gpurun_out/r3m; mkdir -p $O
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_pipeline.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for v in 2 0; do
echo "== phaselift bench blk=$v $(date +%T)"
ACE_HETRD_BLK=$v timeout -k 10 500 python -u bench.py --mode phaselift --steps 1 --warmup 1 --no-cpu-baseline > $O/pl$v.json 2> $O/pl$v.err || { tail -20 $O/pl$v.err; exit 1; }
cut -c1-300 $O/pl$v.json
done
echo "== phaselift trace $(date +%T)"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pl -o run --output-format csv -- python3 bench.py --mode phaselift --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pltrace.log 2>&1 || { tail -20 $O/pltrace.log; exit 1; }
echo "== done $(date +%T)"
