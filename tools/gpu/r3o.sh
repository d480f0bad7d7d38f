set -o pipefail
O=gpurun_out/r3o; mkdir -p $O
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_parity.py tests/test_gpu_config5.py tests/test_gpu_pipeline.py tests/test_gpu_private.py -k "phaselift or nuclear or config5 or golden" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
B="--no-cpu-baseline --no-regime-p --no-refine-input"
echo "== nuclear bench $(date +%T)"
timeout -k 10 500 python -u bench.py --variant A2nuclear --steps 5 $B > $O/nuclear.json 2> $O/nuclear.err || { tail -20 $O/nuclear.err; exit 1; }
cut -c1-250 $O/nuclear.json
echo "== config5 bench $(date +%T)"
timeout -k 10 500 python -u bench.py --mode config5 --steps 3 $B > $O/config5.json 2> $O/config5.err || { tail -20 $O/config5.err; exit 1; }
cut -c1-250 $O/config5.json
for v in 2 0; do
echo "== phaselift bench blk=$v $(date +%T)"
ACE_HETRD_BLK=$v timeout -k 10 500 python -u bench.py --mode phaselift --steps 1 --warmup 1 --no-cpu-baseline > $O/pl$v.json 2> $O/pl$v.err || { tail -20 $O/pl$v.err; exit 1; }
cut -c1-250 $O/pl$v.json
done
echo "== phaselift trace $(date +%T)"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pl -o run --output-format csv -- python3 bench.py --mode phaselift --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pltrace.log 2>&1 || { tail -20 $O/pltrace.log; exit 1; }
echo "== nuclear trace $(date +%T)"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/nuc -o run --output-format csv -- python3 bench.py --variant A2nuclear --steps 1 --warmup 1 $B --no-prof > $O/nuctrace.log 2>&1 || { tail -20 $O/nuctrace.log; exit 1; }
echo "== done $(date +%T)"
