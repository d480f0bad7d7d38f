set -o pipefail
O=gpurun_out/r3l; mkdir -p $O
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_phaselift.py tests/test_gpu_pipeline.py tests/test_gpu_driver.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo "== driver bench $(date +%T)"
timeout -k 10 500 python -u bench.py --mode driver --steps 3 > $O/driver.json 2> $O/driver.err || { tail -20 $O/driver.err; exit 1; }
cut -c1-400 $O/driver.json
echo "== phaselift bench $(date +%T)"
timeout -k 10 500 python -u bench.py --mode phaselift --steps 1 --warmup 1 --no-cpu-baseline > $O/pl.json 2> $O/pl.err || { tail -20 $O/pl.err; exit 1; }
cut -c1-300 $O/pl.json
echo "== driver trace $(date +%T)"; ACE_DRIVER_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/driver -o run --output-format csv -- python3 tools/dbg/driver_once.py > $O/driver.log 2>&1 || { tail -20 $O/driver.log; exit 1; }
grep "^call" $O/driver.log
echo "== phaselift trace $(date +%T)"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pl -o run --output-format csv -- python3 bench.py --mode phaselift --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pltrace.log 2>&1 || { tail -20 $O/pltrace.log; exit 1; }
echo "== done $(date +%T)"
