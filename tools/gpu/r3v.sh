set -o pipefail
O=gpurun_out/r3v; mkdir -p $O
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_spectral.py tests/test_gpu_phaselift.py tests/test_gpu_pipeline.py tests/test_svt_kat.py tests/test_gpu_driver.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo "== driver bench $(date +%T)"
timeout -k 10 500 python -u bench.py --mode driver --steps 3 --no-cpu-baseline > $O/driver.json 2> $O/driver.err || { tail -20 $O/driver.err; exit 1; }
cut -c1-250 $O/driver.json
echo "== phaselift bench $(date +%T)"
timeout -k 10 500 python -u bench.py --mode phaselift --steps 1 --warmup 1 --no-cpu-baseline > $O/pl.json 2> $O/pl.err || { tail -20 $O/pl.err; exit 1; }
cut -c1-250 $O/pl.json
echo "== phaselift trace $(date +%T)"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pl -o run --output-format csv -- python3 bench.py --mode phaselift --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pltrace.log 2>&1 || { tail -20 $O/pltrace.log; exit 1; }
echo "== driver trace $(date +%T)"; ACE_DRIVER_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/driver -o run --output-format csv -- python3 tools/dbg/driver_once.py > $O/driverprof.log 2>&1 || { tail -20 $O/driverprof.log; exit 1; }
grep "^call" $O/driverprof.log
echo "== done $(date +%T)"
