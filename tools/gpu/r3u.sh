set -o pipefail
O=gpurun_out/r3u; mkdir -p $O
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pipeline.py tests/test_gpu_driver.py tests/test_gpu_spectral.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo "== driver bench $(date +%T)"
timeout -k 10 500 python -u bench.py --mode driver --steps 3 --no-cpu-baseline > $O/driver.json 2> $O/driver.err || { tail -20 $O/driver.err; exit 1; }
cut -c1-300 $O/driver.json
echo "== pipeline bench $(date +%T)"
timeout -k 10 500 python -u bench.py --mode pipeline --steps 1 --no-cpu-baseline > $O/pipe.json 2> $O/pipe.err || { tail -20 $O/pipe.err; exit 1; }
cut -c1-250 $O/pipe.json
echo "== driver trace $(date +%T)"; ACE_DRIVER_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/driver -o run --output-format csv -- python3 tools/dbg/driver_once.py > $O/driver.log 2>&1 || { tail -20 $O/driver.log; exit 1; }
grep "^call" $O/driver.log
echo "== done $(date +%T)"
