set -o pipefail
O=gpurun_out/r3n; mkdir -p $O
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_config5.py tests/test_gpu_pipeline.py tests/test_gpu_private.py -k "nuclear or config5 or Nuclear" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
B="--no-cpu-baseline --no-regime-p --no-refine-input"
echo "== nuclear bench $(date +%T)"
timeout -k 10 500 python -u bench.py --variant A2nuclear --steps 5 $B > $O/nuclear.json 2> $O/nuclear.err || { tail -20 $O/nuclear.err; exit 1; }
cut -c1-250 $O/nuclear.json
echo "== config5 bench $(date +%T)"
timeout -k 10 500 python -u bench.py --mode config5 --steps 3 $B > $O/config5.json 2> $O/config5.err || { tail -20 $O/config5.err; exit 1; }
cut -c1-250 $O/config5.json
echo "== done $(date +%T)"
