set -o pipefail
O=gpurun_out/r3p; mkdir -p $O
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_config5.py tests/test_gpu_pipeline.py tests/test_gpu_private.py tests/test_gpu_driver.py -k "nuclear or config5" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
B="--no-cpu-baseline --no-regime-p --no-refine-input"
echo "== nuclear bench $(date +%T)"
timeout -k 10 500 python -u bench.py --variant A2nuclear --steps 5 $B > $O/nuclear.json 2> $O/nuclear.err || { tail -20 $O/nuclear.err; exit 1; }
cut -c1-250 $O/nuclear.json
echo "== config5 bench $(date +%T)"
timeout -k 10 500 python -u bench.py --mode config5 --steps 3 $B > $O/config5.json 2> $O/config5.err || { tail -20 $O/config5.err; exit 1; }
cut -c1-250 $O/config5.json
st() { local tag=$1; shift; echo "== stats $tag $(date +%T)"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- python3 bench.py $B --no-prof "$@" > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }; }
pmc() { local tag=$1 cnt=$2; shift 2; echo "== pmc $tag $cnt $(date +%T)"; timeout -k 10 -s KILL 300 rocprofv3 --pmc $cnt -d $O/${tag}_$cnt -o run --output-format csv -- python3 bench.py $B --no-prof "$@" > $O/${tag}_$cnt.log 2>&1 || { tail -20 $O/${tag}_$cnt.log; exit 1; }; }
st nuclear --variant A2nuclear --steps 1 --warmup 1
st config5 --mode config5 --steps 1 --warmup 1
pmc nuclear FETCH_SIZE --variant A2nuclear --steps 1 --warmup 0
pmc nuclear WRITE_SIZE --variant A2nuclear --steps 1 --warmup 0
pmc config5 FETCH_SIZE --mode config5 --global-batch 16384 --steps 1 --warmup 0
pmc config5 WRITE_SIZE --mode config5 --global-batch 16384 --steps 1 --warmup 0
echo "== done $(date +%T)"
