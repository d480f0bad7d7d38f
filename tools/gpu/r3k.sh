set -o pipefail
O=gpurun_out/r3k; mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --no-prof --no-regime-p --no-refine-input"
run() { local tag=$1; shift; echo "== $tag $(date +%T)"; timeout -k 10 500 python -u bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }; cut -c1-300 $O/$tag.json; }
st() { local tag=$1; shift; echo "== stats $tag $(date +%T)"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- $B "$@" > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }; }
pmc() { local tag=$1 cnt=$2; shift 2; echo "== pmc $tag $cnt $(date +%T)"; timeout -k 10 -s KILL 300 rocprofv3 --pmc $cnt -d $O/${tag}_$cnt -o run --output-format csv -- $B "$@" > $O/${tag}_$cnt.log 2>&1 || { tail -20 $O/${tag}_$cnt.log; exit 1; }; }
run nuclear --variant A2nuclear --steps 3
run config5 --mode config5 --steps 2
st nuclear --variant A2nuclear --steps 1 --warmup 1
st config5 --mode config5 --steps 1 --warmup 1
pmc nuclear FETCH_SIZE --variant A2nuclear --steps 1 --warmup 0
pmc nuclear WRITE_SIZE --variant A2nuclear --steps 1 --warmup 0
pmc config5 FETCH_SIZE --mode config5 --global-batch 16384 --steps 1 --warmup 0
pmc config5 WRITE_SIZE --mode config5 --global-batch 16384 --steps 1 --warmup 0
echo "== driver trace $(date +%T)"; ACE_DRIVER_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/driver -o run --output-format csv -- python3 tools/dbg/driver_once.py > $O/driver.log 2>&1 || { tail -20 $O/driver.log; exit 1; }
grep "^call" $O/driver.log
echo "== done $(date +%T)"
