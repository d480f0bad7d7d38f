set -o pipefail
O=gpurun_out/r3r; mkdir -p $O
export TMPDIR=/tmp
run() { local tag=$1; shift; echo "== $tag $(date +%T)"; timeout -k 10 600 python -u bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }; cut -c1-200 $O/$tag.json; }
run pipeline --mode pipeline
run phaselift --mode phaselift --steps 1
B="--no-cpu-baseline --no-regime-p --no-refine-input --no-prof"
st() { local tag=$1; shift; echo "== stats $tag $(date +%T)"; timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- python3 bench.py $B "$@" > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }; }
pmc() { local tag=$1 cnt=$2; shift 2; echo "== pmc $tag $cnt $(date +%T)"; timeout -k 10 -s KILL 300 rocprofv3 --pmc $cnt -d $O/${tag}_$cnt -o run --output-format csv -- python3 bench.py $B "$@" > $O/${tag}_$cnt.log 2>&1 || { tail -20 $O/${tag}_$cnt.log; exit 1; }; }
st unit --steps 1 --warmup 1
st pipeline --mode pipeline --steps 1 --warmup 0
st phaselift --mode phaselift --steps 1 --warmup 0
pmc unit FETCH_SIZE --steps 1 --warmup 0
pmc unit WRITE_SIZE --steps 1 --warmup 0
echo "== done $(date +%T)"
