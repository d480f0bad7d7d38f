set -o pipefail
O=gpurun_out/r3t; mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --no-regime-p --no-refine-input"
run() { local tag=$1; shift; echo "== $tag $(date +%T)"; timeout -k 10 300 python -u bench.py $B "$@" > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }; cut -c1-160 $O/$tag.json; }
run base --steps 10
ACE_LIB=tools/libace_nt.so run nt --steps 10
run base2 --steps 10
ACE_LIB=tools/libace_nt.so run nt2 --steps 10
pmc() { local tag=$1 cnt=$2; shift 2; echo "== pmc $tag $cnt $(date +%T)"; timeout -k 10 -s KILL 300 rocprofv3 --pmc $cnt -d $O/${tag}_$cnt -o run --output-format csv -- python3 bench.py $B --no-prof "$@" > $O/${tag}_$cnt.log 2>&1 || { tail -20 $O/${tag}_$cnt.log; exit 1; }; }
pmc base FETCH_SIZE --steps 1 --warmup 0
pmc base WRITE_SIZE --steps 1 --warmup 0
ACE_LIB=tools/libace_nt.so pmc nt FETCH_SIZE --steps 1 --warmup 0
ACE_LIB=tools/libace_nt.so pmc nt WRITE_SIZE --steps 1 --warmup 0
echo "== done $(date +%T)"
