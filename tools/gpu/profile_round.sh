# Round profiles: kernel statistics and HBM PMC passes per workload (run before the bench lines,
# whose `traffic` fields read the PMC summaries from profiles/).  Usage on the GPU box:
#   bash tools/gpu/profile_round.sh <out-tag>
# then: python3 tools/pmc_summary.py <fetch csv> <write csv> profiles/r<R>_v<V>[_<tag>]_pmc_hbm.json
set -o pipefail
O=gpurun_out/${1:-prof}; mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --no-regime-p --no-refine-input --no-configs --no-prof"
st() { local tag=$1; shift; echo "== stats $tag $(date +%T)"; timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- python3 bench.py $B "$@" > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }; }
pmc() { local tag=$1 cnt=$2; shift 2; echo "== pmc $tag $cnt $(date +%T)"; timeout -k 10 -s KILL 300 rocprofv3 --pmc $cnt -d $O/${tag}_$cnt -o run --output-format csv -- python3 bench.py $B "$@" > $O/${tag}_$cnt.log 2>&1 || { tail -20 $O/${tag}_$cnt.log; exit 1; }; }
st unit --steps 1 --warmup 1
st nuclear --variant A2nuclear --steps 1 --warmup 1
st config5 --mode config5 --steps 1 --warmup 1
st pipeline --mode pipeline --steps 1 --warmup 0
st phaselift --mode phaselift --steps 1 --warmup 0
pmc unit FETCH_SIZE --steps 1 --warmup 0
pmc unit WRITE_SIZE --steps 1 --warmup 0
pmc pipeline FETCH_SIZE --mode pipeline --steps 1 --warmup 0 --batch 1024
pmc pipeline WRITE_SIZE --mode pipeline --steps 1 --warmup 0 --batch 1024
pmc phaselift FETCH_SIZE --mode phaselift --steps 1 --warmup 0 --iters 20
pmc phaselift WRITE_SIZE --mode phaselift --steps 1 --warmup 0 --iters 20
echo "== done $(date +%T)"
