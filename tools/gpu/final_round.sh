# Round-end measurement: full GPU suite, smoke, pipeline PMC at the bench batch, then every bench line.
set -o pipefail
O=gpurun_out/${1:-final}; mkdir -p $O
export TMPDIR=/tmp
R=${2:-r03_v10}
echo "== full gpu tests $(date +%T)"
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo "== smoke $(date +%T)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
B="--no-cpu-baseline --no-regime-p --no-refine-input --no-configs --no-prof"
pmc() { local tag=$1 cnt=$2; shift 2; echo "== pmc $tag $cnt $(date +%T)"; timeout -k 10 -s KILL 300 rocprofv3 --pmc $cnt -d $O/${tag}_$cnt -o run --output-format csv -- python3 bench.py $B "$@" > $O/${tag}_$cnt.log 2>&1 || { tail -20 $O/${tag}_$cnt.log; exit 1; }; }
pmc pipeline FETCH_SIZE --mode pipeline --steps 1 --warmup 0
pmc pipeline WRITE_SIZE --mode pipeline --steps 1 --warmup 0
python3 tools/pmc_summary.py $O/pipeline_FETCH_SIZE/run_counter_collection.csv $O/pipeline_WRITE_SIZE/run_counter_collection.csv profiles/${R}_pipeline_pmc_hbm.json > $O/pipeline_pmc.txt && cp profiles/${R}_pipeline_pmc_hbm.json $O/
run() { local tag=$1; shift; echo "== $tag $(date +%T)"; timeout -k 10 600 python -u bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }; cut -c1-200 $O/$tag.json; }
run unit
run nuclear --variant A2nuclear --steps 5
run config5 --mode config5 --steps 3
run driver --mode driver --steps 3
run pipeline --mode pipeline
run phaselift --mode phaselift --steps 1
echo "== done $(date +%T)"
