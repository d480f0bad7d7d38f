# A/B of the unit bench between the tree's libace.so and an alternative build (ACE_LIB), with the HBM PMC
# passes of each (FETCH_SIZE, WRITE_SIZE, separate runs):  bash tools/gpu/libab.sh <tag> <alt.so> ["bench args"]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; ALT=$2; ARGS=${3:-"--no-cpu-baseline --no-regime-p --no-refine-input --no-configs --steps 5"}
O=gpurun_out/$TAG; mkdir -p $O
B="--no-cpu-baseline --no-regime-p --no-refine-input --no-configs --no-prof --steps 1 --warmup 1"
for rep in 1 2; do
  for v in base alt; do
    L=2ace-mmwave-channel-estimation_amd/ace_amd/libace.so; [ $v = alt ] && L=$ALT
    ACE_LIB=$L timeout -k 10 300 python3 -u bench.py $ARGS > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -20 $O/${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${v}_$rep.json'));print('$v', d['value'], d['ms_per_step'], d['kernels_ms'])"
  done
done
for v in base alt; do
  L=2ace-mmwave-channel-estimation_amd/ace_amd/libace.so; [ $v = alt ] && L=$ALT
  for c in FETCH_SIZE WRITE_SIZE; do
    ACE_LIB=$L timeout -k 10 -s KILL 300 rocprofv3 --pmc $c -d $O/${v}_$c -o run --output-format csv -- python3 bench.py $B > $O/${v}_$c.log 2>&1 || { tail -20 $O/${v}_$c.log; exit 1; }
  done
  echo "== $v"
  python3 tools/pmc_summary.py $O/${v}_FETCH_SIZE/run_counter_collection.csv $O/${v}_WRITE_SIZE/run_counter_collection.csv $O/${v}_pmc.json 4096 unit | head -8
  rm -rf $O/${v}_FETCH_SIZE $O/${v}_WRITE_SIZE
done
