# Unit-mode profiles of the current build: rocprofv3 kernel statistics and the two HBM PMC passes
# (FETCH_SIZE, WRITE_SIZE), one solve each.  Usage on the GPU box: bash tools/gpu/profile_unit.sh <tag> <rNN_vNN>
set -o pipefail
O=gpurun_out/${1:-punit}; mkdir -p $O
R=${2:-r03_v13}
export TMPDIR=/tmp
B="--no-cpu-baseline --no-regime-p --no-refine-input --no-configs --no-prof"
echo "== stats $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 bench.py $B --steps 1 --warmup 1 > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $c $(date +%T)"
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $c -d $O/$c -o run --output-format csv -- python3 bench.py $B --steps 1 --warmup 0 > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
done
python3 tools/pmc_summary.py $O/FETCH_SIZE/run_counter_collection.csv $O/WRITE_SIZE/run_counter_collection.csv $O/${R}_pmc_hbm.json > $O/${R}_pmc_hbm.txt
cp $O/stats/run_kernel_stats.csv $O/${R}_unit_kernel_stats.csv
python3 tools/iter_buckets.py $O/stats/run_kernel_trace.csv > $O/${R}_unit_buckets.txt || true
head -12 $O/${R}_pmc_hbm.txt
echo "== done $(date +%T)"
