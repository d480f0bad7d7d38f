# PhaseLift (config 4) profiles for the round: kernel statistics of the full 200-iteration bench step and
# HBM PMC passes (FETCH_SIZE, WRITE_SIZE) at 20 iterations.  Usage: bash tools/gpu/prof_pl.sh <R_V tag>
set -o pipefail
export TMPDIR=/tmp
R=${1:-r06_v1}
O=gpurun_out/prof_$R; mkdir -p $O
B="--no-cpu-baseline --no-prof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/st -o run --output-format csv -- python3 bench.py --mode phaselift --steps 1 --warmup 0 $B > $O/st.log 2>&1 || { tail -20 $O/st.log; exit 1; }
cp $O/st/run_kernel_stats.csv $O/${R}_phaselift_kernel_stats.csv
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $c -d $O/$c -o run --output-format csv -- python3 bench.py --mode phaselift --steps 1 --warmup 0 --iters 20 $B > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
done
python3 tools/pmc_summary.py $O/FETCH_SIZE/run_counter_collection.csv $O/WRITE_SIZE/run_counter_collection.csv $O/${R}_phaselift_pmc_hbm.json 512 phaselift > $O/${R}_phaselift_pmc_hbm.txt
head -12 $O/${R}_phaselift_pmc_hbm.txt
python3 tools/kstats.py $O/${R}_phaselift_kernel_stats.csv 10
rm -rf $O/st $O/FETCH_SIZE $O/WRITE_SIZE
