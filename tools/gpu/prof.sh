# Round profiles: rocprofv3 kernel statistics and the HBM PMC passes (FETCH_SIZE, WRITE_SIZE, separate
# runs) per bench workload; the PMC summaries record the profiled batch (_meta) so that bench.py can
# rescale them to its own line.  Usage on the GPU box: bash tools/gpu/prof.sh <out-dir> <rNN_vNN> <modes...>
# modes: unit nuclear config5 pipeline phaselift refine private
set -o pipefail
O=gpurun_out/${1:-prof}; R=${2:-r05_v1}; shift 2
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --no-regime-p --no-refine-input --no-configs --no-prof"
args() {
  case $1 in
    unit) echo "--steps 1 --warmup 1";;
    nuclear) echo "--variant A2nuclear --steps 1 --warmup 1";;
    config5) echo "--mode config5 --global-batch 16384 --steps 1 --warmup 1";;
    pipeline) echo "--mode pipeline --batch 1024 --steps 1 --warmup 0";;
    phaselift) echo "--mode phaselift --iters 20 --steps 1 --warmup 0";;
    refine) echo "--mode refine --steps 1 --warmup 1 --no-default-profile";;
    private) echo "--private --steps 1 --warmup 1";;
  esac
}
batch() { case $1 in config5) echo 16384;; pipeline) echo 1024;; phaselift) echo 512;; *) echo 4096;; esac; }
for md in "$@"; do
  a=$(args $md)
  echo "== stats $md $(date +%T)"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${md}_st -o run --output-format csv -- python3 bench.py $B $a > $O/${md}_st.log 2>&1 || { tail -20 $O/${md}_st.log; exit 1; }
  cp $O/${md}_st/run_kernel_stats.csv $O/${R}_${md}_kernel_stats.csv
  python3 tools/iter_buckets.py $O/${md}_st/run_kernel_trace.csv > $O/${R}_${md}_iter_buckets.txt 2>/dev/null || true
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== pmc $md $c $(date +%T)"
    timeout -k 10 -s KILL 400 rocprofv3 --pmc $c -d $O/${md}_$c -o run --output-format csv -- python3 bench.py $B $a > $O/${md}_$c.log 2>&1 || { tail -20 $O/${md}_$c.log; exit 1; }
  done
  tg=$md; [ $md = unit ] && tg=""
  python3 tools/pmc_summary.py $O/${md}_FETCH_SIZE/run_counter_collection.csv $O/${md}_WRITE_SIZE/run_counter_collection.csv $O/${R}${tg:+_$tg}_pmc_hbm.json $(batch $md) $md > $O/${R}${tg:+_$tg}_pmc_hbm.txt
  rm -rf $O/${md}_st $O/${md}_FETCH_SIZE $O/${md}_WRITE_SIZE
done
echo "== done $(date +%T)"
