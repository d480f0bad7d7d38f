# A/B of bench lines under environment settings, alternating, one process each:
#   bash tools/gpu/envab.sh <tag> "<bench args>" "ENV=A ..." "ENV=B ..." ...   ("-" = no extra env)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; ARGS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    [ "$e" = "-" ] && e=""
    env $e timeout -k 10 300 python3 -u bench.py $ARGS > $O/${i}_$rep.json 2> $O/${i}_$rep.err || { tail -20 $O/${i}_$rep.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open('$O/${i}_$rep.json'));print('$rep', repr('$e'), d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))"
  done
done
