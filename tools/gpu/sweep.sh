#!/bin/bash
# Knob sweep of the unit bench: bash tools/gpu/sweep.sh <tag> "<ENV=V ...>" "<ENV=V ...>" ...
# Each argument is one environment setting ("-" = defaults); prints the rec/s of each run.
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
B="--steps 10 --warmup 3 --no-cpu-baseline --no-regime-p --no-refine-input --no-configs"
i=0
for s in "$@"; do
  i=$((i+1))
  e=""; [ "$s" != "-" ] && e="$s"
  timeout -k 10 300 env $e ACE_MSR_TRACE=1 python -u bench.py $B > $O/$i.json 2> $O/$i.err || { echo "run $i ($s) failed"; tail -20 $O/$i.err; exit 1; }
  v=$(python3 -c "import json,sys; d=json.loads(open('$O/$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")
  echo "$i [$s] $v $(grep -c 'msr check' $O/$i.err) checks; first run: $(grep -m1 'msr h 0' $O/$i.err)"
done
