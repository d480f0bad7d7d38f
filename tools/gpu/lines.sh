# Every bench line of the round on one box (after the PMC summaries of tools/gpu/prof.sh are in profiles/):
#   bash tools/gpu/lines.sh <out-dir> <lines...>   lines: unit nuclear config5 pipeline phaselift driver refine private
set -o pipefail
O=gpurun_out/${1:-lines}; shift
mkdir -p $O
export TMPDIR=/tmp
for l in "$@"; do
  case $l in
    unit) a="";;
    nuclear) a="--variant A2nuclear --steps 5";;
    config5) a="--mode config5 --steps 3";;
    pipeline) a="--mode pipeline";;
    phaselift) a="--mode phaselift --steps 1";;
    driver) a="--mode driver --steps 3";;
    refine) a="--mode refine --steps 3";;
    private) a="--private --steps 3";;
    beamformer) a="--mode beamformer --steps 3";;
    *) echo "unknown line $l"; exit 2;;
  esac
  echo "== $l $(date +%T)"
  timeout -k 10 900 python3 -u bench.py $a > $O/$l.json 2> $O/$l.err || { tail -20 $O/$l.err; exit 1; }
  cut -c1-300 $O/$l.json
done
echo "== done $(date +%T)"
