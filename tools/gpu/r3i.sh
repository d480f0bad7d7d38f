set -o pipefail
O=gpurun_out/r3i; mkdir -p $O
export TMPDIR=/tmp
run() { local tag=$1; shift; echo "== $tag $(date +%T)"; timeout -k 10 500 python -u bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }; cut -c1-600 $O/$tag.json; }
run unit --steps 3
run config5 --mode config5 --steps 2
run driver --mode driver --steps 5
run nuclear --variant A2nuclear --steps 3
run pipeline --mode pipeline --steps 1
run phaselift --mode phaselift --steps 1
echo "== done $(date +%T)"
