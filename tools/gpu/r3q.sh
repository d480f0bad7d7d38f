set -o pipefail
O=gpurun_out/r3q; mkdir -p $O
export TMPDIR=/tmp
echo "== full gpu tests $(date +%T)"
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo "== smoke $(date +%T)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
run() { local tag=$1; shift; echo "== $tag $(date +%T)"; timeout -k 10 600 python -u bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }; cut -c1-200 $O/$tag.json; }
run unit
run nuclear --variant A2nuclear --steps 5
run config5 --mode config5 --steps 3
run driver --mode driver --steps 3
echo "== done $(date +%T)"
