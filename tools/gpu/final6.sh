# Round-6 validation on one box: full GPU suite, smoke, then the default bench line (the driver's command).
set -o pipefail
export TMPDIR=/tmp
T=${1:-r06_v2}
O=gpurun_out/$T; mkdir -p $O
echo "== full gpu tests $(date +%T)"
timeout -k 10 1500 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests > $O/${T}_gputest.log 2>&1 || { tail -40 $O/${T}_gputest.log; exit 1; }
tail -2 $O/${T}_gputest.log
echo "== smoke $(date +%T)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { tail -20 $O/${T}_smoke.log; exit 1; }
tail -2 $O/${T}_smoke.log
echo "== bench $(date +%T)"
timeout -k 10 900 python -u bench.py > $O/${T}_bench_default.json 2> $O/${T}_bench_default.err || { tail -20 $O/${T}_bench_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${T}_bench_default.json').read().strip().splitlines()[-1]); print(d['metric'], d['value']); [print(k, v.get('value') if isinstance(v, dict) else v) for k, v in d.items() if k.startswith('config') or k == 'pipeline']"
echo "== done $(date +%T)"
