# GPU suite + unit bench (shared) + private bench, with zfast
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-p7}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('S value', d['value'], d['kernels_ms'], d['roofline']['frac'])"
timeout -k 10 200 python bench.py --private --no-cpu-baseline > $O/bench_p.json 2> $O/bench_p.err || { tail $O/bench_p.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_p.json'));print('P value', d['value'], d['kernels_ms'], d['roofline']['frac'])"
ACE_ZFAST=0 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_nozf.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_nozf.json'));print('S nozfast value', d['value'], d['kernels_ms'])"
