# regime P setup: recursive Schur-complement inverse (default) vs Gauss-Jordan (ACE_PC_GJ=1)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-q3}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_private.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --private --no-cpu-baseline > $O/bench_p.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_p.json'));print('P', d['value'], d['kernels_ms'])"
ACE_PC_GJ=1 timeout -k 10 300 python bench.py --private --no-cpu-baseline > $O/bench_pgj.json 2>> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_pgj.json'));print('P GJ', d['value'], d['kernels_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --private --steps 2 --warmup 1 --no-cpu-baseline --no-prof > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
