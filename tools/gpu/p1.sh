set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/p1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_private.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -30 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --private --batch 4096 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
