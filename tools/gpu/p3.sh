set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-p3}; mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_gpu_private.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --private --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('value', d['value'], d['kernels_ms'], d['roofline']['frac'])"
ACE_LIB=tools/libace_stamps_pc.so timeout -k 10 120 python tools/stamp_pgk.py > $O/stamps.log 2>&1 || { tail $O/stamps.log; exit 1; }
grep pgk $O/stamps.log | head -14
