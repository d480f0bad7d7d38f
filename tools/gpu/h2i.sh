set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/h2i; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_heev2.py tests/test_gpu_phaselift.py -x -q --timeout 300 --timeout-method thread > $O/t1.log 2>&1; rc=$?
tail -3 $O/t1.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/t1.log | head -20; exit 1; }
timeout -k 10 300 python bench.py --mode phaselift --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_pl.json 2> $O/bench_pl.err || { tail -20 $O/bench_pl.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_pl.json').read().strip().splitlines()[-1]); print('phaselift', d['value'], d['ms_per_step'], d['kernels_total_ms'])"
ACE_LIB=ablib/libace_h2s.so timeout -k 10 300 python bench.py --mode phaselift --batch 512 --iters 200 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
python3 - <<'PY'
import re
L = open('gpurun_out/h2i/stamps.log').read().splitlines()
for key in ('trieig', 'he2hb', 'hb2st'):
    rows = [l for l in L if l.startswith(key)]
    print(key, len(rows))
    for l in rows[:3] + rows[len(rows)//2:len(rows)//2+3] + rows[-3:]:
        print('  ', l)
PY
