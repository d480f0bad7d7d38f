set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/h2k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_horizon.py -x -v -s --timeout 500 --timeout-method thread > $O/t1.log 2>&1; rc=$?
grep -E "PASS|FAIL|held|Error|assert" $O/t1.log | head -20
[ $rc -eq 0 ] || { tail -30 $O/t1.log; exit 1; }
ACE_LIB=ablib/libace_h2s.so timeout -k 10 300 python bench.py --mode phaselift --batch 512 --iters 200 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
python3 - <<'PY'
L = open('gpurun_out/h2k/stamps.log').read().splitlines()
for key in ('trieig', 'he2hb', 'hb2st'):
    rows = [l for l in L if l.startswith(key)]
    print(key, len(rows))
    for l in rows[:3] + rows[len(rows)//2:len(rows)//2+3] + rows[-3:]:
        print('  ', l)
PY
