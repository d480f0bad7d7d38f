set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/h2n; mkdir -p $O
ACE_LIB=ablib/libace_h2s.so timeout -k 10 300 python bench.py --mode phaselift --batch 512 --iters 200 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
python3 - <<'PY'
import collections
L = open('gpurun_out/h2n/stamps.log').read().splitlines()
rows = [l for l in L if l.startswith('trieig-slow')]
print('slow WGs', len(rows))
mc = collections.Counter(int(l.split('maxcl ')[1].split(' ')[0]) for l in rows)
print('maxcl histogram', sorted(mc.items()))
for l in rows[:8] + rows[-8:]:
    print('  ', l)
PY
rm -f $O/stamps.log
