set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/h2h; mkdir -p $O
for side in 0 1; do
ACE_PROX_SIDE=$side timeout -k 10 300 rocprofv3 --kernel-trace -d $O/pl$side -o run --output-format csv -- python3 bench.py --mode phaselift --batch 512 --iters 200 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pl$side.log 2>&1 || { tail -20 $O/pl$side.log; exit 1; }
python3 - $side <<'PY'
import csv, sys, collections
side = sys.argv[1]
rows = list(csv.DictReader(open(f'gpurun_out/h2h/pl{side}/run_kernel_trace.csv')))
by = collections.defaultdict(list)
for r in rows:
    by[r['Kernel_Name'][:30]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
for k in ('ace::(anonymous namespace)::tri', 'ace::(anonymous namespace)::bt2', 'ace::(anonymous namespace)::he2'):
    for kk, v in by.items():
        if kk.startswith(k):
            q = [round(x, 2) for x in v[::24]]
            print(f"side {side} {kk:30s} n {len(v)} total {sum(v):8.1f} ms samples {q}")
PY
rm -rf $O/pl$side
done
