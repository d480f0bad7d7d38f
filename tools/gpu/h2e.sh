set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/h2e; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/pl -o run --output-format csv -- python3 bench.py --mode phaselift --batch 512 --iters 200 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pl.log 2>&1 || { tail -20 $O/pl.log; exit 1; }
cp $O/pl/run_kernel_stats.csv $O/pl_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/h2e/pl/run_kernel_trace.csv')))
import collections
by = collections.defaultdict(list)
for r in rows:
    by[r['Kernel_Name'][:40]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:8]:
    print(f"{k:40s} n {len(v):5d} total {sum(v):9.1f} ms max {max(v):8.2f} first {v[:3]} last {v[-3:]}")
PY
rm -rf $O/pl
