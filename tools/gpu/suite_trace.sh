# The full GPU suite, a PhaseLift kernel trace and a short unit bench (r06).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/suite_trace; mkdir -p $O
timeout -k 10 1500 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests > $O/t1.log 2>&1; rc=$?
tail -3 $O/t1.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/t1.log | head -20; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/pl -o run --output-format csv -- python3 bench.py --mode phaselift --batch 512 --iters 200 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pl.log 2>&1 || { tail -20 $O/pl.log; exit 1; }
grep -h '"metric"' $O/pl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('phaselift', d['value'], d['ms_per_step'])"
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open('gpurun_out/suite_trace/pl/run_kernel_trace.csv')))
by = collections.defaultdict(list)
for r in rows:
    by[r['Kernel_Name'][:40]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:7]:
    print(f"{k:40s} n {len(v):5d} total {sum(v):9.1f} ms max {max(v):8.2f} first {[round(x,3) for x in v[:3]]}")
PY
rm -rf $O/pl
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs > $O/unit.json 2> $O/unit.err || { tail -20 $O/unit.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/unit.json').read().strip().splitlines()[-1]); print('unit', d['value'], d['ms_per_step'])"
