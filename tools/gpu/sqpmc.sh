# SQ counters of the PhaseLift eigensolver kernels (one --pmc pass, a 4-iteration run)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sq; mkdir -p $O
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d $O/p -o run --output-format csv -- python3 bench.py --mode phaselift --batch 512 --iters 4 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open('gpurun_out/sq/p/run_counter_collection.csv')))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r['Kernel_Name'].replace('ace::(anonymous namespace)::', '').replace('void ', '').split('(')[0][:28]
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, c in agg.items():
    if not any(s in k for s in ('he2hb', 'hb2st', 'bt2q', 'trieig', 'zgemm3m')):
        continue
    wc = c['SQ_WAVE_CYCLES'] or 1
    print(f"{k:28s} valu/wave-cyc {c['SQ_ACTIVE_INST_VALU']/wc:.3f} lds-wait {c['SQ_WAIT_INST_LDS']/wc:.3f} any-wait {c['SQ_WAIT_ANY']/wc:.3f} "
          f"valu-insts/wave {c['SQ_INSTS_VALU']/max(c['SQ_WAVES'],1):.0f} lds-insts/wave {c['SQ_INSTS_LDS']/max(c['SQ_WAVES'],1):.0f} busy {c['SQ_BUSY_CYCLES']:.3g}")
PY
