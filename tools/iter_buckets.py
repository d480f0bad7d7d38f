"""Where one unit solve's time goes, by iteration index: from a rocprofv3 kernel trace of
`bench.py --steps 1 --warmup 0` (one 200-iteration solve per sub-batch stream), the wall time
between consecutive gyf/gyk launches on each sub-batch stream, summed per iteration bucket.
Diagnostic only.  usage: iter_buckets.py run_kernel_trace.csv"""
import collections
import csv
import sys

ITER = ("gyf_kernel", "gyk_kernel", "nms_kernel")
rows = list(csv.DictReader(open(sys.argv[1])))
byst = collections.defaultdict(list)
allk = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    allk.append((s, e, r["Kernel_Name"][:60], r["Stream_Id"]))
    if any(k in r["Kernel_Name"] for k in ITER):
        byst[r["Stream_Id"]].append((s, e))
allk.sort()
t0 = allk[0][0]
print(f"trace span {(allk[-1][1] - t0) / 1e6:.3f} ms, {len(allk)} kernels")
edges = [0, 1, 6, 11, 21, 31, 41, 51, 61, 81, 121, 161, 201]
for st, ev in sorted(byst.items()):
    ev.sort()
    nsolve = len(ev) // 200
    print(f"stream {st}: {len(ev)} iteration launches ({nsolve} solves)")
    for sv in range(nsolve):
        e = ev[200 * sv:200 * (sv + 1)]
        starts = [s for s, _ in e] + [e[-1][1]]
        per = [(starts[i + 1] - starts[i]) / 1e3 for i in range(200)]
        durs = [(x1 - x0) / 1e3 for x0, x1 in e]
        print(f"  solve {sv}: first launch at {(e[0][0] - t0) / 1e6:.3f} ms, last end {(e[-1][1] - t0) / 1e6:.3f} ms")
        for a, b in zip(edges[:-1], edges[1:]):
            lo, hi = a, min(b, 200)
            if lo >= hi:
                continue
            p = per[lo:hi]
            d = durs[lo:hi]
            print(f"    it {lo:3d}-{hi - 1:3d}: wall {sum(p) / 1e3:7.3f} ms  period avg {sum(p) / len(p):7.1f} us"
                  f"  iter-kernel avg {sum(d) / len(d):7.1f} us")
# the setup / init kernels before the first iteration launch
first = min(ev[0][0] for ev in byst.values())
pre = collections.Counter()
for s, e, k, _ in allk:
    if s < first:
        pre[k] += e - s
print("before the first iteration launch (device time, ms):")
for k, v in pre.most_common(8):
    print(f"  {v / 1e6:7.3f}  {k}")
