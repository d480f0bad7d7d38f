"""Where one unit solve's time goes, by iteration index: from a rocprofv3 kernel trace of
`bench.py --steps K` (200-iteration solves, one per sub-batch stream and step), the wall time
between consecutive iteration launches on each sub-batch stream, summed per iteration bucket.
An iteration launch is gyf / gyk / nms_kernel (one iteration) or an m-space run (msr_kernel),
which covers the iterations of its solve that no per-iteration launch ran (200 minus their
count; its wall time is spread evenly over them).  A solve starts at its init Z-step launch
(zstep1w_kernel<true> / zstep_kernel<.., true, ..>) on the stream.  Diagnostic only.
usage: iter_buckets.py run_kernel_trace.csv [iters]"""
import collections
import csv
import sys

ITER = ("gyf_kernel", "gyk_kernel", "nms_kernel")
RUN = "msr_kernel"
INIT = ("zstep1w_kernel<true>", "zstep_kernel<0, true", "nms_init")
NIT = int(sys.argv[2]) if len(sys.argv) > 2 else 200
rows = list(csv.DictReader(open(sys.argv[1])))
byst = collections.defaultdict(list)
allk = []
for r in rows:
    s, e, name = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]
    allk.append((s, e, name[:60], r["Stream_Id"]))
    kind = "it" if any(k in name for k in ITER) else "run" if RUN in name else "init" if any(k in name for k in INIT) else None
    if kind:
        byst[r["Stream_Id"]].append((s, e, kind))
allk.sort()
t0 = allk[0][0]
print(f"trace span {(allk[-1][1] - t0) / 1e6:.3f} ms, {len(allk)} kernels")
edges = [0, 1, 6, 11, 21, 31, 41, 51, 61, 81, 121, 161, 201]
tot = collections.defaultdict(float)
nsolves = 0
for st, ev in sorted(byst.items()):
    ev.sort()
    solves, cur = [], None
    for s, e, kind in ev:
        if kind == "init":
            cur = []
            solves.append(cur)
        elif cur is not None:
            cur.append((s, e, kind))
    solves = [sv for sv in solves if sv]
    print(f"stream {st}: {len(solves)} solves")
    for k, sv in enumerate(solves):
        nit = sum(1 for x in sv if x[2] == "it")
        nrun = sum(1 for x in sv if x[2] == "run")
        run_iters = (NIT - nit) / nrun if nrun else 0.0
        starts = [x[0] for x in sv] + [sv[-1][1]]
        per = []   # (iterations covered, wall us) per launch, in order
        for i, x in enumerate(sv):
            n = run_iters if x[2] == "run" else 1.0
            per.append((n, (starts[i + 1] - starts[i]) / 1e3))
        # spread to iteration indices 0 .. NIT-1
        it_wall = []
        for n, w in per:
            it_wall += [w / n] * int(round(n))
        it_wall = (it_wall + [0.0] * NIT)[:NIT]
        nsolves += 1
        print(f"  solve {k}: {nit} iteration launches, {nrun} m-space runs ({run_iters:.0f} iterations each), "
              f"wall {(sv[-1][1] - sv[0][0]) / 1e6:.3f} ms")
        for a, b in zip(edges[:-1], edges[1:]):
            lo, hi = a, min(b, NIT)
            if lo < hi:
                tot[(lo, hi)] += sum(it_wall[lo:hi])
print(f"mean over {nsolves} solve-streams (iteration index 0 = iteration 1):")
for (lo, hi), v in sorted(tot.items()):
    w = v / max(1, nsolves)
    print(f"    it {lo + 1:3d}-{hi:3d}: wall {w / 1e3:7.3f} ms  period avg {w / (hi - lo):7.1f} us")
# the setup / init kernels before the first iteration launch
first = min(x[0] for ev in byst.values() for x in ev if x[2] != "init")
pre = collections.Counter()
for s, e, k, _ in allk:
    if s < first:
        pre[k] += e - s
print("before the first iteration launch (device time, ms):")
for k, v in pre.most_common(8):
    print(f"  {v / 1e6:7.3f}  {k}")
