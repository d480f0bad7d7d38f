"""Steady-state view of a rocprofv3 kernel trace of the unit bench: per-class median durations
and one iteration's launch timeline.  Diagnostic only.  usage: timeline.py run_kernel_trace.csv"""
import csv
import statistics as S
import sys

KEYS = {"zstep1w_kernel<false>": "Z", "gyf_kernel": "Y", "zstep1w_compact_kernel": "C", "gyk_kernel": "G", "i8a_kernel": "A", "i8ah_kernel<false, false>": "H", "i8ah_kernel<false, true>": "F", "zlean_kernel": "L", "dual_fix_kernel": "D"}
ev = []
for r in csv.DictReader(open(sys.argv[1])):
    for k, c in KEYS.items():
        if k in r["Kernel_Name"]:
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), c, r["Stream_Id"]))
ev.sort()
for c in "AGHFYZCLD":
    d = sorted(e - s for s, e, k, _ in ev if k == c)
    if d:
        print(f"{c} n={len(d)} median {S.median(d) / 1e3:.1f} us  p10 {d[len(d) // 10] / 1e3:.1f}  p90 {d[9 * len(d) // 10] / 1e3:.1f}")
s0 = sorted({st for _, _, _, st in ev})[0]
A0 = [s for s, e, k, st in ev if k in "GY" and st == s0]
it = [(A0[i + 1] - A0[i]) / 1e3 for i in range(len(A0) - 1)]
print("iteration period (us), stream", s0, ": median", round(S.median(it), 1))
i = min(len(A0) - 3, 300)
for s, e, k, st in ev:
    if A0[i] - 1000 <= s <= A0[i + 1]:
        print(f"{(s - A0[i]) / 1e3:8.1f} {(e - A0[i]) / 1e3:8.1f} {(e - s) / 1e3:6.1f} {k} stream {st}")
