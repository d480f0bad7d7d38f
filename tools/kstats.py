"""Print the top kernels of a rocprofv3 kernel_stats.csv: name, calls, average ms, share."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 10]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e6:9.3f} ms {float(r['Percentage']):6.2f} %")
