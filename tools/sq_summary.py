"""Summarise rocprofv3 SQ counter passes per kernel (values normalised by SQ_WAVE_CYCLES)."""
import collections, csv, sys

def main(*paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].replace("void ", "").replace("ace::(anonymous namespace)::", "")
            k = k.split("(int")[0].split("(ace::")[0][:40]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in sorted(agg.items()):
        if not any(s in k for s in ("zgemm", "zstep", "pre_", "ystep", "gemv", "inv_ipk", "gyk", "i8ah", "i8a_", "hetrd", "trieig", "backxf", "wy_")):
            continue
        wc = d.get("SQ_WAVE_CYCLES", 0) or 1
        print(f"{k:40s} wave_cycles={wc:.3e}")
        print("    " + "  ".join(f"{c[3:]}={v / wc:.3f}" for c, v in sorted(d.items()) if c != "SQ_WAVE_CYCLES"))

if __name__ == "__main__":
    main(*sys.argv[1:])
