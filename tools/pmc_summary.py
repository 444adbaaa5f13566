"""Average per-dispatch PMC values of kernels matching a name filter (tools/prof_conv_pmc.sh)."""
import collections
import csv
import glob
import sys

flt = sys.argv[2] if len(sys.argv) > 2 else "conv_x3"
for d in sorted(glob.glob(sys.argv[1] + "/p*/")):
    rows = list(csv.DictReader(open(d + "run_counter_collection.csv")))
    agg = collections.defaultdict(list)
    for r in rows:
        if flt in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(d.split("/")[-2], {k: round(sum(v) / len(v) / 1e6, 3) for k, v in agg.items()})
