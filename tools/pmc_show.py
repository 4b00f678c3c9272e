"""Per-dispatch averages of PMC counters for the kernels named on the command line."""
import collections
import csv
import glob
import sys

d, names = sys.argv[1], sys.argv[2:] or ["rx_decode"]
for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if not any(n in k for n in names):
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add(r["Dispatch_Id"])
    for k, v in agg.items():
        n = len(cnt[k])
        print(f.split("/")[-2], k, n, " ".join(f"{c}={x / n:.3e}" for c, x in sorted(v.items())))
