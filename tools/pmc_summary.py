"""Summarise tools/pmc_passes.sh output: per kernel, mean of each counter over dispatches."""
import collections
import csv
import glob
import sys

out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:34]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items()):
    if not k.startswith("pbf"):
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:34s} {sum(v) / len(v):14.4g}")
