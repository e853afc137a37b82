"""Average rocprofv3 --pmc counter values per kernel (one row per counter) from every
*_counter_collection.csv under a directory. Usage: pmc_summary.py DIR [kernel-substring]"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
vals = collections.defaultdict(list)
for f in glob.glob(f"{root}/**/*_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if pat and pat not in k:
            continue
        vals[(k[:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(vals.items()):
    print(f"{k:60s} {c:28s} n={len(v):3d} mean={sum(v) / len(v):.4g}")
