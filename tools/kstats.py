"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel totals and, for kernels called
once per level, the per-call-index average (``--cycle K`` groups calls modulo K)."""
import argparse
import collections
import csv
import glob

ap = argparse.ArgumentParser()
ap.add_argument("path", help="directory holding *_kernel_trace.csv (searched recursively)")
ap.add_argument("--top", type=int, default=14)
ap.add_argument("--cycle", nargs="*", default=[], help="name=K pairs")
a = ap.parse_args()
import os
f = max(glob.glob(f"{a.path}/**/*_kernel_trace.csv", recursive=True), key=os.path.getmtime)
rows = list(csv.DictReader(open(f)))
seq = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]
tot = collections.defaultdict(float)
cnt = collections.Counter()
for k, t in seq:
    tot[k] += t
    cnt[k] += 1
all_us = sum(tot.values())
for k in sorted(tot, key=tot.get, reverse=True)[:a.top]:
    print(f"{k[:64]:64s} {cnt[k]:6d} {tot[k] / 1e3:9.2f} ms {tot[k] / cnt[k]:8.1f} us "
          f"{100 * tot[k] / all_us:5.1f}%")
print(f"total {all_us / 1e3:.2f} ms")
for spec in a.cycle:
    name, K = spec.split("=")
    xs = [t for k, t in seq if name in k]
    by = collections.defaultdict(list)
    for i, t in enumerate(xs):
        by[i % int(K)].append(t)
    print(name, " ".join(f"{i}:{sum(v) / len(v):.1f}" for i, v in sorted(by.items())))
