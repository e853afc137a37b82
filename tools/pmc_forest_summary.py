"""Per-kernel PMC summary of tools/pmc_forest.sh (level engine vs per-tree kernel): counters
summed over dispatches; ratios: L2 hit rate, issued-instruction cycles and
instruction-wait cycles per wave cycle, LDS bank-conflict cycles per LDS-active cycle.
FETCH_SIZE is printed raw (rocprofv3's derived unit, summed over dispatches and XCDs).
Usage: pmc_forest_summary.py gpurun_out/pmc_forest"""
import collections
import csv
import glob
import sys

out = sys.argv[1]
lines = []
for eng in ("level", "tree"):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{out}/{eng}_set*/**/*_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            if "lv_" not in k and "forest_grow" not in k:
                continue
            vals[k.split("(")[0][:34]][r["Counter_Name"]] += float(r["Counter_Value"])
    tot = collections.defaultdict(float)
    for c in vals.values():
        for n, v in c.items():
            tot[n] += v
    vals["ALL " + eng] = tot

    def ratio(c, a, b):
        return c.get(a, 0) / c[b] if c.get(b) else float("nan")
    for k, c in sorted(vals.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        hit, miss = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        l2 = hit / (hit + miss) if hit + miss else float("nan")
        lines.append(
            f"{eng:5s} {k:34s} wave-cyc {c.get('SQ_WAVE_CYCLES', 0):9.3g} L2hit {l2:5.3f} "
            f"inst/wave-cyc {ratio(c, 'SQ_ACTIVE_INST_ANY', 'SQ_WAVE_CYCLES'):5.3f} "
            f"wait/wave-cyc {ratio(c, 'SQ_WAIT_INST_ANY', 'SQ_WAVE_CYCLES'):5.3f} "
            f"lds-conf {ratio(c, 'SQ_LDS_BANK_CONFLICT', 'SQ_LDS_IDX_ACTIVE'):5.3f} "
            f"VALU {c.get('SQ_INSTS_VALU', 0):9.3g} LDS {c.get('SQ_INSTS_LDS', 0):9.3g} "
            f"VMEM_RD {c.get('SQ_INSTS_VMEM_RD', 0):9.3g} FETCH_SIZE(raw) {c.get('FETCH_SIZE', 0):9.3g}")
print("\n".join(lines))
