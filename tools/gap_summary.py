"""Idle gaps between kernels in a rocprofv3 kernel trace (``--kernel-trace --output-format
csv``): over the window from the first to the last kernel whose name matches PATTERN, the
time covered by at least one kernel, the idle time, and the gaps by size -- how much of a
host-driven loop (the forest level engine, tools/forest_level_probe.py) is host overhead.

  python tools/gap_summary.py TRACE.csv [PATTERN]     (default pattern: lv_)
"""
import csv
import re
import sys


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"lv_")
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in rows)
    hit = [e for e in ev if pat.search(e[2])]
    if not hit:
        print("no kernel matches", pat.pattern)
        return
    w0, w1 = hit[0][0], max(e[1] for e in hit)
    iv = sorted((max(s, w0), min(e, w1)) for s, e, _ in ev if e > w0 and s < w1)
    busy, gaps, cur = 0, [], None
    for s, e in iv:
        if cur is None:
            cur = [s, e]
        elif s <= cur[1]:
            cur[1] = max(cur[1], e)
        else:
            busy += cur[1] - cur[0]
            gaps.append(s - cur[1])
            cur = [s, e]
    busy += cur[1] - cur[0]
    span = w1 - w0
    big = [g for g in gaps if g > 10_000]
    print(f"window {span / 1e6:.2f} ms, {len(hit)} matching kernels of {len(iv)}: busy "
          f"{busy / 1e6:.2f} ms ({100 * busy / span:.1f} %), idle {(span - busy) / 1e6:.2f} ms "
          f"in {len(gaps)} gaps; gaps > 10 us: {len(big)} totalling {sum(big) / 1e6:.2f} ms "
          f"(median {sorted(big)[len(big) // 2] / 1e3 if big else 0:.1f} us)")


if __name__ == "__main__":
    main()
