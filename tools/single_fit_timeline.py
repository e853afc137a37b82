"""Kernel sequence of the LAST single-fit replay in a kernel trace of ``bench.py --parity 0``
(the latency replays run last): every kernel from the replay's first kernel to its last,
with start offset, duration and the idle gap before it; then the replay's wall, busy time
and the sums per kernel class. Shows what sits on the single call's critical path.

  python tools/single_fit_timeline.py TRACE.csv
"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0])
                for r in rows)
    grams = [i for i, e in enumerate(ev) if "gram_bf16_pair" in e[2]]
    g = grams[-1]
    # the replay starts after the previous replay's last kernel: walk back from the last Gram
    # to the largest gap (the host sync + barrier between replays)
    i0 = g
    while i0 > 0 and ev[i0][0] - ev[i0 - 1][1] < 50_000:
        i0 -= 1
    seq = ev[i0:]
    t0 = seq[0][0]
    end = t0
    busy = 0
    cls = defaultdict(int)
    print(f"{'start_us':>9} {'dur_us':>8} {'gap_us':>7}  kernel")
    for s, e, k in seq:
        gap = max(0, s - end)
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {gap / 1e3:7.1f}  {k[-70:]}")
        busy += max(0, e - max(s, end))
        end = max(end, e)
        cls[k[-40:]] += e - s
    wall = end - t0
    print(f"replay wall {wall / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {(wall - busy) / 1e3:.1f} us")
    for k, v in sorted(cls.items(), key=lambda kv: -kv[1])[:12]:
        print(f"  {v / 1e3:9.1f} us  {k}")


if __name__ == "__main__":
    main()
