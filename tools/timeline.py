"""Timeline of a rocprofv3 kernel trace (``--kernel-trace --output-format csv``): for the
last ``--window`` ms of the trace, the busy time of each kernel class, the time covered by
at least one kernel, the time covered by the Gram, and the idle gaps.

  python tools/timeline.py gpurun_out/prof_bench/bench_kernel_trace.csv [--window 20]

Used to see where a bench step's time goes when two cross-fits overlap on two streams
(profiles/README.md).
"""
import argparse
import csv
import re
from collections import defaultdict

CLASSES = [("gram", r"gram_bf16_pair|gram_bf16_256|gram_bf16_kernel"),
           ("gram_reduce", r"gram_pair_reduce|slab_reduce|gram_.*reduce"),
           ("path", r"enet_path_kernel"),
           ("cvloss", r"cvloss"),
           ("resid", r"dml_resid"),
           ("prepare", r"enet_prep"),
           ("other", r".")]


def klass(name):
    for c, pat in CLASSES:
        if re.search(pat, name):
            return c
    return "other"


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def length(iv):
    return sum(b - a for a, b in iv)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window", type=float, default=20.0, help="ms at the end of the trace")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
           r.get("Queue_Id", "")) for r in rows]
    t1 = max(e[1] for e in ev)
    t0 = t1 - int(a.window * 1e6)
    ev = [(max(s, t0), e, n, q) for s, e, n, q in ev if e > t0]
    per = defaultdict(list)
    for s, e, n, q in ev:
        per[klass(n)].append((s, e))
    span = t1 - t0
    print(f"window {span / 1e6:.2f} ms, {len(ev)} kernels, queues "
          f"{sorted(set(q for *_, q in ev))}")
    for c, _ in CLASSES:
        if per[c]:
            iv = per[c]
            print(f"  {c:12s} n={len(iv):4d} sum={sum(e - s for s, e in iv) / 1e6:8.3f} ms  "
                  f"covered={length(union(iv)) / 1e6:8.3f} ms")
    allu = union([(s, e) for s, e, *_ in ev])
    busy = length(allu)
    print(f"  any kernel covered {busy / 1e6:.3f} ms ({100 * busy / span:.1f}%), idle "
          f"{(span - busy) / 1e6:.3f} ms")
    g = union(per["gram"])
    print(f"  gram covered {length(g) / 1e6:.3f} ms ({100 * length(g) / span:.1f}%)")
    gaps = [(allu[i][1], allu[i + 1][0]) for i in range(len(allu) - 1)]
    gaps = sorted(gaps, key=lambda x: x[0] - x[1])[:8]
    print("  largest idle gaps (us):", [round((b - a) / 1e3, 1) for a, b in gaps])
    # intervals where no Gram runs: which kernels run there
    nog = defaultdict(int)
    gi = 0
    for c, iv in per.items():
        if c == "gram":
            continue
        for s, e in iv:
            cov = 0
            for a_, b_ in g:
                cov += max(0, min(e, b_) - max(s, a_))
            nog[c] += (e - s) - cov
    print("  kernel time outside any Gram (ms):",
          {c: round(v / 1e6, 3) for c, v in nog.items() if v})
    ng = span - length(g)
    print(f"  time with no Gram running: {ng / 1e6:.3f} ms")



def overlapped(trace, last=12):
    """Print the last ``last`` Gram / path kernels on the side-stream queues (the timed,
    overlapped part of a bench run) with their queue, start, end and duration."""
    rows = list(csv.DictReader(open(trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), klass(r["Kernel_Name"]),
                 r["Queue_Id"]) for r in rows)
    qs = sorted(set(e[3] for e in ev))
    side = [e for e in ev if e[3] != qs[0] and e[2] in ("gram", "path", "prepare", "cvloss")]
    t0 = side[0][0]
    for s, e, c, q in side[-last:]:
        print(f"  {(s - t0) / 1e6:9.3f} {(e - t0) / 1e6:9.3f} {(e - s) / 1e6:6.3f} {c:8s} q{q}")


if __name__ == "__main__":
    main()
