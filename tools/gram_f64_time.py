"""Time the fp64 (parity-mode) Gram alone: N=1e7 rows x P=512 fp64 panel (41 GB in HBM),
ops/gram.gram -> csrc/gram.hip gram_small_kernel<double> + fixed-order fp64 reduce.
Prints ms per Gram and the TFLOP/s of the upper-triangle tiles it computes.

    python tools/gram_f64_time.py [rows]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ate_replication_causalml_amd  # noqa: E402,F401


def main():
    import torch
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.ops import gram as G
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10_000_000
    dev = torch.device("cuda", 0)
    pan = synthetic_panel(n, p=500, dtype="f64", device=dev)
    torch.cuda.synchronize()
    G.gram(pan)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        G.gram(pan)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ms = 1e3 * min(ts)
    P = pan.P
    nt = P // 64
    flop = 2.0 * pan.ld * (nt * (nt + 1) // 2) * 64 * 64
    print(f"fp64 Gram rows={pan.ld} P={P}: {ms:.2f} ms (min of 5; all {[round(1e3 * t, 2) for t in ts]}),"
          f" {flop / (ms * 1e-3) / 1e12:.1f} TFLOP/s over the upper-triangle 64x64 tiles", flush=True)


if __name__ == "__main__":
    main()
