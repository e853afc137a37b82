"""Run the bf16 Gram kernel alone on the N=1e7, p=500 bench panel (A/B of the 256-tile
kernel variants, and for PMC profiling). Usage: gram_only.py [N] [tri|pair|tile256 ...]; ATE_BLOCKED=0 for a column-major panel"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ate_replication_causalml_amd.data.device_dgp import synthetic_panel  # noqa: E402
from ate_replication_causalml_amd.data import device_dgp  # noqa: E402

device_dgp.BYTE_PANEL = True      # the byte copy, so that pair / pair16 A/B both run
from ate_replication_causalml_amd.ops import gram as gram_mod  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else int(1e7)
variants = sys.argv[2:] or [gram_mod.GRAM_KERNEL]
pan = synthetic_panel(n, p=500, folds=5, seed=1991, dtype="bf16", device=torch.device("cuda", 0),
                      blocked=os.environ.get("ATE_BLOCKED", "1") == "1",
                      dgp=os.environ.get("ATE_DGP", "tutorial"))
ref = None
stage = os.environ.get("ATE_GRAM_STAGE", "all")   # "tiles": the tile kernel alone (no slab reduce)
for v in variants:
    # "tri": the split-triangle kernel (P == 512); "pair": the paired-tile kernel
    gram_mod.GRAM_KERNEL = "pair" if v in ("tri", "pair16") else v
    gram_mod.GRAM_TRI = v == "tri"
    gram_mod.BYTE_COLS = v != "pair16"      # pair16: the panel's byte columns read as bf16
    gram_mod._plan_cache.clear()
    for _ in range(3):
        G = gram_mod.gram(pan)
    torch.cuda.synchronize()
    e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e[0].record()
    for _ in range(10):
        gram_mod.gram(pan, stage=stage)
    e[1].record()
    torch.cuda.synchronize()
    G = G.clone()
    diff = 0.0 if ref is None else float((G - ref).abs().max() / ref.abs().max())
    ref = G if ref is None else ref
    print(f"kernel {v}: gram ms {e[0].elapsed_time(e[1]) / 10:.3f}  rel-diff vs first {diff:.2e}",
          flush=True)
