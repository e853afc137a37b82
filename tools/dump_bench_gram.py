"""Dump the bench panel's fold Gram stack (N=1e7, p=500, bf16 panel, 5 segments) for
CPU-side studies of the CV path solver (tools/enet_sim.py):

  python tools/dump_bench_gram.py OUTDIR      (GPU box)

Writes OUTDIR/G.npy (float64 [nseg, P, P]) and OUTDIR/meta.json (column map, segment
row counts)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ate_replication_causalml_amd.data.device_dgp import synthetic_panel  # noqa: E402
from ate_replication_causalml_amd.ops.gram import gram  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/gram_dump"
os.makedirs(out, exist_ok=True)
dev = torch.device("cuda", 0)
pan = synthetic_panel(int(1e7), p=500, folds=5, seed=1991, dtype="bf16", device=dev,
                      dgp=os.environ.get("ATE_DGP", "tutorial"))
G = gram(pan).double().cpu().numpy()
np.save(os.path.join(out, "G.npy"), G)
meta = {"xcols": [int(c) for c in pan.xcols], "Y": int(pan.cols["Y"]), "W": int(pan.cols["W"]),
        "one": int(pan.cols["one"]), "seg_nreal": [int(c) for c in pan.seg_nreal],
        "P": int(G.shape[1])}
with open(os.path.join(out, "meta.json"), "w") as f:
    json.dump(meta, f)
print("dumped", G.shape, out, flush=True)
