"""HBM read-rate reference points on the 10.24 GB bench panel (one MI355X): torch reductions
and copies over the same buffer the Gram streams (is ~4.2 TB/s a property of the Gram's
access pattern or of the buffer?)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ate_replication_causalml_amd.data.device_dgp import synthetic_panel  # noqa: E402


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - a) / reps


dev = torch.device("cuda", 0)
pan = synthetic_panel(10_000_000, p=500, folds=5, seed=1, dtype="bf16", device=dev, blocked=True)
X = pan.data
nb = X.numel() * 2
flat = X.view(-1).view(torch.int32)
s = t(lambda: flat.sum(dtype=torch.int64))
print(f"int32 sum over {nb / 1e9:.2f} GB: {s * 1e3:.3f} ms = {nb / s / 1e12:.2f} TB/s", flush=True)
f32 = X.view(-1).view(torch.float32)
s = t(lambda: torch.amax(f32))
print(f"amax(fp32 view): {s * 1e3:.3f} ms = {nb / s / 1e12:.2f} TB/s", flush=True)
out = torch.empty_like(X)
s = t(lambda: out.copy_(X))
print(f"copy (read+write {2 * nb / 1e9:.1f} GB): {s * 1e3:.3f} ms = {2 * nb / s / 1e12:.2f} TB/s",
      flush=True)
