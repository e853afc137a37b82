"""Does the buffer matter? Runs tools/hbm_stream.hip's LDS-DMA stream (64 KB x 2 stages, one
512-thread workgroup per CU) over (a) a torch.empty byte buffer and (b) the N=1e7 p=500 bench
panel from synthetic_panel (blocked), and compares with the Gram tile kernel on that panel.
  hipcc -O3 -shared -fPIC --offload-arch=gfx950 tools/hbm_stream.hip -o tools/libhbm_stream.so
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ate_replication_causalml_amd.data.device_dgp import synthetic_panel  # noqa: E402

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libhbm_stream.so"))
lib.hbm_dma_probe.restype = ctypes.c_float
lib.hbm_dma_probe.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_int]


def probe(t, tag):
    nb = t.numel() * t.element_size()
    for wg, share in ((256, 1), (1024, 1), (256, 2)):
        ms = lib.hbm_dma_probe(t.data_ptr(), nb, wg, 5, share)
        print(f"{tag:28s} wg={wg:5d} readers/byte={share}: {ms:.3f} ms = {nb / ms / 1e9:.2f} TB/s", flush=True)


dev = torch.device("cuda", 0)
nb = 10_240_000_000
b = torch.empty(nb, dtype=torch.uint8, device=dev)
b.fill_(1)
probe(b, "torch.empty byte buffer")
del b
torch.cuda.empty_cache()
pan = synthetic_panel(10_000_000, p=500, folds=5, seed=1, dtype="bf16", device=dev, blocked=True)
print("panel shape", tuple(pan.data.shape), "strides", pan.strides(), flush=True)
probe(pan.data, "bench panel (blocked)")
