"""Does GPU_MAX_HW_QUEUES set from Python take effect? 8 streams x one long sleep kernel:
wall ~1x a sleep if the streams get their own hardware queues, ~2x with 4 queues.
  python tools/hwq_probe.py before|after|none   (set the variable before / after import torch)"""
import os
import sys
import time

mode = sys.argv[1] if len(sys.argv) > 1 else "before"
if mode == "before":
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
import torch  # noqa: E402
if mode == "after":
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
torch.cuda.init()
ss = [torch.cuda.Stream() for _ in range(8)]
torch.cuda._sleep(1000)
torch.cuda.synchronize()
t0 = time.perf_counter()
torch.cuda._sleep(200_000_000)
torch.cuda.synchronize()
one = time.perf_counter() - t0
t0 = time.perf_counter()
for s in ss:
    with torch.cuda.stream(s):
        torch.cuda._sleep(200_000_000)
torch.cuda.synchronize()
eight = time.perf_counter() - t0
print(f"{mode}: env={os.environ.get('GPU_MAX_HW_QUEUES')} one sleep {one*1e3:.1f} ms, 8 streams {eight*1e3:.1f} ms "
      f"({eight/one:.2f}x)", flush=True)
