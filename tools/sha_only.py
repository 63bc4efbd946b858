"""Hash-engine driver for profiling: one 64 GiB volume chunked, its chunks
hashed with one budget-bounded slice, then drained (the first slice is the
full-width regime: one tile per workgroup)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from volsync_amd import DeviceChunker, MaxSize, MinSize, TestPol, synth_fill_device  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--gib", type=float, default=64)
ap.add_argument("--slice", type=int, default=8192)
ap.add_argument("--vols", type=int, default=1)
a = ap.parse_args()
n = int(a.gib * (1 << 30))
buf = torch.empty(n, dtype=torch.uint8, device="cuda")
synth_fill_device(buf.data_ptr(), 2, 0, n)
torch.cuda.synchronize()
dc = DeviceChunker(TestPol, MinSize, MaxSize, 20)
dc.set_hash_slice(a.slice)
dc.timing(True)
t0 = time.perf_counter()
for _ in range(a.vols):
    dc.process(buf.data_ptr(), n, 0, True)
dc.wait()
dt = time.perf_counter() - t0
ms, cnt = dc.timing(False)
print(f"{a.vols} x {a.gib} GiB: {dt * 1e3:.1f} ms, stages {ms} launches {cnt}")
