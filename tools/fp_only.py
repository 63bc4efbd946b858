"""Fingerprint-stage driver for profiling: scan() only (fingerprint + candidate
index + speculative walks) over a device-resident synthetic volume."""
import argparse, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from volsync_amd import DeviceChunker, TestPol, MinSize, MaxSize, synth_fill_device
ap = argparse.ArgumentParser(); ap.add_argument("--gib", type=float, default=16); ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
n = int(a.gib * (1 << 30))
buf = torch.empty(n, dtype=torch.uint8, device="cuda")
synth_fill_device(buf.data_ptr(), 2, 0, n); torch.cuda.synchronize()
dc = DeviceChunker(TestPol, MinSize, MaxSize, 20)
dc.timing(True)
for _ in range(a.reps):
    dc.scan(buf.data_ptr(), n, 0, 0, n, True)
    dc.stitch(0)
ms, cnt = dc.timing(False)
print(f"fingerprint {ms[0]/a.reps:.3f} ms/volume = {n/(ms[0]/a.reps)/1e6:.1f} GB/s ({os.environ.get('VSGPU_FP_VARIANT','2')})")
