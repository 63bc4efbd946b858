"""Co-residency A/B: the fingerprint pass of one 64 GiB
volume and a SHA-256 hash of X GB of 64 KiB blobs, alone and launched
together, under the library build in VSGPU_LIB.  The co-residency build
(tools/build_variant.sh corun -DVS_FP_LB=1024 -DVS_FP_THREADS=640) runs the
fingerprint's persistent grid at 10 waves per CU within a 128-VGPR budget,
which leaves two SIMDs room for one split SHA-256 workgroup (32 KiB of LDS
beside the tables' 128 KiB) on every CU; --sha-grid 1 gives the hash launch
one workgroup per CU.  Wall times over interleaved repeats, the volume and the
blobs generated once.
  VSGPU_LIB=... python tools/corun.py --sha-gb 4,8 --sha-grid 1"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--gib", type=int, default=64)
ap.add_argument("--sha-gb", default="4,8")
ap.add_argument("--sha-grid", type=int, default=1, help="SHA-256 workgroups per CU (0 = default 5)")
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()

import torch  # noqa: E402

from volsync_amd import DeviceChunker, DeviceSha256, MaxSize, MinSize, TestPol, synth_fill_device  # noqa: E402
from volsync_amd._lib import VS_OPT_SHA_GRID_PER_CU  # noqa: E402

dev = torch.device("cuda", 0)
dlen = a.gib << 30
buf = torch.empty(dlen, dtype=torch.uint8, device=dev)
synth_fill_device(buf.data_ptr(), 2, 0, dlen, device=0, stream=torch.cuda.current_stream(dev).cuda_stream)
torch.cuda.synchronize(dev)
dc = DeviceChunker(TestPol, MinSize, MaxSize, 20, device=0)
sh = DeviceSha256(0)
sh.set_wide(0xffffffff, 0)                      # split mode only
sh.set_option(VS_OPT_SHA_GRID_PER_CU, a.sha_grid)
hs = torch.cuda.Stream(dev)
blob = 64 << 10
res = {}


def fp():
    dc.scan(buf.data_ptr(), dlen, 0, 0, dlen, True)


def run(x_gb, which):
    n = int(x_gb * 1e9) // blob
    offs = torch.arange(n, dtype=torch.int64, device=dev) * blob
    lens = torch.full((n,), blob, dtype=torch.int32, device=dev)
    out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if which in ("fp", "both"):
        fp()
    if which in ("sha", "both"):
        sh.run(buf.data_ptr(), offs.data_ptr(), lens.data_ptr(), n, out.data_ptr(), hs.cuda_stream)
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) * 1e3


fp()
torch.cuda.synchronize(dev)
for x in [float(v) for v in a.sha_gb.split(",")]:
    run(x, "sha")
    for r in range(a.rounds):
        for which in ("fp", "sha", "both"):
            res.setdefault(f"{x}:{which}", []).append(run(x, which))
    med = {w: statistics.median(res[f"{x}:{w}"]) for w in ("fp", "sha", "both")}
    print(f"X {x} GB: fp {med['fp']:.1f} ms, sha {med['sha']:.1f} ms, sum {med['fp'] + med['sha']:.1f}, "
          f"together {med['both']:.1f} ms", flush=True)
print(json.dumps({"lib": os.environ.get("VSGPU_LIB", "in-tree"), "sha_grid": a.sha_grid,
                  "ms": {k: [round(v, 2) for v in vs] for k, vs in res.items()}}))
dc.close()
sh.close()
