"""Where and when the single-pass drain's tiles run (VS_SHA_TRACE builds:
tools/build_variant.sh shatrace -DVS_SHA_TRACE=1, then VSGPU_LIB=...).
One volume (C2, or --share R/8 for a C3 rank) per drain rule; per rule it
prints the latency (quad) tiles' start / duration spread and how many split
tiles ran on a CU (and on a SIMD) while a quad tile was running there.
  VSGPU_LIB=volsync_amd/lib/var/shatrace/libvsgpu.so python tools/sha_trace.py --share 3/8"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--gib", type=int, default=64)
ap.add_argument("--share", default=None)
ap.add_argument("--quad", default="auto:1,auto:0")
a = ap.parse_args()

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import _goldens  # noqa: E402
from volsync_amd import DeviceChunker, MaxSize, MinSize, TestPol, synth_fill_device  # noqa: E402
from volsync_amd._lib import VS_OPT_SHA_ISOLATE, VS_OPT_SHA_QUAD_PCT, lib  # noqa: E402
from volsync_amd.shard import ShardSpec  # noqa: E402

fn = lib.vs_debug_sha_trace
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]

dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev).cuda_stream
if a.share:
    r, w = (int(x) for x in a.share.split("/"))
    seed, total = 3, w * (128 << 30)
    spec = ShardSpec.for_rank(total, w, r, MaxSize)
    entry = _goldens()["cdc"]["3"][str(total)]["ranks"][r]["entry"]
else:
    seed, total = 2, a.gib << 30
    spec = ShardSpec.for_rank(total, 1, 0, MaxSize)
dlen = spec.data_hi - spec.data_lo
buf = torch.empty(dlen, dtype=torch.uint8, device=dev)
synth_fill_device(buf.data_ptr(), seed, spec.data_lo, dlen, device=0, stream=stream)
torch.cuda.synchronize(dev)
dc = DeviceChunker(TestPol, MinSize, MaxSize, 20, device=0)


def one():
    if a.share:
        dc.scan(buf.data_ptr(), dlen, spec.data_lo, spec.own_lo, spec.own_hi, spec.final)
        dc.stitch(entry)
        return dc.finish()
    return dc.process(buf.data_ptr(), dlen, 0, True)[0]


n0 = one()
dc.wait()
from bench import _chunk_records  # noqa: E402
rec = np.frombuffer(_chunk_records(dc, n0), dtype=np.uint64).reshape(n0, 7)
lmax_blocks = int(rec[:, 1].max()) // 64 + 1   # the longest chunk's SHA-256 blocks
print("longest chunk", int(rec[:, 1].max()), "bytes,", lmax_blocks, "blocks", flush=True)
cap = 1 << 16
arr = np.zeros((cap, 4), np.uint64)
n = ctypes.c_uint32(0)
out = {}
for q in a.quad.split(","):
    qp, iso = (q.split(":") + ["1"])[:2]
    dc.set_option(VS_OPT_SHA_QUAD_PCT, -1 if qp == "auto" else int(qp))
    dc.set_option(VS_OPT_SHA_ISOLATE, int(iso))
    fn(None, 0, ctypes.byref(n), 1)
    one()
    dc.wait()
    torch.cuda.synchronize(dev)
    fn(arr.ctypes.data, cap, ctypes.byref(n), 1)
    t = arr[: n.value]
    quad = (t[:, 0] >> np.uint64(63)) == 1
    cyc = ((t[:, 0] >> np.uint64(20)) & np.uint64((1 << 43) - 1)).astype(np.int64)
    hw = (t[:, 1] & np.uint64(0xffffffff)).astype(np.int64)
    xcc = (t[:, 1] >> np.uint64(32)).astype(np.int64)
    cu = xcc * 4096 + ((hw >> 13) & 7) * 512 + ((hw >> 12) & 1) * 256 + ((hw >> 8) & 15)
    simd = cu * 4 + ((hw >> 4) & 3)
    t0, t1 = t[:, 2].astype(np.int64), t[:, 3].astype(np.int64)
    base = int(t0.min())
    qi = np.nonzero(quad)[0]
    si = np.nonzero(~quad)[0]
    drain0 = int(t0[qi].min()) if len(qi) else base
    res = {"tiles": int(n.value), "quad_tiles": int(len(qi)), "longest_chain_blocks": lmax_blocks}
    if len(qi):
        qs = (t0[qi] - drain0) / 1e5
        qd = (t1[qi] - t0[qi]) / 1e5
        res.update({"quad_start_ms": [round(float(qs.min()), 2), round(float(np.median(qs)), 2),
                                      round(float(qs.max()), 2)],
                    "quad_ms": [round(float(qd.min()), 1), round(float(np.median(qd)), 1),
                                round(float(qd.max()), 1)],
                    # shader clock over the tile (s_memtime cycles / s_memrealtime)
                    "quad_clock_GHz": [round(float(x), 3) for x in
                                       np.percentile(cyc[qi] / np.maximum(t1[qi] - t0[qi], 1) / 10.0, [0, 50, 100])],
                    "quad_distinct_cus": int(len(set(cu[qi].tolist()))),
                    "quad_distinct_simds": int(len(set(simd[qi].tolist())))})
        # split tiles overlapping a quad tile in time on its CU / SIMD
        on_cu = on_simd = 0
        for k in qi:
            ov = (t0[si] < t1[k]) & (t1[si] > t0[k])
            on_cu += int(np.sum(ov & (cu[si] == cu[k])))
            on_simd += int(np.sum(ov & (simd[si] == simd[k])))
        res["split_tiles_beside_quad"] = {"same_cu": on_cu, "same_simd": on_simd}
        late = si[t0[si] >= drain0]
        if len(late):
            res["split_after_drain_start_ms"] = round(float((t1[late].max() - drain0) / 1e5), 1)
    res["span_ms"] = round(float((t1.max() - base) / 1e5), 1)
    if len(si):
        res["split_clock_GHz_median"] = round(float(np.median(cyc[si] / np.maximum(t1[si] - t0[si], 1) / 10.0)), 3)
    out[q] = res
    print(q, json.dumps(res), flush=True)
print(json.dumps({"volume": a.share or f"C2 {a.gib} GiB", "rules": out}))
dc.close()
