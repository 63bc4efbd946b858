"""Single-pass latency of one volume (no replay): scan .. drain, every blob ID
final, per drain rule.  One process, volume generated once.
  python tools/single_pass.py --gib 64                 # C2 (seed 2)
  python tools/single_pass.py --share 3/8              # C3 rank 3 (128 GiB of the seed-3 TiB)
  --quad auto:1,auto:2,auto:0   drain rules to compare, interleaved: VS_OPT_SHA_QUAD_PCT
                              (auto = -1) : VS_OPT_SHA_ISOLATE (quad tiles per reserved CU)
Prints one line per pass and a JSON summary (min / median per rule)."""
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
ap.add_argument("--share", default=None)
ap.add_argument("--quad", default="auto:1,auto:0")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--no-check", action="store_true", help="timing diagnostics (VS_SHA_DIAG builds): skip the golden check")
a = ap.parse_args()

import torch  # noqa: E402

from bench import _chunk_records, _goldens  # noqa: E402
from volsync_amd import DeviceChunker, MaxSize, MinSize, TestPol, synth_fill_device  # noqa: E402
from volsync_amd._lib import VS_OPT_SHA_ISOLATE, VS_OPT_SHA_QUAD_PCT  # noqa: E402
from volsync_amd.shard import ShardSpec  # noqa: E402

dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev).cuda_stream
if a.share:
    r, w = (int(x) for x in a.share.split("/"))
    seed, total = 3, w * (128 << 30)
    spec = ShardSpec.for_rank(total, w, r, MaxSize)
    gold = _goldens()["cdc"]["3"][str(total)]["ranks"][r]
    entry = gold["entry"]
else:
    seed, total = 2, a.gib << 30
    spec = ShardSpec.for_rank(total, 1, 0, MaxSize)
    gold = _goldens()["cdc"]["2"].get(str(total))
    entry = None
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


rules = a.quad.split(",")
res = {q: [] for q in rules}
one()
dc.wait()
for rd in range(a.rounds):
    for q in rules:
        qp, iso = (q.split(":") + ["1"])[:2]
        dc.set_option(VS_OPT_SHA_QUAD_PCT, -1 if qp == "auto" else int(qp))
        dc.set_option(VS_OPT_SHA_ISOLATE, int(iso))
        torch.cuda.synchronize(dev)
        dc.timing(True)
        t0 = time.perf_counter()
        n = one()
        dc.wait()
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) * 1e3
        ms, _ = dc.timing(False)
        det = dc.timing_detail()
        res[q].append(dt)
        import hashlib
        d = hashlib.sha256(_chunk_records(dc, n)).hexdigest()
        if gold is not None and not a.no_check and (n, d) != (gold["chunks"], gold["digest"]):
            print(f"[{q} r{rd}] CHUNK LIST DIFFERS FROM THE GOLDEN", flush=True)
            sys.exit(1)
        print(f"[{q} r{rd}] {dt:.1f} ms  fp {ms[0]:.1f}  sha(outside fp) {det['sha_outside_fp_ms']:.1f}"
              f"  latency-mode chains {det['quad_chains']}  chunks {n}", flush=True)
ok = gold is not None and not a.no_check   # every pass's list was checked against it above
print(json.dumps({"volume": a.share or f"C2 {a.gib} GiB", "bytes": spec.own_hi - spec.own_lo,
                  "golden_match_every_pass": ok,
                  "ms": {q: {"min": round(min(v), 1), "median": round(statistics.median(v), 1)}
                         for q, v in res.items()},
                  "lib": os.environ.get("VSGPU_LIB", "in-tree")}))
dc.close()
