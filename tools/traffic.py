"""Per-volume HBM traffic of the hot kernels from a committed profile summary
(tools/summarize_prof.py output: FETCH_SIZE / WRITE_SIZE passes, gfx950
FETCH_SIZE correction already applied), written to profiles/traffic.json for
bench.py's roofline.traffic.

usage: python tools/traffic.py profiles/<name> --volumes V --volume-bytes N
  V = volumes the profiled command processed (warmup + steps + the single-volume run)
"""
import argparse
import json
import os

KERNELS = {"fingerprint": "fp_kernel<2>", "sha256": "sha_slice_kernel"}

ap = argparse.ArgumentParser()
ap.add_argument("prof")
ap.add_argument("--volumes", type=int, required=True)
ap.add_argument("--volume-bytes", type=int, default=1 << 36)
a = ap.parse_args()
s = json.load(open(os.path.join(a.prof, "summary.json")))
out = {"source": a.prof, "volumes": a.volumes, "volume_bytes": a.volume_bytes}
for stage, k in KERNELS.items():
    e = s[k]
    tot = (e["hbm_read_bytes_per_dispatch"] + e["hbm_write_bytes_per_dispatch"]) * e["calls"]
    out[stage] = {"kernel": k, "bytes_per_volume": tot / a.volumes,
                  "ratio_to_algorithmic": tot / a.volumes / a.volume_bytes}
json.dump(out, open(os.path.join(os.path.dirname(a.prof.rstrip("/")), "traffic.json"), "w"),
          indent=1)
print(json.dumps(out, indent=1))
