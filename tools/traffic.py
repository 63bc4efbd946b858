"""Per-unit HBM traffic of the hot kernels from committed profile summaries
(tools/summarize_prof.py output: FETCH_SIZE / WRITE_SIZE passes, gfx950
FETCH_SIZE correction already applied), written to profiles/traffic.json for
bench.py's roofline.traffic.

usage: python tools/traffic.py profiles/<round> [--volumes V] [--volume-bytes N]
  <round>/c2:   the C2 bench under tools/prof_mode.sh (V = volumes it processed:
                warmup + steps + the single-volume run)
  <round>/c4:   the C4 bench (--mode rsync): rs_walk_spec_kernel bytes per
                source byte (one launch per step over the whole source)
  <round>/seal: the seal bench: seal_ctr_kernel / seal_mac_kernel bytes per
                plaintext byte
"""
import argparse
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("prof")
ap.add_argument("--volumes", type=int, default=4)
ap.add_argument("--volume-bytes", type=int, default=1 << 36)
ap.add_argument("--c4-source-bytes", type=int, default=68719492223)
ap.add_argument("--seal-bytes", type=int, default=68718991021)
# rank 3 of 8 of the real C4 (--mode rsync --share 3/8 --per-gpu-gib 32): its own S range
ap.add_argument("--c4-share-source-bytes", type=int, default=34359736410)
a = ap.parse_args()


def load(sub):
    p = os.path.join(a.prof, sub, "summary.json")
    return json.load(open(p)) if os.path.exists(p) else None


def total(e):
    return (e["hbm_read_bytes_per_dispatch"] + e["hbm_write_bytes_per_dispatch"]) * e["calls"]


# sections this profile round does not hold keep their earlier source
tj = os.path.join(os.path.dirname(a.prof.rstrip("/")), "traffic.json")
out = json.load(open(tj)) if os.path.exists(tj) else {}
def find(s, base, prefix=None):
    """the summary entry of kernel `base` (template arguments ignored, or
    the one whose name starts with `prefix`)"""
    for n, v in s.items():
        if (n.startswith(prefix) if prefix else n.split("<")[0] == base):
            return v
    raise KeyError(base)


s = load("c2")
if s:
    out.update({"source": a.prof, "volumes": a.volumes, "volume_bytes": a.volume_bytes})
    # the fingerprint variant the C2 bench runs (fp_kernel<3, ...>: FAST53 since
    # round 5): the fp_kernel instantiation with the most time
    fp = max((v for n, v in s.items() if n.split("<")[0] == "fp_kernel"),
             key=lambda v: v.get("total_ms", 0))
    for stage, k in {"fingerprint": "fp_kernel", "sha256": "sha_slice_kernel"}.items():
        t = total(fp if k == "fp_kernel" else find(s, k))
        out[stage] = {"kernel": k, "bytes_per_volume": t / a.volumes,
                      "ratio_to_algorithmic": t / a.volumes / a.volume_bytes}
s = load("c4")
if s:
    e = find(s, "rs_walk_spec_kernel")
    per = e["hbm_read_bytes_per_dispatch"] + e["hbm_write_bytes_per_dispatch"]
    out["rs_walk_spec"] = {"kernel": "rs_walk_spec_kernel", "source": os.path.join(a.prof, "c4"),
                           "bytes_per_source_byte": per / a.c4_source_bytes}
s = load("c4_share")
if s:
    e = find(s, "rs_walk_spec_kernel")
    per = e["hbm_read_bytes_per_dispatch"] + e["hbm_write_bytes_per_dispatch"]
    out["rs_walk_spec_share"] = {
        "kernel": "rs_walk_spec_kernel", "source": os.path.join(a.prof, "c4_share"),
        "config": "--mode rsync --share 3/8 --per-gpu-gib 32 (2 M-block table)",
        "bytes_per_source_byte": per / a.c4_share_source_bytes}
s = load("seal")
if s:
    for stage, k in {"seal_ctr": "seal_ctr_kernel", "seal_mac": "seal_mac_kernel"}.items():
        e = next((v for n, v in s.items() if n.split("<")[0] == k), None)
        if e and "hbm_read_bytes_per_dispatch" in e:
            per = e["hbm_read_bytes_per_dispatch"] + e["hbm_write_bytes_per_dispatch"]
            out[stage] = {"kernel": k, "source": os.path.join(a.prof, "seal"),
                          "bytes_per_plain_byte": per / a.seal_bytes}
json.dump(out, open(tj, "w"), indent=1)
print(json.dumps(out, indent=1))
