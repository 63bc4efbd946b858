"""Summarise a rocprofv3 output directory (tools/profile.sh layout) per kernel.

usage: python tools/summarize_prof.py gpurun_out/prof_<tag> [--out profiles/<name>]

Reads <dir>/trace/*_kernel_stats.csv (kernel-trace --stats) and every
<dir>/pmc_*/*_counter_collection.csv (one --pmc pass each), and writes
summary.json + summary.md: per kernel the dispatch count, average duration
and the per-dispatch average of each counter.  HBM bytes follow
MI355X_MICROARCH.md section HBM: FETCH_SIZE (KiB) reads 1/2 of a wide
coalesced stream on gfx950, so hbm_read_bytes = 2 * FETCH_SIZE * 1024;
WRITE_SIZE (KiB) is exact for 16-B stores.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import shutil


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n.replace("void ", "").replace("vsgpu::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    stats = {}
    for f in glob.glob(os.path.join(a.dir, "trace", "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            stats[short(r["Name"])] = {"calls": int(r["Calls"]),
                                       "avg_us": float(r["AverageNs"]) / 1e3,
                                       "total_ms": float(r["TotalDurationNs"]) / 1e6,
                                       "pct": float(r["Percentage"])}
    counters = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(a.dir, "pmc_*", "*counter_collection.csv")):
        per = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
        for (d, c), v in per.items():
            counters[names[d]][c].append(v)
    out = {}
    for k in sorted(set(stats) | set(counters), key=lambda x: -stats.get(x, {}).get("total_ms", 0)):
        e = dict(stats.get(k, {}))
        for c, vals in counters.get(k, {}).items():
            e[c] = sum(vals) / len(vals)
        if "FETCH_SIZE" in e:
            e["hbm_read_bytes_per_dispatch"] = 2 * e["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in e:
            e["hbm_write_bytes_per_dispatch"] = e["WRITE_SIZE"] * 1024
        out[k] = e
    dst = a.out or a.dir
    os.makedirs(dst, exist_ok=True)
    json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    lines = ["| kernel | calls | avg us | % time | extra |", "|---|---|---|---|---|"]
    for k, e in out.items():
        extra = ", ".join(f"{c}={v:.4g}" for c, v in e.items()
                          if c not in ("calls", "avg_us", "total_ms", "pct"))
        lines.append(f"| {k} | {e.get('calls', '')} | {e.get('avg_us', 0):.1f} | "
                     f"{e.get('pct', 0):.2f} | {extra} |")
    open(os.path.join(dst, "summary.md"), "w").write("\n".join(lines) + "\n")
    if a.out:
        for f in glob.glob(os.path.join(a.dir, "trace", "*kernel_stats.csv")):
            shutil.copy(f, dst)
    print("\n".join(lines[:14]))


if __name__ == "__main__":
    main()
