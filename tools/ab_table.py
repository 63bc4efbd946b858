"""Tabulate bench.py --mode rsync / cdc JSON lines: value, step time, the
walk's kernel times, false alarms, matches and the golden checks.
  python tools/ab_table.py gpurun_out/bench_ab_*.log      (one bench log each)
  python tools/ab_table.py gpurun_out/ab_share.log         (tools/ab.py output:
                                                            [variant rN] rc=.. lines)"""
import json
import os
import re
import sys


def fmt(name, d):
    k = d.get("kernels_ms_per_step", {})
    ms = d.get("match_stats", {})
    ex = d.get("exact", {})
    fsm = (d.get("file_sum") or {}).get("golden_match")
    return (f"{name:32s} {d['value']:9.1f} {d.get('unit', '')} {d['ms_per_step']:8.2f} ms/step  "
            f"walk_spec {k.get('walk_spec', float('nan')):7.2f}  stitch "
            f"{k.get('walk_stitch', float('nan')):6.2f}  fa {ms.get('false_alarms')}  matches "
            f"{ms.get('matches', d.get('config', {}).get('chunks'))}  golden "
            f"{ex.get('golden_match')}" + (f"  file_sum {fsm}" if fsm is not None else ""))


def table(path):
    rows, last = [], None
    for line in open(path, errors="replace"):
        m = re.match(r"\[(\S+) (r\d+)\] rc=(\d+) (.*)", line)
        if m:   # tools/ab.py
            try:
                rows.append(fmt(f"{m.group(1)} {m.group(2)}",
                                json.loads(m.group(4).split(" | ")[-1])))
            except ValueError:
                rows.append(f"{m.group(1)} {m.group(2)} rc {m.group(3)} (no JSON line)")
        elif line.startswith("{"):
            last = line
    if last is not None:
        rows.append(fmt(os.path.basename(path), json.loads(last)))
    return rows or [f"{os.path.basename(path)} (no JSON line)"]


if __name__ == "__main__":
    for p in sys.argv[1:]:
        for r in table(p):
            print(r)
