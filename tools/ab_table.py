"""Tabulate tools/ab.py logs of bench.py --mode rsync lines: variant, round,
value, walk_spec ms, false alarms, matches.
  python tools/ab_table.py gpurun_out/ab_share.log [...]"""
import json
import re
import sys

for path in sys.argv[1:]:
    print(f"== {path}")
    for line in open(path):
        m = re.match(r"\[(\S+) (r\d+)\] rc=(\d+) (.*)", line)
        if not m:
            continue
        try:
            d = json.loads(m.group(4).split(" | ")[-1])
        except ValueError:
            print(m.group(1), m.group(2), "rc", m.group(3), "(no JSON line)")
            continue
        ms = d.get("match_stats", {})
        print(f"{m.group(1):8s} {m.group(2)} {d['value']:9.2f} GB/s  walk_spec "
              f"{d.get('kernels_ms_per_step', {}).get('walk_spec', float('nan')):7.3f} ms  "
              f"fa {ms.get('false_alarms')}  matches {ms.get('matches')}")
