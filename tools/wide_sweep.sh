#!/bin/bash
# C2 bench over SHA-256 throughput-mode thresholds / drain budgets: "min:drain" pairs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for p in "$@"; do
  w=${p%%:*}; d=${p##*:}
  timeout -k 10 300 python bench.py --no-cpu-baseline --hash-wide $w --wide-drain $d > gpurun_out/sw_$p.log 2>&1 || { tail -20 gpurun_out/sw_$p.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sw_$p.log').read().strip().splitlines()[-1]); print('$p', d['value'], d['ms_per_step'], d['stages_ms_per_step'], d['single_volume']['ms'])"
done
