#!/bin/bash
# C5 small-files bench and C2 bench, SHA-256 engine throughput mode on (default) / off
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
set -o pipefail
for w in 0 0xffffffff; do
  timeout -k 10 300 python bench.py --mode smallfiles --steps 3 --warmup 1 --hash-wide $w --no-cpu-baseline > gpurun_out/c5_w$w.log 2>&1 || { tail -20 gpurun_out/c5_w$w.log; exit 1; }
  tail -1 gpurun_out/c5_w$w.log | cut -c1-700
done
for w in 0 0xffffffff; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --hash-wide $w > gpurun_out/bench_w$w.log 2>&1 || { tail -20 gpurun_out/bench_w$w.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_w$w.log').read().strip().splitlines()[-1]); print('$w', d['value'], d['ms_per_step'], d['stages_ms_per_step'], d['sha_slices'], d['single_volume']['ms'])"
done
