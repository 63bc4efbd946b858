#!/bin/bash
# Sweep bench.py variants on one box: each run under its own time limit; stop at
# the first fault / timeout.  Usage: tools/bench_sweep.sh "<args1>" "<args2>" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i+1))
  echo "=== sweep$i: $a" >> gpurun_out/sweep.log
  timeout -k 10 300 python bench.py --no-cpu-baseline $a > gpurun_out/sweep$i.log 2>&1
  rc=$?
  echo "rc=$rc" >> gpurun_out/sweep.log
  tail -1 gpurun_out/sweep$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['stages_ms_per_step'], d['single_volume']['ms'])" >> gpurun_out/sweep.log 2>&1
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
