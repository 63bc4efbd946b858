#!/bin/bash
# Round-end evidence: GPU tests, smoke, default bench (C2, with cpu_baseline),
# C5 and C4 bench lines, then rocprofv3 passes over the default bench command.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_check.sh smoke tests bench || exit $?
grep -q "rc=0" gpurun_out/steps.log || exit 1
timeout -k 10 400 python bench.py --mode smallfiles > gpurun_out/bench_c5.log 2>&1 || { tail -20 gpurun_out/bench_c5.log; exit 1; }
tail -1 gpurun_out/bench_c5.log | cut -c1-300
timeout -k 10 600 python bench.py --mode rsync --steps 3 --warmup 1 > gpurun_out/bench_c4.log 2>&1 || { tail -20 gpurun_out/bench_c4.log; exit 1; }
tail -1 gpurun_out/bench_c4.log | cut -c1-300
timeout -k 10 400 python bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 > gpurun_out/bench_c4_share.log 2>&1 || { tail -20 gpurun_out/bench_c4_share.log; exit 1; }
tail -1 gpurun_out/bench_c4_share.log | cut -c1-300
bash tools/profile.sh final || exit $?
cat gpurun_out/prof_final/steps.log
