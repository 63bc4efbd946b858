#!/bin/bash
# C4 at its real table size: one rank's share (3 of 8: 32 GiB of D, the full
# 2 M-block table, 32 GiB of S) on one GPU; then the default C2 line again
# (box-to-box spread).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 \
  > gpurun_out/bench_c4_share.log 2>&1 || { tail -20 gpurun_out/bench_c4_share.log; exit 1; }
tail -1 gpurun_out/bench_c4_share.log | cut -c1-2500
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_c2b.log 2>&1 || { tail -20 gpurun_out/bench_c2b.log; exit 1; }
tail -1 gpurun_out/bench_c2b.log | cut -c1-600
