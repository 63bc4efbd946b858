#!/bin/bash
# walk phase profile (VSGPU_WALK_PROF=1) at the 64 GiB C4 shape and at one
# rank's share of the real C4 (3/8, 2 M-block table)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
VSGPU_WALK_PROF=1 timeout -k 10 300 python bench.py --mode rsync --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/walkprof_c4.log 2>&1 || exit 1
grep "walk prof" gpurun_out/walkprof_c4.log | tail -1
VSGPU_WALK_PROF=1 timeout -k 10 300 python bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 2 --warmup 1 > gpurun_out/walkprof_share.log 2>&1 || exit 1
grep "walk prof" gpurun_out/walkprof_share.log | tail -1
