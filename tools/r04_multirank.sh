#!/bin/bash
# N-rank rehearsals on one GPU (VSGPU_BENCH_SHARED_GPU=1: every rank on
# cuda:0, collectives over gloo): the CDC byte-range shards at 2 and 4 ranks
# and the rsync walk + R7 relay at 4 ranks, each checking its gathered output
# against the full-size goldens.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export VSGPU_BENCH_SHARED_GPU=1
bash tools/gpu.sh bench cdc2 --gpus 2 --per-gpu-gib 4 --steps 3 --warmup 1 &&
bash tools/gpu.sh bench cdc4 --gpus 4 --per-gpu-gib 2 --steps 3 --warmup 1 &&
bash tools/gpu.sh bench c4relay4 --mode rsync --gpus 4 --per-gpu-gib 4 --steps 2 --warmup 1
