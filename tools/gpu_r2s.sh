#!/bin/bash
# C3's per-GPU share (128 GiB resident) on one GPU, and the 2-rank rehearsal
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --per-gpu-gib 128 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c2_128.log 2>&1
rc=$?; echo "128 GiB rc=$rc"; tail -1 gpurun_out/bench_c2_128.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc
VSGPU_BENCH_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --per-gpu-gib 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3_shared.log 2>&1
rc=$?; echo "shared rc=$rc"; tail -1 gpurun_out/bench_c3_shared.log | cut -c1-500; exit $rc
