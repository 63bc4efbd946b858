#!/bin/bash
# rsync GPU tests + C4 bench after the device-side match collection, then the
# 2-rank device-path rehearsal on one GPU (gloo collectives) for C2 and C4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rsync.py tests/test_native_abi.py -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/rs_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rs_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode rsync --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1
rc=$?; echo "c4 rc=$rc"; tail -1 gpurun_out/bench_c4.log | cut -c1-1500; [ $rc -eq 0 ] || exit $rc
export VSGPU_BENCH_SHARED_GPU=1
timeout -k 10 300 python bench.py --gpus 2 --per-gpu-gib 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3_shared.log 2>&1
rc=$?; echo "c3 shared rc=$rc"; tail -1 gpurun_out/bench_c3_shared.log | cut -c1-800; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 2 --mode rsync --per-gpu-gib 4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4_shared.log 2>&1
rc=$?; echo "c4 shared rc=$rc"; tail -1 gpurun_out/bench_c4_shared.log | cut -c1-800; exit $rc
