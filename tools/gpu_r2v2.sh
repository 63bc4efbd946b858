#!/bin/bash
# rsync GPU tests, then the C4 line and one rank's share of the real C4 with
# the capped blocked filter (2^25 bits)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rsync.py tests/test_native_abi.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rsync_tests.log 2>&1 || { tail -30 gpurun_out/rsync_tests.log; exit 1; }
tail -2 gpurun_out/rsync_tests.log
timeout -k 10 300 python bench.py --mode rsync --steps 3 --warmup 1 > gpurun_out/bench_c4.log 2>&1 || { tail -20 gpurun_out/bench_c4.log; exit 1; }
tail -1 gpurun_out/bench_c4.log | cut -c1-700
timeout -k 10 300 python bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 > gpurun_out/bench_c4_share.log 2>&1 || { tail -20 gpurun_out/bench_c4_share.log; exit 1; }
tail -1 gpurun_out/bench_c4_share.log | cut -c1-1200
