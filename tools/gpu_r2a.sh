#!/bin/bash
# round-2 iteration: GPU tests (cdc + rsync), walk phase profile, C4 and host-fed benches
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_cdc.py tests/test_gpu_rsync.py -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?; tail -3 gpurun_out/gputests.log; [ $rc -ne 0 ] && exit $rc
bash tools/c4_walkprof.sh || exit $?
timeout -k 10 300 python bench.py --mode host --steps 2 --warmup 1 > gpurun_out/bench_host.log 2>&1
rc=$?; tail -1 gpurun_out/bench_host.log; exit $rc
