#!/bin/bash
# streaming + file-sum iteration: CDC GPU tests, rsync file-sum tests, host-fed bench, C4 bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cdc.py tests/test_gpu_rsync.py -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?; tail -3 gpurun_out/gputests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --mode host --steps 2 --warmup 1 > gpurun_out/bench_host.log 2>&1
rc=$?; tail -1 gpurun_out/bench_host.log | cut -c1-1500; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --mode rsync --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1
rc=$?; tail -1 gpurun_out/bench_c4.log | cut -c1-300; exit $rc
