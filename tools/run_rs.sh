#!/bin/bash
# rsync GPU tests + C4 bench line (each step under its own limit; stop on fault)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rsync.py -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?; tail -5 gpurun_out/gputests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --mode rsync --steps 3 --warmup 1 ${RS_ARGS} > gpurun_out/bench_rs.log 2>&1
rc=$?; tail -3 gpurun_out/bench_rs.log; exit $rc
