#!/bin/bash
# 4-lane signature kernel: rsync GPU tests + C4 bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rsync.py tests/test_native_abi.py -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/rs_tests.log 2>&1
rc=$?; tail -2 gpurun_out/rs_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode rsync --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1
rc=$?; echo "c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.loads(open('gpurun_out/bench_c4.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernels_ms_per_step'], d['signatures_GBps'])"
