#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 120 ./tools/valu/valu_peak > gpurun_out/valu_peak.json; echo "valu rc=$?"
timeout -k 10 600 python -u -m pytest tests/test_gpu_cdc.py tests/test_gpu_rsync.py -v -m gpu -x -k "blocks or verify or reconstruct or dedup or file_sum" --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?; tail -3 gpurun_out/gputests.log; exit $rc
