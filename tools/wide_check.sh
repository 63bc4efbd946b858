#!/bin/bash
# wide-mode SHA-256: parity first, then C2 bench with the default threshold and with the mode off
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_cdc.py -v -m gpu -x --timeout 120 --timeout-method thread -k "wide" > gpurun_out/wide_tests.log 2>&1 || { tail -30 gpurun_out/wide_tests.log; exit 1; }
tail -3 gpurun_out/wide_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
for w in "${@:-0 0xffffffff}"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --hash-wide $w > gpurun_out/bench_w$w.log 2>&1 || { tail -20 gpurun_out/bench_w$w.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_w$w.log').read().strip().splitlines()[-1]); print('$w', d['value'], d['ms_per_step'], d['stages_ms_per_step'], d['sha_slices'], d['single_volume']['ms'])"
done
