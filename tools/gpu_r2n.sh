#!/bin/bash
# A/B of the speculative walk's workgroup size (768 vs 1024 threads) on C4,
# with the per-wave phase profile of each, and the walk tests at 1024.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for wg in 768 1024; do
  VSGPU_WALK_WG=$wg timeout -k 10 300 python bench.py --mode rsync --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c4_wg$wg.log 2>&1
  rc=$?; echo "wg $wg rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/c4_wg$wg.log; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c4_wg$wg.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernels_ms_per_step'])"
  VSGPU_WALK_PROF=1 VSGPU_WALK_WG=$wg timeout -k 10 300 python bench.py --mode rsync --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/c4_prof_wg$wg.log 2>&1
  rc=$?; grep "walk prof" gpurun_out/c4_prof_wg$wg.log | tail -1; [ $rc -eq 0 ] || exit $rc
done
VSGPU_WALK_WG=1024 timeout -k 10 600 python -u -m pytest tests/test_gpu_rsync.py -v -m gpu -x -k "walk or c4 or golden or oracle" --timeout 120 --timeout-method thread > gpurun_out/rs_tests_1024.log 2>&1
rc=$?; tail -2 gpurun_out/rs_tests_1024.log; exit $rc
