#!/bin/bash
# SHA kernel tests after the tile-broadcast change; C2 A/B: fingerprint
# workgroup 768 / 512 x hash slice budget 512 / 4096 / 16384
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cdc.py -v -m gpu -x -k "sha or golden or oracle" --timeout 120 --timeout-method thread > gpurun_out/cdc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/cdc_tests.log; [ $rc -eq 0 ] || exit $rc
for wg in 768 512; do for sl in 512 4096 16384; do
  VSGPU_FP_WG=$wg timeout -k 10 300 python bench.py --no-cpu-baseline --hash-slice $sl > gpurun_out/ab_${wg}_$sl.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "wg $wg slice $sl rc=$rc"; tail -3 gpurun_out/ab_${wg}_$sl.log; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_${wg}_$sl.log').read().strip().splitlines()[-1]); print('$wg', '$sl', d['value'], d['ms_per_step'], d['stages_ms_per_step'], d['single_volume']['ms'])"
done; done
