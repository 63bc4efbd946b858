#!/bin/bash
# C2 co-residence A/B: fingerprint 512 threads + budgeted slices capped at 1 WG per CU
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in "768 5 512" "512 1 2048" "512 1 8192" "512 1 32768" "768 1 8192"; do
  set -- $cfg
  VSGPU_FP_WG=$1 VSGPU_SHA_SLICE_WGS=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --hash-slice $3 > gpurun_out/co_$1_$2_$3.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "cfg $cfg rc=$rc"; tail -3 gpurun_out/co_$1_$2_$3.log; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/co_$1_$2_$3.log').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'], d['stages_ms_per_step'], d['single_volume']['ms'])"
done
