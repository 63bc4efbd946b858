#!/bin/bash
# C2 bench A/B of the fingerprint variants (VSGPU_FP_FAST=0 generic, 1 fast, 2 address-only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # run <tag> <env> <args>
  timeout -k 10 300 env $2 python bench.py --no-cpu-baseline $3 > gpurun_out/ab_$1.log 2>&1 || { tail -20 gpurun_out/ab_$1.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ab_$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['stages_ms_per_step'], d['single_volume']['stages_ms']['fingerprint'], d.get('pipeline_valu_frac'))"
}
for v in "$@"; do run fp$v VSGPU_FP_FAST=$v "--hash-slice 512"; done
