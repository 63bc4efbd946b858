#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --per-gpu-gib 128 --no-cpu-baseline > gpurun_out/bench_c2_128_k10.log 2>&1
rc=$?; echo "128 GiB k10 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.loads(open('gpurun_out/bench_c2_128_k10.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['stages_ms_per_step'], d['sha_slices'], d['single_volume']['ms'])"
