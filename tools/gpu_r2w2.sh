#!/bin/bash
# fingerprint at 16 waves per CU (VS_FP_THREADS=1024, 128 VGPRs) vs 12 (768):
# C2 line twice each, alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/fpw
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/fpw/c2_768_$i.log 2>&1 || exit 1
  VSGPU_LIB=$PWD/volsync_amd/lib_t1024/libvsgpu.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/fpw/c2_1024_$i.log 2>&1 || exit 1
  for t in 768 1024; do
    python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], j['value'], j['stages_ms_per_step'], j['single_volume']['ms'], j['config']['chunks'])" gpurun_out/fpw/c2_${t}_$i.log $t
  done
done
