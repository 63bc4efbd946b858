#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; REPO=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python bench.py --mode host --steps 2 --warmup 1 > gpurun_out/bench_host.log 2>&1
rc=$?; tail -1 gpurun_out/bench_host.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['frac_of_h2d'], d['stream_stats'])"; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r2g.sh
python3 - gpurun_out/profile_host/host_kernel_trace.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
t0 = int(rows[0]['Start_Timestamp'])
for r in rows:
    n = r['Kernel_Name']
    if 'sha_slice' in n or 'fp_kernel' in n:
        a, b = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if 700e6 < a - t0 < 800e6:
            print('%-10s start %.3f end %.3f grid %d' % ('slice' if 'sha' in n else 'fp', (a-t0)/1e6, (b-t0)/1e6, int(r['Grid_Size_X'])//int(r['Workgroup_Size_X'])))
PY
