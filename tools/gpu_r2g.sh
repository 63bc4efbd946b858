#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; REPO=$(pwd); mkdir -p gpurun_out
OUT=$REPO/gpurun_out/prof_host; mkdir -p $OUT; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o trace --output-format csv -- python3 $REPO/bench.py --mode host --per-gpu-gib 16 --steps 1 --warmup 1) > $OUT/trace.log 2>&1
echo "host trace rc=$?"
F=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 tools/trace_stream.py $F > gpurun_out/host_timeline.txt 2>&1; head -12 gpurun_out/host_timeline.txt
python3 - "$F" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
seen = set()
for r in rows:
    n = r["Kernel_Name"].split("(")[0][-30:]
    if n in seen: continue
    seen.add(n)
    print(n, "grid", r["Grid_Size_X"], "wg", r["Workgroup_Size_X"], "vgpr", r["VGPR_Count"], "lds", r["LDS_Block_Size"])
PY
mkdir -p gpurun_out/profile_host; cp $F gpurun_out/profile_host/host_kernel_trace.csv; rm -rf $OUT/trace
