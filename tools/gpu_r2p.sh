#!/bin/bash
# C2 timeline (kernel trace of the default bench) and the step-count sweep
cd "${GRAFT_REPO_ROOT:-/root/repo}"; REPO=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out/c2tl
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex "sha_slice|fp_kernel" -d $REPO/gpurun_out/c2tl/tr -o tr --output-format csv -- python3 $REPO/bench.py --no-cpu-baseline) > gpurun_out/c2tl/run.log 2>&1
echo "trace rc=$?"
f=$(find gpurun_out/c2tl/tr -name "*kernel_trace.csv" | head -1)
python3 tools/c2_timeline.py $f > gpurun_out/c2tl/timeline.txt; echo "timeline rc=$?"
rm -rf gpurun_out/c2tl/tr
tail -1 gpurun_out/c2tl/run.log | cut -c1-300
for k in 10 30; do
  timeout -k 10 300 python bench.py --steps $k --warmup 2 --no-cpu-baseline > gpurun_out/c2_k$k.log 2>&1
  rc=$?; echo "k=$k rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.loads(open('gpurun_out/c2_k$k.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['stages_ms_per_step'])"
done
