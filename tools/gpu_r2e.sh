#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; REPO=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rsync.py -v -m gpu -x -k file_sum --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?; tail -2 gpurun_out/gputests.log; [ $rc -ne 0 ] && exit $rc
OUT=$REPO/gpurun_out/prof_host; mkdir -p $OUT; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o trace --output-format csv -- python3 $REPO/bench.py --mode host --per-gpu-gib 16 --steps 1 --warmup 1) > $OUT/trace.log 2>&1
echo "host trace rc=$?"
F=$(find $OUT/trace -name "*kernel_trace.csv" | head -1); echo "csv: $F"
python3 tools/trace_stream.py $F > gpurun_out/host_timeline.txt 2>&1; head -50 gpurun_out/host_timeline.txt
rm -rf $OUT/trace
timeout -k 10 300 python bench.py --mode rsync --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1
rc=$?; tail -1 gpurun_out/bench_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['file_sum'])"; exit $rc
