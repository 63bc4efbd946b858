#!/bin/bash
# C4 bench (with the file checksum), C4 counter profile, kernel trace of the host-fed bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --mode rsync --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 || { tail -5 gpurun_out/bench_c4.log; exit 1; }
tail -1 gpurun_out/bench_c4.log | cut -c1-300
bash tools/prof_c4.sh c4b || exit $?
OUT=gpurun_out/prof_host; mkdir -p $OUT; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --mode host --per-gpu-gib 16 --steps 1 --warmup 1) > $OUT/trace.log 2>&1
echo "host trace rc=$?"
python3 tools/summarize_prof.py $OUT --out gpurun_out/profile_host > /dev/null 2>&1
cp $OUT/trace/trace_kernel_trace.csv gpurun_out/profile_host/ 2>/dev/null
cp $OUT/trace.log gpurun_out/profile_host/
rm -rf $OUT
