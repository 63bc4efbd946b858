#!/bin/bash
# Round-end evidence in one GPU call: tools/final_check.sh (tests, smoke, C2/C5/C4
# bench lines, rocprofv3 passes over C2) plus a kernel trace of the C4 rsync bench,
# summarised on the box into gpurun_out/profile/ (large per-dispatch CSVs pruned so
# the copy-back stays under gpurun's 64 MiB).  Usage: tools/round_end.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/final_check.sh || exit $?
bash tools/prof_rsync.sh c4 --steps 3 --warmup 1 || exit $?
grep -q "trace rc=0" gpurun_out/prof_c4/steps.log || exit 1
P=gpurun_out/profile
mkdir -p $P/c4
python3 tools/summarize_prof.py gpurun_out/prof_final --out $P || exit 1
python3 tools/trace_timed.py gpurun_out/prof_final/trace/trace_kernel_trace.csv > $P/timed_region.txt || exit 1
cp gpurun_out/prof_final/trace/trace_kernel_stats.csv gpurun_out/prof_final/trace/trace_kernel_trace.csv $P/
cp gpurun_out/prof_c4/trace/trace_kernel_stats.csv $P/c4/
cp gpurun_out/bench.log $P/bench_c2.log
cp gpurun_out/bench_c5.log gpurun_out/bench_c4.log $P/
cp gpurun_out/prof_final/trace.log $P/bench_c2_under_rocprof.log
cp gpurun_out/prof_c4/trace.log $P/c4/bench_c4_under_rocprof.log
rm -rf gpurun_out/prof_final gpurun_out/prof_c4
du -sh gpurun_out
