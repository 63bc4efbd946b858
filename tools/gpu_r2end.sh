#!/bin/bash
# Round-2 end evidence on the final code: tools/final_check.sh (GPU tests,
# smoke, C2 / C5 / C4 / C4-share lines, rocprofv3 passes over C2) plus
# rocprofv3 passes over one rank's share of the real C4; summaries into
# gpurun_out/profile/, large per-dispatch CSVs pruned.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/final_check.sh || exit $?
bash tools/profile.sh share --mode rsync --share 3/8 --per-gpu-gib 32 --steps 2 --warmup 1 || exit $?
P=gpurun_out/profile
mkdir -p $P/c2 $P/c4_share
python3 tools/summarize_prof.py gpurun_out/prof_final --out $P/c2 || exit 1
python3 tools/summarize_prof.py gpurun_out/prof_share --out $P/c4_share || exit 1
python3 tools/trace_timed.py gpurun_out/prof_final/trace/trace_kernel_trace.csv > $P/c2/timed_region.txt || true
cp gpurun_out/prof_final/trace/trace_kernel_stats.csv $P/c2/
cp gpurun_out/prof_share/trace/trace_kernel_stats.csv $P/c4_share/
cp gpurun_out/prof_final/steps.log $P/c2/; cp gpurun_out/prof_share/steps.log $P/c4_share/
cp gpurun_out/bench.log $P/bench_c2.log
cp gpurun_out/bench_c5.log gpurun_out/bench_c4.log gpurun_out/bench_c4_share.log gpurun_out/gputests.log gpurun_out/smoke.log $P/
rm -rf gpurun_out/prof_final gpurun_out/prof_share
du -sh gpurun_out
