#!/bin/bash
# Walk A/B on one box (bench lines without R7, so the walk is the step):
# wide 16-window flushes (default) against four-window flushes, with and
# without the LDS prefilter, at one rank of the real C4 and at the 64 GiB
# shape.  Stops at the first failure; tools/ab_table.py tabulates the logs.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
S="--mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum"
C="--mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline"
bash tools/gpu.sh bench ab_share_wide $S &&
bash tools/gpu.sh bench ab_share_q4 $S --walk-opt walk_flush_windows=4 &&
bash tools/gpu.sh bench ab_share_wide_nopf $S --walk-opt walk_prefilter=0 &&
bash tools/gpu.sh bench ab_share_wide_span16k $S --walk-opt walk_flush_span=16384 &&
bash tools/gpu.sh bench ab_share_wide_span32k $S --walk-opt walk_flush_span=32768 &&
bash tools/gpu.sh bench ab_c4_wide $C &&
bash tools/gpu.sh bench ab_c4_q4 $C --walk-opt walk_flush_windows=4 &&
bash tools/gpu.sh bench ab_c4_wide_nopf $C --walk-opt walk_prefilter=0 &&
bash tools/gpu.sh bench ab_c4_wide_span32k $C --walk-opt walk_flush_span=32768 &&
bash tools/gpu.sh bench ab_share_wide2 $S || exit $?
python3 tools/ab_table.py gpurun_out/bench_ab_*.log | tee gpurun_out/ab_walk_table.txt
