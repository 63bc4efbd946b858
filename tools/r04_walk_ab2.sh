#!/bin/bash
# Wide flushes through the LDS ring against four-window flushes: exactness
# (the walk tests) then the share and 64 GiB lines, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
S="--mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum"
C="--mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline"
bash tools/gpu.sh tests tests/test_gpu_rsync.py -x -k "walk or c4 or stitch or shard or golden" &&
bash tools/gpu.sh bench ab2_share_wide $S &&
bash tools/gpu.sh bench ab2_share_q4 $S --walk-opt walk_flush_windows=4 &&
bash tools/gpu.sh bench ab2_c4_wide $C --walk-opt walk_flush_windows=16 &&
bash tools/gpu.sh bench ab2_c4_q4 $C --walk-opt walk_flush_windows=4 &&
bash tools/gpu.sh bench ab2_share_wide_nopred $S --walk-opt walk_flush_predict=0 &&
bash tools/gpu.sh bench ab2_c4_q4_nopred $C --walk-opt walk_flush_windows=4,walk_flush_predict=0 &&
bash tools/gpu.sh bench ab2_share_q4_nopred $S --walk-opt walk_flush_windows=4,walk_flush_predict=0 &&
bash tools/gpu.sh bench ab2_share_wide_r2 $S || exit $?
python3 tools/ab_table.py gpurun_out/bench_ab2_*.log | tee gpurun_out/ab2_walk_table.txt
