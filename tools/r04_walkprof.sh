#!/bin/bash
# Walk phase profiles (VS_WALK_PROF build, tools/build_variant.sh walkprof
# -DVS_WALK_PROF=1) of wide and four-window flushes at one rank of the real C4
# and the 64 GiB shape, then the FETCH/WRITE/SQ passes of the share line for
# both.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
S="--share 3/8 --per-gpu-gib 32"
for v in "share_wide:$S" "share_q4:$S --walk-opt walk_flush_windows=4" "c4_wide:" "c4_q4:--walk-opt walk_flush_windows=4"; do
  tag=${v%%:*}; args=${v#*:}
  bash tools/c4_walkprof.sh $args > gpurun_out/walkprof_$tag.txt 2>&1 || exit $?
  cp gpurun_out/bench_walkprof.log gpurun_out/bench_walkprof_$tag.log
done
P="--mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum"
bash tools/gpu.sh prof r04_share_wide rs_walk $P &&
bash tools/gpu.sh prof r04_share_q4 rs_walk $P --walk-opt walk_flush_windows=4
