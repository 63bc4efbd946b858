#!/bin/bash
# Segment length A/B with the shipped walk (VS_OPT_WALK_SEGMENT_BLOCKS 16, 24,
# 32 = default, 48) at one rank of the real C4 and the 64 GiB shape.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
S="--mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum"
C="--mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline"
for r in 0 1; do
  for sb in ${SEGS:-16 24 32 48}; do
    bash tools/gpu.sh bench seg_share_${sb}_r$r $S --walk-opt walk_segment_blocks=$sb || exit $?
    bash tools/gpu.sh bench seg_c4_${sb}_r$r $C --walk-opt walk_segment_blocks=$sb || exit $?
  done
done
python3 tools/ab_table.py gpurun_out/bench_seg_*.log | tee gpurun_out/seg_table.txt
