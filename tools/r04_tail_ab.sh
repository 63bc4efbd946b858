#!/bin/bash
# Tail segments A/B (VS_OPT_WALK_TAIL_PCT 0 = default, 20, 40): the walk
# tests with the option, then both C4 lines, two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
S="--mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum"
C="--mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline"
[ -n "$NOTEST" ] || bash tools/gpu.sh tests tests/test_gpu_rsync.py -x -k "segment_lengths or stitch or real_density" || exit $?
for r in 0 1; do
  for tp in ${TAILS:-0 20 40}; do
    bash tools/gpu.sh bench tail_share_${tp}_r$r $S --walk-opt walk_tail_pct=$tp || exit $?
    bash tools/gpu.sh bench tail_c4_${tp}_r$r $C --walk-opt walk_tail_pct=$tp || exit $?
  done
done
python3 tools/ab_table.py gpurun_out/bench_tail_*.log | tee gpurun_out/tail_table.txt
