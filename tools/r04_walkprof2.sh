#!/bin/bash
# Walk phase profiles of the shipped walk (VS_WALK_PROF build) at one rank of
# the real C4 and at the 64 GiB shape.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
bash tools/c4_walkprof.sh --share 3/8 --per-gpu-gib 32 > gpurun_out/walkprof2_share.txt 2>&1 &&
bash tools/c4_walkprof.sh > gpurun_out/walkprof2_c4.txt 2>&1
