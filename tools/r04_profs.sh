#!/bin/bash
# rocprofv3 kernel traces + FETCH/WRITE/SQ/LDS passes (tools/gpu.sh prof) of
# C2 and of one rank of the real C4, then the walk phase profiles and the
# VS_WIDE_MIN A/B (tools/r04_walkprof.sh).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
bash tools/gpu.sh prof r04_c2 '.*' --steps 5 --warmup 1 &&
bash tools/r04_walkprof.sh &&
bash tools/gpu.sh bench c4md5fs --mode rsync --csum md5 --per-gpu-gib 8 --steps 1 --warmup 0 --no-cpu-baseline
