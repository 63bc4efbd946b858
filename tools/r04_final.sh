#!/bin/bash
# Round-4 closing run on one box: the whole -m gpu suite, smoke(), the bench
# lines (tools/r04_benches.sh), all of C3 rank by rank (tools/c3_ranks.sh),
# then rocprofv3 kernel traces + FETCH/WRITE/SQ/LDS passes of C2 and of one
# rank of the real C4.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
bash tools/gpu.sh tests &&
bash tools/gpu.sh smoke &&
bash tools/r04_benches.sh &&
bash tools/c3_ranks.sh &&
bash tools/gpu.sh prof r04_c2 '.*' --steps 5 --warmup 1 &&
bash tools/gpu.sh prof r04_c4share rs_walk --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum
