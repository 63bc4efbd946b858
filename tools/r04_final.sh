#!/bin/bash
# Round-4 closing run on one box: the whole -m gpu suite, smoke(), the bench
# lines (tools/r04_benches.sh) and all of C3 rank by rank (tools/c3_ranks.sh).
# Profiles: tools/r04_profs.sh.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
bash tools/gpu.sh tests &&
bash tools/gpu.sh smoke &&
bash tools/r04_benches.sh &&
bash tools/c3_ranks.sh
