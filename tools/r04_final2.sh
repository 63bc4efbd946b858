#!/bin/bash
# Closing run for the final walk (48-block segments): the whole -m gpu suite,
# smoke(), the bench lines (with and without R7), the walk profiles.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
bash tools/gpu.sh tests &&
bash tools/gpu.sh smoke &&
bash tools/r04_benches.sh &&
bash tools/gpu.sh bench c4share_nofs --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum &&
bash tools/gpu.sh bench c4_nofs --mode rsync --steps 5 --warmup 1 --no-file-sum --no-cpu-baseline &&
bash tools/gpu.sh bench c4share6 --mode rsync --share 3/8 --per-gpu-gib 32 --steps 6 --warmup 1 &&
bash tools/gpu.sh prof r04_c4share_final rs_walk --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum &&
bash tools/gpu.sh prof r04_c4_final rs_walk --mode rsync --steps 3 --warmup 1 --no-file-sum
