#!/bin/bash
# Closing run of the final walk (48-block segments, 2^24-bit filter, 4 KiB
# wide-flush lookahead): the whole -m gpu suite, smoke, the rsync lines with
# and without R7, and the walk profiles.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
bash tools/gpu.sh tests &&
bash tools/gpu.sh smoke &&
bash tools/gpu.sh bench c4share_nofs --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum &&
bash tools/gpu.sh bench c4_nofs --mode rsync --steps 5 --warmup 1 --no-file-sum --no-cpu-baseline &&
bash tools/gpu.sh bench c4share6 --mode rsync --share 3/8 --per-gpu-gib 32 --steps 6 --warmup 1 &&
bash tools/gpu.sh bench c4 --mode rsync --steps 5 --warmup 1 &&
bash tools/gpu.sh bench rsynchost --mode rsync-host --steps 2 --warmup 1 &&
bash tools/gpu.sh bench c2 --steps 10 --warmup 2 &&
bash tools/gpu.sh prof r04_c4share_final rs_walk --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum &&
bash tools/gpu.sh prof r04_c4_final rs_walk --mode rsync --steps 3 --warmup 1 --no-file-sum
