#!/bin/bash
# The 2^24-bit blocked filter at the real table: the rsync GPU tests, the
# share and 64 GiB lines, and the share line's profile.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
bash tools/gpu.sh tests tests/test_gpu_rsync.py tests/test_gpu_rsync_stream.py tests/test_native_abi.py -x &&
bash tools/gpu.sh bench c4share_nofs --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum &&
bash tools/gpu.sh bench c4share6 --mode rsync --share 3/8 --per-gpu-gib 32 --steps 6 --warmup 1 &&
bash tools/gpu.sh bench c4_nofs --mode rsync --steps 5 --warmup 1 --no-file-sum --no-cpu-baseline &&
bash tools/gpu.sh prof r04_c4share_final rs_walk --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum
