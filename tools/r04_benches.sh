#!/bin/bash
# Round-4 bench lines, one GPU step each (tools/gpu.sh), stopping at the first
# failure: C2 (golden_match), C4 shape with R7, one rank of the real C4, the
# host-fed rsync line, the 2-rank shared-GPU rehearsal with the R7 relay, and
# the MD5 mode (host walk).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
bash tools/gpu.sh bench c2 --steps 10 --warmup 2 &&
bash tools/gpu.sh bench c4 --mode rsync --steps 5 --warmup 1 --no-cpu-baseline &&
bash tools/gpu.sh bench c4share --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 &&
bash tools/gpu.sh bench rsynchost --mode rsync-host --steps 2 --warmup 1 &&
VSGPU_BENCH_SHARED_GPU=1 bash tools/gpu.sh bench c4relay2 --mode rsync --gpus 2 --per-gpu-gib 4 --steps 3 --warmup 1 &&
bash tools/gpu.sh bench c4md5 --mode rsync --csum md5 --steps 1 --warmup 0 --no-file-sum --no-cpu-baseline
