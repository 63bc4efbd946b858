#!/bin/bash
# Round-end evidence, part 2: rocprofv3 kernel trace + PMC passes per mode.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/prof_mode.sh c2 "sha_|fp_kernel" || exit $?
bash tools/prof_mode.sh c4 "rs_" --mode rsync || exit $?
bash tools/prof_mode.sh seal "seal_" --mode seal || exit $?
du -sh gpurun_out
