#!/bin/bash
# rocprofv3 passes (trace, FETCH, WRITE, SQ) over the C4 64 GiB-shape bench on the final code
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/profile.sh c4 --mode rsync --steps 2 --warmup 1 || exit $?
mkdir -p gpurun_out/profile_c4
python3 tools/summarize_prof.py gpurun_out/prof_c4 --out gpurun_out/profile_c4 || exit 1
cp gpurun_out/prof_c4/trace/trace_kernel_stats.csv gpurun_out/prof_c4/steps.log gpurun_out/profile_c4/
rm -rf gpurun_out/prof_c4
