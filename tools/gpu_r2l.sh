#!/bin/bash
# Round-2 profile evidence on the current code: rocprofv3 kernel trace + PMC
# passes for C2 (SHA-256 + fingerprint), C4 (device walk + signatures) and the
# seal stage, plus a C4 runtime timeline (kernels, HIP API, copies; no PMC).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; REPO=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/prof_mode.sh c2 "sha_|fp_kernel" || exit $?
bash tools/prof_mode.sh c4 "rs_" --mode rsync || exit $?
bash tools/prof_mode.sh seal "seal_" --mode seal || exit $?
OUT=$REPO/gpurun_out/prof_c4tl
mkdir -p $OUT
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace -d $OUT/tl -o tl --output-format csv -- python3 $REPO/bench.py --mode rsync --steps 2 --warmup 1 --no-cpu-baseline) > $OUT/tl.log 2>&1
echo "c4 timeline rc=$?"
python3 tools/c4_timeline.py $OUT/tl > gpurun_out/profile_c4/timeline.txt 2>&1
echo "timeline rc=$?"
rm -rf $OUT/tl
du -sh gpurun_out
