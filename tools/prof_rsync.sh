#!/bin/bash
# Kernel trace of the C4-shape rsync bench.  Usage: tools/prof_rsync.sh <tag> [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; REPO=$(pwd); TAG=$1; shift
OUT=$REPO/gpurun_out/prof_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "rs_|Radix|Onesweep|scan_|Histogram|synth" -d $OUT/trace -o trace --output-format csv -- python3 $REPO/bench.py --mode rsync --no-cpu-baseline "$@") > $OUT/trace.log 2>&1
echo "trace rc=$?" >> $OUT/steps.log
