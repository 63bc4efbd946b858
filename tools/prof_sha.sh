#!/bin/bash
# Hash-engine profile: kernel trace + PMC passes (each its own run, never
# combined with runtime traces) over tools/sha_only.py.
# Usage: tools/prof_sha.sh <tag> [sha_only args...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
TAG=$1; shift
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="$@"
run() {  # run <name> <timeout> <rocprof args...>
  local name=$1 t=$2; shift 2
  echo "=== $name" >> $OUT/steps.log
  (cd /tmp && timeout -k 10 $t rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 $REPO/tools/sha_only.py $ARGS) > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
}
run trace 300 --kernel-trace --stats
run pmc_a 300 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run pmc_b 300 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum
run pmc_c 300 --kernel-trace --pmc FETCH_SIZE TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
echo done >> $OUT/steps.log
