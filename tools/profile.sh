#!/bin/bash
# rocprofv3 passes over a bench run (kernel trace + stats; PMC passes separate,
# never combined with runtime/sys traces).  Usage: tools/profile.sh <tag> [bench args...]
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
  (cd /tmp && timeout -k 10 $t rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 $REPO/bench.py $ARGS --no-cpu-baseline) > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
}
run trace 600 --kernel-trace --stats
run pmc_fetch 600 --kernel-trace --pmc FETCH_SIZE
run pmc_write 600 --kernel-trace --pmc WRITE_SIZE
run pmc_sq 600 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
echo done >> $OUT/steps.log
