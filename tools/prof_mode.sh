#!/bin/bash
# rocprofv3 over one bench mode: kernel trace + stats, then one PMC pass per
# counter group (never combined with runtime/sys traces), summarised with
# tools/summarize_prof.py.
# Usage: tools/prof_mode.sh <tag> <kernel-regex> [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; REPO=$(pwd); TAG=$1; KRE=$2; shift 2
OUT=$REPO/gpurun_out/prof_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
ARGS="--no-cpu-baseline --steps 2 --warmup 1 $@"
run() {  # run <name> <timeout> <rocprof args...>
  local name=$1 t=$2; shift 2
  echo "=== $name" >> $OUT/steps.log
  (cd /tmp && timeout -k 10 $t rocprofv3 "$@" --kernel-include-regex "$KRE" -d $OUT/$name -o $name --output-format csv -- python3 $REPO/bench.py $ARGS) > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run trace 300 --kernel-trace --stats
run pmc_fetch 300 --kernel-trace --pmc FETCH_SIZE
run pmc_write 300 --kernel-trace --pmc WRITE_SIZE
run pmc_sq 300 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
run pmc_lds 300 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
python3 tools/summarize_prof.py $OUT --out gpurun_out/profile_$TAG > $OUT/summary.log 2>&1
cp $OUT/trace.log gpurun_out/profile_$TAG/bench_under_rocprof.log
rm -rf $OUT/pmc_* $OUT/trace
echo done >> $OUT/steps.log
