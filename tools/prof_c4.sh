#!/bin/bash
# rocprofv3 over the C4-shape rsync bench: kernel trace + stats, then one PMC
# pass per counter group (never combined with runtime/sys traces), summarised
# with tools/summarize_prof.py.  Usage: tools/prof_c4.sh <tag> [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; REPO=$(pwd); TAG=$1; shift
OUT=$REPO/gpurun_out/prof_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
ARGS="--mode rsync --no-cpu-baseline --steps 2 --warmup 1 $@"
run() {  # run <name> <timeout> <rocprof args...>
  local name=$1 t=$2; shift 2
  echo "=== $name" >> $OUT/steps.log
  (cd /tmp && timeout -k 10 $t rocprofv3 "$@" --kernel-include-regex "rs_|synth" -d $OUT/$name -o $name --output-format csv -- python3 $REPO/bench.py $ARGS) > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run trace 300 --kernel-trace --stats
run pmc_fetch 300 --kernel-trace --pmc FETCH_SIZE
run pmc_write 300 --kernel-trace --pmc WRITE_SIZE
run pmc_tcc 300 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum
run pmc_sq 300 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
run pmc_ta 300 --kernel-trace --pmc TA_BUSY_avr TA_BUSY_max
python3 tools/summarize_prof.py $OUT --out gpurun_out/profile_$TAG > $OUT/summary.log 2>&1
cp $OUT/trace.log gpurun_out/profile_$TAG/bench_under_rocprof.log
rm -rf $OUT/pmc_* $OUT/trace
echo done >> $OUT/steps.log
