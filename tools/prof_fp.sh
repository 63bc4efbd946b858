#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; REPO=$(pwd); TAG=$1; shift
OUT=$REPO/gpurun_out/prof_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 $REPO/tools/fp_only.py --gib 16 --reps 2) > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc" >> $OUT/steps.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi; }
run trace --kernel-trace --stats
run fetch --kernel-trace --pmc FETCH_SIZE
run sq --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD
run sq2 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE
run tcc --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum
echo done >> $OUT/steps.log
