#!/bin/bash
# Round-end evidence, part 1: smoke, the whole GPU suite, every bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -f gpurun_out/steps.log
bash tools/gpu_check.sh smoke tests || exit $?
grep -q "gputests rc=0" gpurun_out/steps.log || { echo "gpu tests failed"; exit 1; }
run() {  # run <name> <timeout> <bench args...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python bench.py "$@" > "gpurun_out/bench_$name.log" 2>&1
  local rc=$?
  echo "=== bench_$name rc=$rc"; tail -1 "gpurun_out/bench_$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
run c2 300
run c4 300 --mode rsync --steps 3 --warmup 1
run c5 300 --mode smallfiles
run host 300 --mode host --steps 3 --warmup 1 --no-cpu-baseline
run seal 300 --mode seal --steps 5 --warmup 1
