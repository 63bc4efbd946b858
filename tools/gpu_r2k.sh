#!/bin/bash
# dedup at C5 size, then the bench modes the last call did not reach.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_cdc.py -v -m gpu -x -k "dedup" --timeout 120 --timeout-method thread > gpurun_out/dedup_tests.log 2>&1
rc=$?; tail -4 gpurun_out/dedup_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # run <name> <timeout> <bench args...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python bench.py "$@" > "gpurun_out/bench_$name.log" 2>&1
  local rc=$?
  echo "=== bench_$name rc=$rc"; tail -1 "gpurun_out/bench_$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
run c5 300 --mode smallfiles
run host 300 --mode host --steps 3 --warmup 1 --no-cpu-baseline
run seal 300 --mode seal --steps 5 --warmup 1
