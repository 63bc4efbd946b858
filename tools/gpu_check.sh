#!/bin/bash
# One GPU session: each GPU step under its own time limit; stop at the first
# fault / abort / timeout (exit >= 124); plain test failures (1) continue.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    smoke) step smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step gputests 1500 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread ;;
    testsk) step gputests 1500 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread ;;
    bench_small) step bench_small 600 python bench.py --steps 2 --warmup 1 --per-gpu-gib 8 --no-cpu-baseline ;;
    bench) step bench 900 python bench.py ;;
  esac
done
