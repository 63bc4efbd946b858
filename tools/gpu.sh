#!/bin/bash
# The one lease script for gpurun.  Each invocation runs ONE GPU step under its
# own time limit and exits with its status; chain steps with && so the call
# stops at the first failure, fault or timeout:
#   gpurun -- 'bash tools/gpu.sh tests && bash tools/gpu.sh bench c2'
#
#   smoke                          __graft_entry__.smoke()
#   tests [pytest args...]         the -m gpu suite (default: all of tests/, -x)
#   bench <tag> [bench.py args...] one bench line -> gpurun_out/bench_<tag>.log
#   prof <tag> <kernel-regex> [bench.py args...]
#                                  rocprofv3 kernel trace + stats, then one PMC
#                                  pass per counter group (never combined with
#                                  runtime traces) -> gpurun_out/profile_<tag>/
#   py <script> [args...]          a python script (probes, A/B drivers)
# GPU_STEP_TIMEOUT overrides a step's limit (seconds).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
cmd=$1
shift
step() {  # step <log> <timeout> <cmd...>
  local log=$1 t=${GPU_STEP_TIMEOUT:-$2}
  shift 2
  echo "=== $log: $*" >> gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$log.log" 2>&1
  local rc=$?
  echo "=== $log rc=$rc" | tee -a gpurun_out/steps.log
  tail -n 4 "gpurun_out/$log.log" | cut -c1-400
  return $rc
}
case $cmd in
  smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
  tests)
    [ $# -eq 0 ] && set -- tests -x
    step gputests 1100 python -u -m pytest "$@" -v -m gpu --timeout 120 --timeout-method thread ;;
  bench)
    tag=$1
    shift
    step "bench_$tag" 600 python bench.py "$@" ;;
  prof)
    tag=$1 kre=$2
    shift 2
    repo=$PWD out=$PWD/gpurun_out/prof_$tag
    mkdir -p "$out"
    export TMPDIR=/tmp
    pass() {  # pass <name> <rocprofv3 args...> -- <bench args...>
      local name=$1 ra=()
      shift
      while [ "$1" != "--" ]; do ra+=("$1"); shift; done
      shift
      (cd /tmp && timeout -k 10 "${GPU_STEP_TIMEOUT:-400}" rocprofv3 "${ra[@]}" \
         --kernel-include-regex "$kre" -d "$out/$name" -o "$name" --output-format csv \
         -- python3 "$repo/bench.py" --no-cpu-baseline "$@") > "$out/$name.log" 2>&1
      local rc=$?
      echo "=== prof_$tag $name rc=$rc" | tee -a gpurun_out/steps.log
      return $rc
    }
    pass trace --kernel-trace --stats -- "$@" &&
    pass pmc_fetch --kernel-trace --pmc FETCH_SIZE -- "$@" &&
    pass pmc_write --kernel-trace --pmc WRITE_SIZE -- "$@" &&
    pass pmc_sq --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES \
      SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -- "$@" &&
    pass pmc_lds --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS \
      SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -- "$@" || exit $?
    python3 tools/summarize_prof.py "$out" --out "gpurun_out/profile_$tag" > "$out/summary.log" 2>&1 || exit 1
    cp "$out/trace.log" "gpurun_out/profile_$tag/bench_under_rocprof.log"
    rm -rf "$out"/pmc_* "$out"/trace ;;
  py)
    script=$1
    step "py_$(basename "$script" .py)" 600 python -u "$@" ;;
  *) echo "usage: tools/gpu.sh smoke|tests|bench|prof|py ..." >&2; exit 2 ;;
esac
