#!/bin/bash
# unaligned SHA segment loads: CDC / SHA GPU tests, C2 and C5 benches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_cdc.py tests/test_native_abi.py -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/cdc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/cdc_tests.log; [ $rc -eq 0 ] || exit $rc
for m in "c2 --no-cpu-baseline" "c5 --mode smallfiles --no-cpu-baseline"; do
  set -- $m; name=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/u_$name.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -3 gpurun_out/u_$name.log; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/u_$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'], d.get('stages_ms_per_step'), d.get('single_volume', {}).get('ms'))"
done
