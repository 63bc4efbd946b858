#!/bin/bash
# seal: GPU tests on both paths, then fused vs separate bench; then the walk
# workgroup A/B (tools/gpu_r2n.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_seal.py -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/seal_tests.log 2>&1
rc=$?; tail -3 gpurun_out/seal_tests.log; [ $rc -eq 0 ] || exit $rc
for f in 1 0; do
  VSGPU_SEAL_FUSED=$f timeout -k 10 300 python bench.py --mode seal --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/seal_f$f.log 2>&1
  rc=$?; echo "seal fused=$f rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/seal_f$f.log; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/seal_f$f.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernels'])"
done
bash tools/gpu_r2n.sh
