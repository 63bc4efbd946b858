#!/bin/bash
# fused seal without spills: tests, bench, WRITE_SIZE / FETCH_SIZE passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"; REPO=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_seal.py -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/seal_tests.log 2>&1
rc=$?; tail -2 gpurun_out/seal_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode seal --steps 5 --warmup 1 > gpurun_out/bench_seal.log 2>&1
rc=$?; echo "seal rc=$rc"; tail -1 gpurun_out/bench_seal.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
bash tools/prof_mode.sh seal "seal_" --mode seal || exit $?
grep "seal_ctr" gpurun_out/profile_seal/summary.md | cut -c1-120
python3 -c "import json; s=json.load(open('gpurun_out/profile_seal/summary.json')); e=[v for k,v in s.items() if k.startswith('seal_ctr')][0]; print(e['avg_us'], e['hbm_read_bytes_per_dispatch'], e['hbm_write_bytes_per_dispatch'])"
