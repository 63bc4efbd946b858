cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
VSGPU_WALK_PROF=1 timeout -k 10 300 python bench.py --mode rsync --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1
rc=$?; grep "walk prof" gpurun_out/bench_prof.log | tail -2; tail -1 gpurun_out/bench_prof.log | cut -c1-400; exit $rc
