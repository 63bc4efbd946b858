#!/bin/bash
# Per-wave walk phase profile (s_memtime phases).  The phase
# counters are compiled only into a profiling build (the build flag
# VS_WALK_PROF; no environment variable turns them on), made here first:
#   tools/build_variant.sh walkprof -DVS_WALK_PROF=1
# then on the box: bash tools/c4_walkprof.sh [bench.py args...]; VSGPU_LIB
# (read by volsync_amd/_lib.py, not by the library) selects that build.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
lib=$PWD/volsync_amd/lib/var/walkprof/libvsgpu.so
[ -f "$lib" ] || { echo "build $lib first (tools/build_variant.sh walkprof -DVS_WALK_PROF=1)" >&2; exit 2; }
VSGPU_LIB=$lib timeout -k 10 300 python bench.py --mode rsync --steps 1 --warmup 1 \
  --no-cpu-baseline --no-file-sum "$@" > gpurun_out/bench_walkprof.log 2>&1
rc=$?
grep "walk prof" gpurun_out/bench_walkprof.log | tail -1 | tr ';' '\n'
exit $rc
