#!/bin/bash
# A/B of the walk's filters: LDS prefilter on/off (VSGPU_WALK_LBITS=0) and
# blocked-filter bits per key (VSGPU_RS_FBITS_ADD), at the 64 GiB C4 shape
# and at one rank's share of the real C4 (2 M-block table)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/ab
run() {  # run <tag> <env...>
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --mode rsync --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab/c4_$tag.log 2>&1 || return 1
  env "$@" timeout -k 10 200 python bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 > gpurun_out/ab/share_$tag.log 2>&1 || return 1
  python3 - "$tag" gpurun_out/ab/c4_$tag.log gpurun_out/ab/share_$tag.log <<'PY'
import json, sys
out = [sys.argv[1]]
for f in sys.argv[2:]:
    j = json.loads(open(f).read().strip().splitlines()[-1])
    out.append(f"{j['value']:.1f} GB/s walk {j['kernels_ms_per_step']['walk_spec']:.2f} ms "
               f"fa {j['match_stats']['false_alarms']} m {j['config']['matches']}")
print(" | ".join(out), flush=True)
PY
}
true
true
VSGPU_LIB=$PWD/volsync_amd/lib_r8/libvsgpu.so timeout -k 10 600 python -u -m pytest tests/test_gpu_rsync.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/rsync_tests_r8.log 2>&1 || { tail -30 gpurun_out/ab/rsync_tests_r8.log; exit 1; }
tail -1 gpurun_out/ab/rsync_tests_r8.log
run base X=1 || exit 1
run t512 VSGPU_LIB=$PWD/volsync_amd/lib_t512/libvsgpu.so || exit 1
run r8 VSGPU_LIB=$PWD/volsync_amd/lib_r8/libvsgpu.so || exit 1
run base2 X=1 || exit 1
run r8b VSGPU_LIB=$PWD/volsync_amd/lib_r8/libvsgpu.so || exit 1
