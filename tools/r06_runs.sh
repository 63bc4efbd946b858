#!/bin/bash
# Round 6's GPU runs, one subcommand each (through gpurun; every GPU step has
# its own time limit in tools/gpu.sh or here, and the chain stops at the first
# failure).
#   first   host CPU facts, the CDC GPU tests, the single-pass drain A/B
#           (latency-mode producer priority: qpp0 = -DVS_SHA_QUAD_PPRIO=0),
#           C2 at the driver's 20/5 (single pass, --distinct 3, nproc
#           baselines), C3 rank 3 at 20/5
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
var() { echo "volsync_amd/lib/var/$1/libvsgpu.so"; }
ab() {  # ab <log> <rounds> <libs> <script args...>
  local log=$1 rounds=$2 libs=$3
  shift 3
  timeout -k 10 900 python3 -u tools/ab.py --rounds "$rounds" --libs "$libs" -- "$@" \
    > "gpurun_out/$log.log" 2>&1
  local rc=$?
  echo "=== $log rc=$rc"; tail -n 8 "gpurun_out/$log.log"
  return $rc
}
hostinfo() {
  { echo "nproc $(nproc)"; cat /sys/fs/cgroup/cpu.max 2>&1; grep -m1 "model name" /proc/cpuinfo
    python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; } > gpurun_out/hostinfo.txt
  cat gpurun_out/hostinfo.txt
}
trace() {  # trace <tag> <bench args...>: kernel trace + stats only (no counters)
  local tag=$1 out=$PWD/gpurun_out/trace_$1 repo=$PWD
  shift
  mkdir -p "$out"
  (cd /tmp && TMPDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$out/raw" \
     -o run --output-format csv -- python3 "$repo/bench.py" "$@") > "$out/bench.log" 2>&1
  local rc=$?
  echo "=== trace_$tag rc=$rc"; tail -n 2 "$out/bench.log" | cut -c1-300
  [ $rc -eq 0 ] || return $rc
  find "$out/raw" -name '*kernel_stats.csv' -exec cp {} "$out/kernel_stats.csv" \;
  find "$out/raw" -name '*kernel_trace.csv' -exec cp {} "$out/kernel_trace.csv" \;
  rm -rf "$out/raw"
}
case $1 in
  validate)   # the whole GPU suite, smoke, every bench line
    bash tools/gpu.sh tests && bash tools/gpu.sh smoke && bash "$0" benches ;;
  benches)
    bash tools/gpu.sh bench c2 --gpus 1 --steps 20 --warmup 5 &&
    bash tools/gpu.sh bench c3r3 --share 3/8 --steps 20 --warmup 5 --no-cpu-baseline &&
    bash tools/gpu.sh bench c5 --mode smallfiles --steps 5 --warmup 1 &&
    bash tools/gpu.sh bench c4 --mode rsync --steps 20 --warmup 2 --no-cpu-baseline &&
    bash tools/gpu.sh bench c4share --mode rsync --share 3/8 --per-gpu-gib 32 --steps 10 --warmup 1 &&
    bash tools/gpu.sh bench c4share_nofs --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum &&
    bash tools/gpu.sh bench seal --mode seal --steps 3 --warmup 1 &&
    trace c2 --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --distinct 0 ;;
  cdc)   # the CDC lines (C2 with its companions, C3 rank 3) and the C2 kernel trace
    bash tools/gpu.sh bench c2 --gpus 1 --steps 20 --warmup 5 &&
    bash tools/gpu.sh bench c3r3 --share 3/8 --steps 20 --warmup 5 --no-cpu-baseline &&
    trace c2 --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --distinct 0 ;;
  r7check)   # the C4 shape with R7 again, and with the file-sum trace build
    bash tools/gpu.sh tests tests/test_gpu_rsync.py tests/test_gpu_rsync_stream.py -x -k "file_sum or stream or fifo" &&
    bash tools/gpu.sh bench c4 --mode rsync --steps 10 --warmup 2 --no-cpu-baseline &&
    bash tools/gpu.sh bench c4share --mode rsync --share 3/8 --per-gpu-gib 32 --steps 10 --warmup 1 &&
    VSGPU_LIB=$PWD/$(var fstrace) bash tools/gpu.sh bench c4_fstrace --mode rsync --steps 4 --warmup 1 --no-cpu-baseline ;;
  multirank)   # shared-GPU rehearsals of the N-rank paths (gloo collectives, one card)
    export VSGPU_BENCH_SHARED_GPU=1
    bash tools/gpu.sh bench cdc2 --gpus 2 --per-gpu-gib 4 --steps 3 --warmup 1 &&
    bash tools/gpu.sh bench cdc4 --gpus 4 --per-gpu-gib 2 --steps 3 --warmup 1 &&
    bash tools/gpu.sh bench c4relay4 --mode rsync --gpus 4 --per-gpu-gib 4 --steps 2 --warmup 1 ;;
  walkab)   # walk occupancy A/B at the real C4 rank (w12: 12 waves/CU, 168 VGPRs, no prefilter)
    S="bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline"
    ab ab_walk_share 2 "base=,w12=$(var w12),w12d8=$(var w12d8),w8nopf=$(var w8nopf)" $S ;;
  corun)   # fingerprint + SHA-256 co-residency A/B
    bash tools/gpu.sh py tools/corun.py --sha-gb 4,8,16 --sha-grid 0 && mv gpurun_out/py_corun.log gpurun_out/corun_base_grid5.log &&
    VSGPU_LIB=$PWD/$(var corun) bash tools/gpu.sh py tools/corun.py --sha-gb 4,8,16 --sha-grid 1 && mv gpurun_out/py_corun.log gpurun_out/corun_co_grid1.log &&
    VSGPU_LIB=$PWD/$(var corun) bash tools/gpu.sh py tools/corun.py --sha-gb 4,8,16 --sha-grid 0 && mv gpurun_out/py_corun.log gpurun_out/corun_co_grid5.log ;;
  wideab)   # C2 replay with the drain's bulk in throughput (wide) mode
    for r in 1 2; do
      bash tools/gpu.sh bench c2_split_$r --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --distinct 0 &&
      bash tools/gpu.sh bench c2_wide98k_$r --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --distinct 0 --hash-wide 98304 &&
      bash tools/gpu.sh bench c2_wide256k_$r --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --distinct 0 --hash-wide 262144 --wide-drain 16384 || exit 1
    done ;;
  counters)  # C2 counter passes (traffic, VALU activity) -> gpurun_out/profile_c2
    bash tools/gpu.sh prof c2 'fp_kernel|sha_slice_kernel' --gpus 1 --steps 5 --warmup 1 --distinct 0 ;;
  pscanab)   # STEP probes batched a lane per survivor (product) against per-lane probes (pscan0): walk tests, real-C4 rank, C4 shape
    bash tools/gpu.sh tests tests/test_gpu_rsync.py tests/test_gpu_rsync_stream.py -x && mv gpurun_out/gputests.log gpurun_out/gputests_rsync.log &&
    ab ab_pscan_share 2 "pscan0=$(var pscan0),new=" bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline &&
    ab ab_pscan_c4 2 "pscan0=$(var pscan0),new=" bench.py --mode rsync --steps 5 --warmup 1 --no-file-sum --no-cpu-baseline ;;
  pscanprof)   # walk phase profiles at the real-C4 rank, batched probes (walkprof) and per-lane (walkprof0)
    for v in walkprof walkprof0; do
      VSGPU_LIB=$PWD/$(var $v) timeout -k 10 300 python bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 1 --warmup 1 \
        --no-cpu-baseline --no-file-sum > gpurun_out/bench_$v.log 2>&1 || exit 1
      echo "== $v"; grep "walk prof" gpurun_out/bench_$v.log | tail -1
    done ;;
  latefwab)   # STEP filter words tested after the previous batch's probe results (latefw = -DVS_WALK_LATEFW=1): walk tests, real-C4 rank, C4 shape
    VSGPU_LIB=$PWD/$(var latefw) bash tools/gpu.sh tests tests/test_gpu_rsync.py -x && mv gpurun_out/gputests.log gpurun_out/gputests_rsync_latefw.log &&
    ab ab_latefw_share 2 "latefw=$(var latefw),base=" bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline &&
    ab ab_latefw_c4 2 "latefw=$(var latefw),base=" bench.py --mode rsync --steps 5 --warmup 1 --no-file-sum --no-cpu-baseline ;;
  walkcounters)   # counter passes of the real-C4 rank's walk (spread STEP probes) -> gpurun_out/profile_c4share
    bash tools/gpu.sh prof c4share 'rs_walk_spec_kernel' --mode rsync --share 3/8 --per-gpu-gib 32 --steps 2 --warmup 1 --no-file-sum ;;
  isoab)   # isolated latency kernel: one consumer wave per CU (product) against two (iso2) and HEAD's build (head)
    bash tools/gpu.sh tests tests/test_gpu_cdc.py tests/test_gpu_c3.py -x && mv gpurun_out/gputests.log gpurun_out/gputests_cdc.log &&
    VSGPU_LIB=$PWD/$(var iso2) bash tools/gpu.sh tests tests/test_gpu_cdc.py -x -k "drain or sha256 or blob" && mv gpurun_out/gputests.log gpurun_out/gputests_iso2.log &&
    ab ab_iso_single_c2 2 "head=$(var head),new=,iso2=$(var iso2)" tools/single_pass.py --gib 64 --quad auto --rounds 2 &&
    ab ab_iso_single_c3r3 2 "head=$(var head),new=,iso2=$(var iso2)" tools/single_pass.py --share 3/8 --quad auto --rounds 2 &&
    VSGPU_LIB=$PWD/$(var shatrace) bash tools/gpu.sh py tools/sha_trace.py --gib 64 --quad auto:1 && mv gpurun_out/py_sha_trace.log gpurun_out/trace_c2_iso1.log &&
    VSGPU_LIB=$PWD/$(var iso2trace) bash tools/gpu.sh py tools/sha_trace.py --gib 64 --quad auto:1 && mv gpurun_out/py_sha_trace.log gpurun_out/trace_c2_iso2.log ;;
  distinctab)   # the distinct-volume line, two latency consumers per CU (product) against one (iso1)
    ab ab_distinct 2 "iso1=$(var iso1),new=" bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --distinct 3 ;;
  iso3ab)   # three latency consumers per CU (iso3, ring lead 1) against two (product)
    VSGPU_LIB=$PWD/$(var iso3) bash tools/gpu.sh tests tests/test_gpu_cdc.py tests/test_gpu_c3.py -x && mv gpurun_out/gputests.log gpurun_out/gputests_iso3.log &&
    bash tools/gpu.sh tests tests/test_gpu_cdc.py -x -k "drain or sha256 or blob" && mv gpurun_out/gputests.log gpurun_out/gputests_iso2.log &&
    ab ab_iso3_single_c2 2 "new=,iso3=$(var iso3)" tools/single_pass.py --gib 64 --quad auto --rounds 2 &&
    ab ab_iso3_single_c3r3 2 "new=,iso3=$(var iso3)" tools/single_pass.py --share 3/8 --quad auto --rounds 2 &&
    ab ab_iso3_distinct 2 "new=,iso3=$(var iso3)" bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --distinct 3 ;;
  quadtrace3)   # the C3 rank's drain: latency tiles and the split tail (VS_SHA_TRACE build shatrace)
    VSGPU_LIB=$PWD/$(var shatrace) bash tools/gpu.sh py tools/sha_trace.py --share 3/8 --quad auto:1 &&
    mv gpurun_out/py_sha_trace.log gpurun_out/trace_c3r3_quad.log ;;
  capab)   # latency-mode cap: 16 chains per two CUs (product) against 20 (cap20), C3 rank, C2, distinct
    ab ab_cap_single_c3r3 2 "new=,cap20=$(var cap20)" tools/single_pass.py --share 3/8 --quad auto --rounds 2 &&
    ab ab_cap_single_c2 1 "new=,cap20=$(var cap20)" tools/single_pass.py --gib 64 --quad auto --rounds 2 ;;
  tracec3)   # kernel trace + stats of the C3 rank-3 line (rocprofv3, no counters)
    trace c3r3 --share 3/8 --steps 20 --warmup 5 --no-cpu-baseline ;;
  sharedab)   # chains past the isolated cap in shared-CU latency tiles (product) against split mode (noshared)
    bash tools/gpu.sh tests tests/test_gpu_cdc.py tests/test_gpu_c3.py -x && mv gpurun_out/gputests.log gpurun_out/gputests_cdc.log &&
    ab ab_shared_single_c3r3 2 "noshared=$(var noshared),new=" tools/single_pass.py --share 3/8 --quad auto --rounds 2 &&
    ab ab_shared_single_c2 1 "noshared=$(var noshared),new=" tools/single_pass.py --gib 64 --quad auto --rounds 2 &&
    ab ab_shared_distinct 1 "noshared=$(var noshared),new=" bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --distinct 3 ;;
  shareddist)   # the distinct-volume line again, shared tail (product) against noshared, two rounds
    ab ab_shared_distinct2 2 "noshared=$(var noshared),new=" bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --distinct 3 ;;
  sharedab2)   # shared tail only in tail-bound drains (product) against noshared: C3 rank, distinct
    ab ab_shared2_single_c3r3 2 "noshared=$(var noshared),new=" tools/single_pass.py --share 3/8 --quad auto --rounds 2 &&
    ab ab_shared2_distinct 2 "noshared=$(var noshared),new=" bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --distinct 3 ;;
  sharedreplay)   # the replayed C2 line, shared tail (product) against noshared, three rounds
    ab ab_shared_replay 3 "noshared=$(var noshared),new=" bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --distinct 0 ;;
  quadprobe)   # cycles per latency-mode round alone on a SIMD, per round form (tools/probe/quad_round.hip)
    mkdir -p tools/probe/bin && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/probe/bin/quad_round tools/probe/quad_round.hip &&
    timeout -k 10 60 ./tools/probe/bin/quad_round > gpurun_out/quad_round.txt 2>&1; rc=$?; cat gpurun_out/quad_round.txt; exit $rc ;;
  quadtrace)   # the latency tiles' duration, clock and the longest chain (VS_SHA_TRACE build shatrace)
    VSGPU_LIB=$PWD/$(var shatrace) bash tools/gpu.sh py tools/sha_trace.py --gib 64 --quad auto:1 &&
    mv gpurun_out/py_sha_trace.log gpurun_out/trace_c2_quad.log ;;
  quadfinal)   # the isolated latency form in the product: CDC tests, single pass and the C2 line against HEAD's build (var head)
    bash tools/gpu.sh tests tests/test_gpu_cdc.py tests/test_gpu_c3.py -x && mv gpurun_out/gputests.log gpurun_out/gputests_cdc.log &&
    ab ab_final_single_c2 2 "head=$(var head),new=" tools/single_pass.py --gib 64 --quad auto:1,auto:0 --rounds 2 &&
    ab ab_final_single_c3r3 2 "head=$(var head),new=" tools/single_pass.py --share 3/8 --quad auto --rounds 2 &&
    ab ab_final_c2 2 "head=$(var head),new=" bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --distinct 0 ;;
  first)
    hostinfo &&
    bash tools/gpu.sh tests tests/test_gpu_cdc.py -x &&
    ab ab_single_c3r3 1 "new=,qpp0=$(var qpp0)" tools/single_pass.py --share 3/8 --quad auto,80 --rounds 2 &&
    bash tools/gpu.sh bench c2 --gpus 1 --steps 20 --warmup 5 &&
    bash tools/gpu.sh bench c3r3 --share 3/8 --steps 20 --warmup 5 --no-cpu-baseline ;;
  iso)
    bash tools/gpu.sh tests tests/test_gpu_cdc.py -x -k "sha256 or drain or blob" &&
    bash tools/gpu.sh py tools/single_pass.py --share 3/8 --quad auto:1,auto:0 --rounds 3 &&
    mv gpurun_out/py_single_pass.log gpurun_out/single_c3r3.log &&
    bash tools/gpu.sh py tools/single_pass.py --gib 64 --quad auto:1,auto:0 --rounds 3 &&
    mv gpurun_out/py_single_pass.log gpurun_out/single_c2.log ;;
  isotrace)
    bash tools/r06_runs.sh iso && bash tools/r06_runs.sh trace ;;
  trace)   # where the drain's tiles run (VS_SHA_TRACE build shatrace)
    VSGPU_LIB=$PWD/$(var shatrace) bash tools/gpu.sh py tools/sha_trace.py --share 3/8 --quad auto:1,auto:0,auto:1 &&
    mv gpurun_out/py_sha_trace.log gpurun_out/trace_c3r3.log &&
    VSGPU_LIB=$PWD/$(var shatrace) bash tools/gpu.sh py tools/sha_trace.py --gib 64 --quad auto:1,auto:0 &&
    mv gpurun_out/py_sha_trace.log gpurun_out/trace_c2.log ;;
  *) echo "usage: tools/r06_runs.sh validate|benches|cdc|quadfinal|quadtrace|..." >&2; exit 2 ;;
esac
