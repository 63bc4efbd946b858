#!/bin/bash
# Round 5's GPU runs, one subcommand each (through gpurun; every GPU step has
# its own time limit in tools/gpu.sh or here, and the chain stops at the first
# failure).
#   first     VALU probe 3, the CDC + C3 GPU tests, fingerprint A/B (fpb0 =
#             -DVS_FP_BITOP3=0), C2 bench at the driver's 20/5, its trace-only
#             rocprofv3 run, one C3 rank at 20/5          -> profiles/r05_*
#   second    the whole -m gpu suite, C5 (known-index dedup, golden), the C4
#             shape with R7, one real-C4 rank, a C4 kernel+copy+API trace
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
c4trace() {  # c4trace <tag> <bench args...>: kernels + copies + HIP API (no counters)
  local tag=$1 out=$PWD/gpurun_out/c4trace_$1 repo=$PWD
  shift
  mkdir -p "$out"
  (cd /tmp && TMPDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace --hip-runtime-trace \
     --memory-copy-trace -d "$out/raw" -o run --output-format csv -- python3 "$repo/bench.py" "$@") \
     > "$out/bench.log" 2>&1
  local rc=$?
  echo "=== c4trace_$tag rc=$rc"; tail -n 1 "$out/bench.log" | cut -c1-300
  [ $rc -eq 0 ] || return $rc
  python3 tools/c4_timeline.py "$out/raw" > "$out/timeline.txt" 2>&1
  rm -rf "$out/raw"
}
c4copy() {  # c4copy <tag> <bench args...>: kernels + memory copies (no API trace, no counters)
  local tag=$1 out=$PWD/gpurun_out/c4copy_$1 repo=$PWD
  shift
  mkdir -p "$out"
  (cd /tmp && TMPDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats \
     -d "$out/raw" -o run --output-format csv -- python3 "$repo/bench.py" "$@") > "$out/bench.log" 2>&1
  local rc=$?
  echo "=== c4copy_$tag rc=$rc"; tail -n 1 "$out/bench.log" | cut -c1-300
  [ $rc -eq 0 ] || return $rc
  python3 tools/c4_timeline.py "$out/raw" > "$out/timeline.txt" 2>&1
  find "$out/raw" -name '*_stats.csv' -exec cp {} "$out/" \;
  rm -rf "$out/raw"
}
case $1 in
  first)
    timeout -k 10 120 tools/valu/valu_ops3 > gpurun_out/valu_ops3.json 2> gpurun_out/valu_ops3.err &&
    echo "=== valu_ops3 ok" &&
    bash tools/gpu.sh tests tests/test_gpu_c3.py tests/test_gpu_cdc.py -x &&
    ab fp_ab 3 "fpb0=$(var fpb0),new=" tools/fp_only.py --gib 64 --reps 5 &&
    bash tools/gpu.sh bench c2 --gpus 1 --steps 20 --warmup 5 &&
    trace c2 --gpus 1 --steps 20 --warmup 5 &&
    bash tools/gpu.sh bench c3r3 --share 3/8 --steps 20 --warmup 5 --no-cpu-baseline ;;
  second)
    bash tools/gpu.sh tests &&
    bash tools/gpu.sh bench c5 --mode smallfiles --steps 5 --warmup 1 &&
    bash tools/gpu.sh bench c4 --mode rsync --steps 5 --warmup 1 --no-cpu-baseline &&
    bash tools/gpu.sh bench c4share_nofs --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 \
      --warmup 1 --no-file-sum &&
    c4trace c4 --mode rsync --steps 3 --warmup 1 --no-cpu-baseline ;;
  d2h)
    timeout -k 10 300 tools/probe/bin/d2h_overlap > gpurun_out/d2h_overlap.json 2> gpurun_out/d2h_overlap.err &&
    echo "=== d2h ok" && cat gpurun_out/d2h_overlap.json &&
    c4copy c4 --mode rsync --steps 3 --warmup 1 --no-cpu-baseline ;;
  d2hprof)
    out=$PWD/gpurun_out/d2hprof; mkdir -p "$out"; repo=$PWD
    (cd /tmp && TMPDIR=/tmp timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats \
       -d "$out/cpp" -o run --output-format csv -- "$repo/tools/probe/bin/d2h_overlap") \
       > "$out/cpp.log" 2>&1 && echo "=== cpp ok" &&
    (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats \
       -d "$out/torch" -o run --output-format csv -- python3 "$repo/tools/probe/d2h_torch.py") \
       > "$out/torch.log" 2>&1 && echo "=== torch ok" && tail -n 1 "$out/torch.log" &&
    find "$out" -name '*stats.csv' | sort ;;
  d2hapi)
    out=$PWD/gpurun_out/d2hapi; mkdir -p "$out"; repo=$PWD
    timeout -k 10 200 python3 tools/probe/d2h_apis.py > "$out/plain.log" 2>&1 && echo "=== plain ok" &&
    tail -n 1 "$out/plain.log" &&
    (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats \
       -d "$out/prof" -o run --output-format csv -- python3 "$repo/tools/probe/d2h_apis.py") \
       > "$out/prof.log" 2>&1 && echo "=== prof ok" && rm -f "$out"/prof/*trace.csv ;;
  r7)
    bash tools/gpu.sh tests tests/test_gpu_rsync.py tests/test_gpu_rsync_stream.py -x &&
    bash tools/gpu.sh bench c4r7 --mode rsync --steps 5 --warmup 1 --no-cpu-baseline &&
    bash tools/gpu.sh bench c4r7_10 --mode rsync --steps 10 --warmup 2 --no-cpu-baseline &&
    bash tools/gpu.sh bench c4share_r7 --mode rsync --share 3/8 --per-gpu-gib 32 --steps 6 --warmup 1 &&
    c4copy c4r7 --mode rsync --steps 3 --warmup 1 --no-cpu-baseline ;;
  r7b)
    bash tools/gpu.sh tests tests/test_gpu_rsync.py -x &&
    bash tools/gpu.sh bench c4r7_10 --mode rsync --steps 10 --warmup 2 --no-cpu-baseline &&
    bash tools/gpu.sh bench c4r7_20 --mode rsync --steps 20 --warmup 2 --no-cpu-baseline &&
    bash tools/gpu.sh bench c4share_r7 --mode rsync --share 3/8 --per-gpu-gib 32 --steps 10 --warmup 1 &&
    c4copy c4r7b --mode rsync --steps 3 --warmup 1 --no-cpu-baseline ;;
  fpchains)
    ab fp_chains 3 "base=,t512c4=$(var fpt512c4),t512c3=$(var fpt512c3),c3=$(var fpc3),t1024=$(var fpt1024)" \
      tools/fp_only.py --gib 64 --reps 5 ;;
  walk)  # bank-balanced wide-flush reads (VS_WIDE_RD=1) against the dword reads (rd0)
    S="--mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum"
    C="--mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline"
    L="rd0=$(var rd0),p2=$(var p2),new=,p4=$(var p4)"
    bash tools/gpu.sh tests tests/test_gpu_rsync.py -x &&
    ab walk2_share 2 "$L" bench.py $S &&
    ab walk2_c4 2 "$L" bench.py $C &&
    bash tools/gpu.sh prof r05_walk2_share rs_walk $S ;;
  sdma)  # does an SDMA device-to-host copy slow a latency-bound kernel? (THP / d2d controls)
    cat /sys/kernel/mm/transparent_hugepage/enabled > gpurun_out/thp.txt 2>&1
    timeout -k 10 300 tools/probe/bin/sdma_interf > gpurun_out/sdma_interf.json 2> gpurun_out/sdma_interf.err &&
    echo "=== sdma ok" && cat gpurun_out/sdma_interf.json ;;
  diag)  # sdma probe, R7 with 3 / 2 file-sum jobs and none, C2 counters
    bash tools/r05_runs.sh sdma &&
    bash tools/gpu.sh bench c4r7_j3 --mode rsync --steps 10 --warmup 2 --no-cpu-baseline &&
    bash tools/gpu.sh bench c4r7_j2 --mode rsync --steps 10 --warmup 2 --no-cpu-baseline --file-sum-jobs 2 &&
    bash tools/gpu.sh bench c4_nofs --mode rsync --steps 10 --warmup 2 --no-cpu-baseline --no-file-sum &&
    bash tools/gpu.sh prof r05_c2 "fp_kernel|sha_slice" --gpus 1 --steps 5 --warmup 2 ;;
  r7iso)  # which part of R7 slows the walk: the host chain (fsnochain), the read-back (fsnodma)
    # (historical: the VS_FS_DIAG build flag these variants used was removed
    # after the run, profiles/r05_r7/iso)
    L="base=,nochain=$(var fsnochain),nodma=$(var fsnodma)"
    ab r7iso_c4 2 "$L" bench.py --mode rsync --steps 8 --warmup 2 --no-cpu-baseline ;;
  r7clock)  # the walk's effective clock with and without R7 (one counter pass each)
    for cfg in r7 nofs; do
      extra=""; [ $cfg = nofs ] && extra="--no-file-sum"
      out=$PWD/gpurun_out/r7clock_$cfg; mkdir -p "$out/trace"; repo=$PWD
      (cd /tmp && TMPDIR=/tmp timeout -k 10 400 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_BUSY_CYCLES \
         SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex "rs_walk_spec|rs_sig|fs_contrib" \
         -d "$out/pmc_sq" -o run --output-format csv -- python3 "$repo/bench.py" --mode rsync --steps 4 --warmup 1 \
         --no-cpu-baseline $extra) > "$out/bench.log" 2>&1 || exit $?
      echo "=== r7clock $cfg ok"
      find "$out/pmc_sq" -name '*kernel_stats.csv' -exec cp {} "$out/trace/" \;
      python3 tools/summarize_prof.py "$out" --out "gpurun_out/r7clock_${cfg}_sum" > "$out/sum.log" 2>&1
      rm -rf "$out/pmc_sq"
    done ;;
  r7cyc)  # walk cycles per wave (s_memtime) with and without R7: clock or contention?
    for cfg in r7 nofs r7b; do
      extra=""; [ $cfg = nofs ] && extra="--no-file-sum"
      VSGPU_LIB=$PWD/$(var walkprof) timeout -k 10 400 python bench.py --mode rsync --steps 4 --warmup 1 \
        --no-cpu-baseline $extra > gpurun_out/r7cyc_$cfg.log 2>&1 || exit $?
      echo "=== r7cyc $cfg"; grep "walk prof" gpurun_out/r7cyc_$cfg.log | tail -1 | cut -c1-400
    done ;;
  r7trace)  # per-job file-sum timelines (VS_FS_TRACE build) over four processes, to catch both modes
    for i in 1 2 3 4; do
      VSGPU_LIB=$PWD/$(var fstrace) timeout -k 10 400 python bench.py --mode rsync --steps 8 --warmup 2 \
        --no-cpu-baseline > gpurun_out/r7trace_$i.log 2>&1 || exit $?
      echo "=== r7trace $i: $(tail -1 gpurun_out/r7trace_$i.log | cut -c1-160)"
    done ;;
  numa)  # D2H DMA rate by NUMA node of the destination, by thread count, by SDMA engine
    timeout -k 10 300 tools/probe/bin/d2h_numa > gpurun_out/d2h_numa.json 2> gpurun_out/d2h_numa.err;
    rc=$?; cat gpurun_out/d2h_numa.json; head -5 gpurun_out/d2h_numa.err; exit $rc ;;
  r7eng)  # R7 with the read-back pinned to the preferred SDMA engine: four processes + the share
    bash tools/gpu.sh tests tests/test_gpu_rsync.py -x -k "file_sum" &&
    for i in 1 2 3 4; do
      VSGPU_LIB=$PWD/$(var fstrace) timeout -k 10 400 python bench.py --mode rsync --steps 10 --warmup 2 \
        --no-cpu-baseline > gpurun_out/r7eng_$i.log 2>&1 || exit $?
      echo "=== r7eng $i: $(tail -1 gpurun_out/r7eng_$i.log | cut -c1-160)"
    done &&
    for i in 1 2; do
      timeout -k 10 400 python bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 10 --warmup 1 \
        > gpurun_out/r7eng_share_$i.log 2>&1 || exit $?
      echo "=== r7eng share $i: $(tail -1 gpurun_out/r7eng_share_$i.log | cut -c1-160)"
    done ;;
  final)  # the round's closing evidence -> gpurun_out (copied to profiles/r05_end)
    bash tools/gpu.sh tests && bash tools/gpu.sh smoke && bash "$0" benches ;;
  benches)
    bash tools/gpu.sh bench c2 --gpus 1 --steps 20 --warmup 5 &&
    bash tools/gpu.sh bench c3r3 --share 3/8 --steps 20 --warmup 5 --no-cpu-baseline &&
    bash tools/gpu.sh bench c4 --mode rsync --steps 20 --warmup 2 --no-cpu-baseline &&
    bash tools/gpu.sh bench c4_nofs --mode rsync --steps 5 --warmup 1 --no-file-sum &&
    bash tools/gpu.sh bench c4share --mode rsync --share 3/8 --per-gpu-gib 32 --steps 10 --warmup 1 &&
    bash tools/gpu.sh bench c4share_nofs --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum &&
    bash tools/gpu.sh bench c5 --mode smallfiles --steps 5 --warmup 1 &&
    bash tools/gpu.sh bench seal --mode seal --steps 3 --warmup 1 &&
    trace c2_end --gpus 1 --steps 20 --warmup 5 ;;
  walkwd)  # deeper flush prefetch now that wide_windows holds 136 VGPRs (no callee saves)
    S="--mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum"
    C="--mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline"
    L="base=,wd6=$(var wd6),wd8=$(var wd8)"
    ab walkwd_share 2 "$L" bench.py $S && ab walkwd_c4 2 "$L" bench.py $C ;;
  post)  # after the 8 KiB flush prefetch: the rsync GPU tests and the walk lines
    bash tools/gpu.sh tests tests/test_gpu_rsync.py tests/test_gpu_rsync_stream.py -x &&
    bash tools/gpu.sh bench c4share_nofs_wd8 --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum &&
    bash tools/gpu.sh bench c4_nofs_wd8 --mode rsync --steps 5 --warmup 1 --no-file-sum &&
    bash tools/gpu.sh bench c4_wd8 --mode rsync --steps 20 --warmup 2 --no-cpu-baseline &&
    bash tools/gpu.sh bench c4share_wd8 --mode rsync --share 3/8 --per-gpu-gib 32 --steps 10 --warmup 1 ;;
  fpocc)  # fingerprint occupancy against the SHA slices sharing the CUs: 512 / 768 / 1024 threads
    ab fpocc_c2 2 "base=,t512=$(var fpt512),t768=$(var fpt768)" bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline ;;
  fsab)  # contribution rows kernel: 8 lanes per block (128-byte lines per instruction) against 4
    bash tools/gpu.sh tests tests/test_gpu_rsync.py tests/test_gpu_rsync_stream.py -x -k "file_sum or relay or stream" &&
    ab fsab_c4 2 "fs4=$(var fs4),new=" bench.py --mode rsync --steps 10 --warmup 2 --no-cpu-baseline &&
    ab fsab_share 2 "fs4=$(var fs4),new=" bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 10 --warmup 1 ;;
  fsab2)  # contribution rows kernel: 16 lanes per block against 8
    ab fsab2_c4 2 "new=,fs16=$(var fs16)" bench.py --mode rsync --steps 10 --warmup 2 --no-cpu-baseline ;;
  steprange)  # STEP validity as one range per lane against a compare pair per offset (sr0)
    S="--mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum"
    C="--mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline"
    bash tools/gpu.sh tests tests/test_gpu_rsync.py -x -k "walk or real_density or stitch or shard" &&
    ab sr_share 2 "sr0=$(var sr0),new=" bench.py $S && ab sr_c4 2 "sr0=$(var sr0),new=" bench.py $C ;;
  fsab3)  # contribution rows kernel: 32 / 64 lanes per block against 16
    bash tools/gpu.sh tests tests/test_gpu_rsync.py -x -k "file_sum" &&
    VSGPU_LIB=$PWD/$(var fs64) bash tools/gpu.sh tests tests/test_gpu_rsync.py -x -k "file_sum" &&
    ab fsab3_c4 2 "new=,fs32=$(var fs32),fs64=$(var fs64)" bench.py --mode rsync --steps 10 --warmup 2 --no-cpu-baseline &&
    ab fsab3_share 1 "new=,fs32=$(var fs32),fs64=$(var fs64)" bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 10 --warmup 1 ;;
  endprof)  # counter passes of the final tree's walk (real-C4 rank) and C2 (perturbed: --pmc)
    bash tools/gpu.sh prof r05_end_walkshare rs_walk --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum &&
    bash tools/gpu.sh prof r05_end_c4 "rs_walk|fs_contrib|rs_sig" --mode rsync --steps 3 --warmup 1 ;;
  clean)  # the tree after removing the losing / equal variant paths: walk + file-sum tests and lines
    bash tools/gpu.sh tests tests/test_gpu_rsync.py tests/test_gpu_rsync_stream.py -x &&
    bash tools/gpu.sh bench c4share_nofs_clean --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum &&
    bash tools/gpu.sh bench c4_clean --mode rsync --steps 20 --warmup 2 --no-cpu-baseline &&
    bash tools/gpu.sh bench c4share_clean --mode rsync --share 3/8 --per-gpu-gib 32 --steps 10 --warmup 1 ;;
  last)  # the final tree: the whole GPU suite, smoke, C2 at the driver's 20/5, C5
    bash tools/gpu.sh tests && bash tools/gpu.sh smoke &&
    bash tools/gpu.sh bench c2_last --gpus 1 --steps 20 --warmup 5 &&
    bash tools/gpu.sh bench c5_last --mode smallfiles --steps 5 --warmup 1 ;;
  occ)  # walk occupancy: no LDS prefilter (8 waves / CU), and 12 waves / CU at 168 VGPRs
    S="--mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum"
    C="--mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline"
    VSGPU_LIB=$PWD/$(var occ3) bash tools/gpu.sh tests tests/test_gpu_rsync.py -x -k "walk or real_density or stitch or shard" &&
    ab occ_share 2 "base=,nopf=$(var nopf),occ3=$(var occ3)" bench.py $S &&
    ab occ_c4 2 "base=,nopf=$(var nopf),occ3=$(var occ3)" bench.py $C ;;
  sig)  # signature pass: 8 / 16 lanes per block against 4
    VSGPU_LIB=$PWD/$(var sig16) bash tools/gpu.sh tests tests/test_gpu_rsync.py -x -k "signature or golden or c4_params or sharded" &&
    VSGPU_LIB=$PWD/$(var sig8) bash tools/gpu.sh tests tests/test_gpu_rsync.py -x -k "signatures_vs_golden" &&
    ab sig_share 2 "base=,sig8=$(var sig8),sig16=$(var sig16)" bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum ;;
  sig2)  # signature pass shipped at 8 lanes: the rsync GPU tests, then against 4 lanes at both shapes
    bash tools/gpu.sh tests tests/test_gpu_rsync.py tests/test_gpu_rsync_stream.py -x &&
    ab sig2_share 3 "sig8=,sig4=$(var sig4)" bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum &&
    ab sig2_c4 3 "sig8=,sig4=$(var sig4)" bench.py --mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline ;;
  wprof)  # walk phases per wave, with the wide flushes' iterations and windows per pass
    for cfg in share c4; do
      if [ $cfg = share ]; then args="--share 3/8 --per-gpu-gib 32"; else args="--no-cpu-baseline"; fi
      VSGPU_LIB=$PWD/$(var walkprof) timeout -k 10 400 python bench.py --mode rsync --steps 3 --warmup 1 \
        --no-file-sum $args > gpurun_out/wprof_$cfg.log 2>&1 || exit $?
      echo "=== wprof $cfg"; grep "walk prof" gpurun_out/wprof_$cfg.log | tail -1 | cut -c1-900
    done ;;
  prio)  # wave priority: STEP batches (latency chains) above flushes and RUN windows (VALU)
    S="--mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum"
    C="--mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline"
    VSGPU_LIB=$PWD/$(var prio2) bash tools/gpu.sh tests tests/test_gpu_rsync.py -x -k "walk or real_density or stitch" &&
    ab prio_share 2 "base=,prio1=$(var prio1),prio2=$(var prio2)" bench.py $S &&
    ab prio_c4 2 "base=,prio1=$(var prio1),prio2=$(var prio2)" bench.py $C ;;
  dw4)  # wide flush: dword-aligned ds_read_b64 (no selects) against qword-aligned + selects
    S="--mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum"
    C="--mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline"
    VSGPU_LIB=$PWD/$(var dw4) bash tools/gpu.sh tests tests/test_gpu_rsync.py -x -k "walk or real_density or stitch or shard" &&
    ab dw4_share 3 "base=,dw4=$(var dw4)" bench.py $S &&
    ab dw4_c4 2 "base=,dw4=$(var dw4)" bench.py $C ;;
  margin)  # walk segments starting a margin before a block boundary (16 KiB shipped) against unaligned (m0)
    S="--mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum"
    C="--mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline"
    bash tools/gpu.sh tests tests/test_gpu_rsync.py tests/test_gpu_rsync_stream.py -x &&
    ab margin_share 2 "m16k=,m0=$(var m0),m4k=$(var m4096),m64k=$(var m65536)" bench.py $S &&
    ab margin_c4 2 "m16k=,m0=$(var m0),m4k=$(var m4096),m64k=$(var m65536)" bench.py $C ;;
  margin2)  # segment margin 8 / 24 / 32 KiB against the shipped 16 KiB, then the share walk's counters
    S="--mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum"
    ab margin2_share 2 "m16k=,m8k=$(var m8192),m24k=$(var m24576),m32k=$(var m32768)" bench.py $S &&
    bash tools/gpu.sh prof r05_end4_walkshare rs_walk --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum ;;
  margin3)  # the shipped 24 KiB margin: the rsync GPU tests and the share / 64 GiB lines
    bash tools/gpu.sh tests tests/test_gpu_rsync.py tests/test_gpu_rsync_stream.py -x &&
    bash tools/gpu.sh bench c4share_nofs_m24 --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum &&
    bash tools/gpu.sh bench c4share_m24 --mode rsync --share 3/8 --per-gpu-gib 32 --steps 10 --warmup 1 &&
    bash tools/gpu.sh bench c4_m24 --mode rsync --steps 20 --warmup 2 --no-cpu-baseline ;;
  *) echo "usage: tools/r05_runs.sh first|second|d2h|d2hprof|d2hapi|r7|r7b|fpchains|walk" >&2; exit 2 ;;
esac
