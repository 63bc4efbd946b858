#!/bin/bash
# Round 4's GPU runs, one subcommand each (run on the box through gpurun; each
# step has its own time limit in tools/gpu.sh and the steps stop at the first
# failure).  The A/B variants were built with tools/build_variant.sh as noted;
# where the winner became the code or the variant lost, its macro is gone
# (regs, aligned, sha, shalds),
# and the lines stay as the record of how the committed logs were made.
#
#   closing     the whole -m gpu suite, smoke(), the bench lines, all of C3
#               rank by rank                               -> profiles/r04_end
#   benches     C2, C4 shape, one real-C4 rank, rsync-host, 2-rank relay, MD5
#   rsync       the rsync lines with and without R7        -> profiles/r04_end/final
#   profiles    rocprofv3 trace + PMC passes of C2, one real-C4 rank, C4 shape
#   multirank   shared-GPU rehearsals: CDC at 2 and 4 ranks, rsync + R7 relay at 4
#   flush       flush width / early flush / prefilter / span options -> profiles/r04_walk_ab, r04_walk_lds
#   regs        build d4sk (-DVS_WIDE_D=4 -DVS_WIDE_SK_LDS=1), sklds (-DVS_WIDE_SK_LDS=1)
#   aligned     build aligned (-DVS_WIDE_ALIGNED=1)        -> profiles/r04_walk_lds/ab5_*
#   step        build fb24 (-DVS_FBITS_CAP=24u); buckets, prefilter -> profiles/r04_walk_step
#   seg         segment lengths (SEGS="16 24 32 48 64 96") -> profiles/r04_walk_step
#   lookahead   build wd2, wd4, wd6 (-DVS_WIDE_D=N)        -> profiles/r04_walk_step/ab_wd*
#   tail        tail shares (TAILS="0 10 15 20 30 40")     -> profiles/r04_walk_step/tail*
#   sha         build shaalt (-DVS_SHA_ALTERNATE=1)         -> profiles/r04_sha_ab
#   predict     build p1, p6 (-DVS_PREDICT=N), wd2 (-DVS_WIDE_D=2) -> profiles/r04_walk_step/ab_pred*
#   shalds      build shalds (-DVS_SHA_LDS_WINDOW=1)        -> profiles/r04_sha_ab
#   taildiv     build td3, td6 (-DVS_TAIL_DIV=N: tail segments a third / sixth long)
#   runring     build rr2, rr6 (-DVS_WALK_RRING=N: RUN-window blocks in flight)
#   walkprof    build walkprof (-DVS_WALK_PROF=1): walk phase profiles
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
S="--mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum"
C="--mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline"
var() { echo "volsync_amd/lib/var/$1/libvsgpu.so"; }
ab() {  # ab <log> <rounds> <libs> <bench args...>
  local log=$1 rounds=$2 libs=$3
  shift 3
  timeout -k 10 600 python3 -u tools/ab.py --rounds "$rounds" --libs "$libs" -- bench.py "$@" \
    > "gpurun_out/$log.log" 2>&1
}
case $1 in
  closing)
    bash tools/gpu.sh tests && bash tools/gpu.sh smoke && bash "$0" benches && bash tools/c3_ranks.sh ;;
  benches)
    bash tools/gpu.sh bench c2 --steps 10 --warmup 2 &&
    bash tools/gpu.sh bench c4 --mode rsync --steps 5 --warmup 1 --no-cpu-baseline &&
    bash tools/gpu.sh bench c4share --mode rsync --share 3/8 --per-gpu-gib 32 --steps 6 --warmup 1 &&
    bash tools/gpu.sh bench rsynchost --mode rsync-host --steps 2 --warmup 1 &&
    VSGPU_BENCH_SHARED_GPU=1 bash tools/gpu.sh bench c4relay2 --mode rsync --gpus 2 --per-gpu-gib 4 --steps 3 --warmup 1 &&
    bash tools/gpu.sh bench c4md5 --mode rsync --csum md5 --steps 1 --warmup 0 --no-file-sum --no-cpu-baseline &&
    bash tools/gpu.sh bench c4md5fs --mode rsync --csum md5 --per-gpu-gib 8 --steps 1 --warmup 0 --no-cpu-baseline ;;
  rsync)
    bash tools/gpu.sh bench c4share_nofs $S &&
    bash tools/gpu.sh bench c4_nofs --mode rsync --steps 5 --warmup 1 --no-file-sum --no-cpu-baseline &&
    bash tools/gpu.sh bench c4share6 --mode rsync --share 3/8 --per-gpu-gib 32 --steps 6 --warmup 1 &&
    bash tools/gpu.sh bench c4 --mode rsync --steps 5 --warmup 1 &&
    bash tools/gpu.sh bench rsynchost --mode rsync-host --steps 2 --warmup 1 ;;
  profiles)
    bash tools/gpu.sh prof r04_c2 '.*' --steps 5 --warmup 1 &&
    bash tools/gpu.sh prof r04_c4share_final rs_walk $S &&
    bash tools/gpu.sh prof r04_c4_final rs_walk --mode rsync --steps 3 --warmup 1 --no-file-sum ;;
  multirank)
    export VSGPU_BENCH_SHARED_GPU=1
    bash tools/gpu.sh bench cdc2 --gpus 2 --per-gpu-gib 4 --steps 3 --warmup 1 &&
    bash tools/gpu.sh bench cdc4 --gpus 4 --per-gpu-gib 2 --steps 3 --warmup 1 &&
    bash tools/gpu.sh bench c4relay4 --mode rsync --gpus 4 --per-gpu-gib 4 --steps 2 --warmup 1 ;;
  flush)
    for o in walk_flush_windows=16 walk_flush_windows=4 walk_flush_predict=0 \
             walk_flush_windows=4,walk_flush_predict=0 walk_prefilter=0 walk_flush_span=32768; do
      bash tools/gpu.sh bench "flush_share_${o//[=,]/_}" $S --walk-opt "$o" &&
      bash tools/gpu.sh bench "flush_c4_${o//[=,]/_}" $C --walk-opt "$o" || exit $?
    done ;;
  regs)
    ab ab3_share 2 "base=,d4sk=$(var d4sk),sklds=$(var sklds)" $S &&
    ab ab3_c4 2 "base=,d4sk=$(var d4sk),sklds=$(var sklds)" $C ;;
  aligned)
    ab ab5_share 2 "base=,aligned=$(var aligned)" $S && ab ab5_c4 2 "base=,aligned=$(var aligned)" $C ;;
  step)
    ab ab6_fb 2 "base=,fb24=$(var fb24)" $S && ab ab6_bb19 2 base= $S --walk-opt bucket_bits=19 &&
    ab ab6_nopf 2 base= $S --walk-opt walk_prefilter=0 && ab ab6_c4_fb 2 "base=,fb24=$(var fb24)" $C ;;
  seg)
    for r in 0 1; do for sb in ${SEGS:-16 24 32 48 64 96}; do
      bash tools/gpu.sh bench "seg_share_${sb}_r$r" $S --walk-opt "walk_segment_blocks=$sb" &&
      bash tools/gpu.sh bench "seg_c4_${sb}_r$r" $C --walk-opt "walk_segment_blocks=$sb" || exit $?
    done; done ;;
  lookahead)
    L="wd2=$(var wd2),wd4=$(var wd4),wd6=$(var wd6)"
    ab ab_wd2_share 2 "$L" $S && ab ab_wd2_c4 2 "$L" $C ;;
  tail)
    for r in 0 1; do for tp in ${TAILS:-0 10 15 20 30 40}; do
      bash tools/gpu.sh bench "tail_share_${tp}_r$r" $S --walk-opt "walk_tail_pct=$tp" &&
      bash tools/gpu.sh bench "tail_c4_${tp}_r$r" $C --walk-opt "walk_tail_pct=$tp" || exit $?
    done; done ;;
  sha)
    ab ab_sha_c2 3 "base=,shaalt=$(var shaalt)" --steps 10 --warmup 2 --no-cpu-baseline &&
    ab ab_sha_c5 1 "base=,shaalt=$(var shaalt)" --mode smallfiles --steps 5 --warmup 1 --no-cpu-baseline ;;
  predict)
    L="base=,p1=$(var p1),p6=$(var p6),wd2=$(var wd2)"
    ab ab_pred_share 2 "$L" $S && ab ab_pred_c4 2 "$L" $C ;;
  shalds)
    ab ab_shalds_c2 3 "base=,shalds=$(var shalds)" --steps 10 --warmup 2 --no-cpu-baseline &&
    ab ab_shalds_c5 1 "base=,shalds=$(var shalds)" --mode smallfiles --steps 5 --warmup 1 --no-cpu-baseline ;;
  taildiv)
    L="base=,td3=$(var td3),td6=$(var td6)"
    ab ab_td_share 2 "$L" $S && ab ab_td_c4 2 "$L" $C ;;
  runring)
    L="base=,rr2=$(var rr2),rr6=$(var rr6)"
    ab ab_rr_share 2 "$L" $S && ab ab_rr_c4 2 "$L" $C ;;
  walkprof)
    bash tools/c4_walkprof.sh --share 3/8 --per-gpu-gib 32 > gpurun_out/walkprof2_share.txt 2>&1 &&
    bash tools/c4_walkprof.sh > gpurun_out/walkprof2_c4.txt 2>&1 ;;
  *) echo "usage: tools/r04_runs.sh closing|benches|rsync|profiles|multirank|flush|regs|aligned|step|seg|lookahead|tail|sha|predict|shalds|taildiv|runring|walkprof" >&2
     exit 2 ;;
esac
