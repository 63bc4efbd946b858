#!/bin/bash
# Walk phase profiles (VS_WALK_PROF build: tools/build_variant.sh walkprof
# -DVS_WALK_PROF=1) at one rank of the real C4 and at the 64 GiB shape, then
# the rocprofv3 trace + FETCH/WRITE/SQ/LDS passes of the share line, then an
# A/B of wide passes for every flush (VS_WIDE_MIN=1) against the default.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
S="--share 3/8 --per-gpu-gib 32"
L="base=,wmin1=volsync_amd/lib/var/wmin1/libvsgpu.so"
bash tools/c4_walkprof.sh $S > gpurun_out/walkprof_share.txt 2>&1 &&
cp gpurun_out/bench_walkprof.log gpurun_out/bench_walkprof_share.log &&
bash tools/c4_walkprof.sh > gpurun_out/walkprof_c4.txt 2>&1 &&
cp gpurun_out/bench_walkprof.log gpurun_out/bench_walkprof_c4.log &&
bash tools/gpu.sh prof r04_c4share rs_walk --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum &&
timeout -k 10 300 python3 -u tools/ab.py --rounds 2 --libs $L -- bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum > gpurun_out/ab4_share.log 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --rounds 2 --libs $L -- bench.py --mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline > gpurun_out/ab4_c4.log 2>&1 &&
python3 tools/ab_table.py gpurun_out/ab4_share.log gpurun_out/ab4_c4.log | tee gpurun_out/ab4_table.txt
