#!/bin/bash
# Register-budget variants of the wide flush (tools/build_variant.sh d4sk
# -DVS_WIDE_D=4 -DVS_WIDE_SK_LDS=1; sklds -DVS_WIDE_SK_LDS=1), interleaved on
# one box (tools/ab.py) at one rank of the real C4 and the 64 GiB shape, plus
# the four-window flush under each build.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
L="base=,d4sk=volsync_amd/lib/var/d4sk/libvsgpu.so,sklds=volsync_amd/lib/var/sklds/libvsgpu.so"
S="--mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum"
C="--mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline"
timeout -k 10 500 python3 -u tools/ab.py --rounds 2 --libs $L -- bench.py $S > gpurun_out/ab3_share.log 2>&1 &&
timeout -k 10 500 python3 -u tools/ab.py --rounds 2 --libs $L -- bench.py $C > gpurun_out/ab3_c4.log 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --rounds 1 --libs $L -- bench.py $S --walk-opt walk_flush_windows=4 > gpurun_out/ab3_share_q4.log 2>&1 || exit $?
python3 tools/ab_table.py gpurun_out/ab3_share.log gpurun_out/ab3_c4.log gpurun_out/ab3_share_q4.log | tee gpurun_out/ab3_table.txt
