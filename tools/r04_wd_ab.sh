#!/bin/bash
# Wide-flush lookahead A/B (KiB in flight per wave: 8 = default, 4; 12 does not unroll),
# interleaved on one box at one rank of the real C4 and the 64 GiB shape.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
L="wd4=volsync_amd/lib/var/wd4/libvsgpu.so,wd2=volsync_amd/lib/var/wd2/libvsgpu.so,wd6=volsync_amd/lib/var/wd6/libvsgpu.so"
timeout -k 10 400 python3 -u tools/ab.py --rounds 2 --libs $L -- bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum > gpurun_out/ab_wd2_share.log 2>&1 &&
timeout -k 10 400 python3 -u tools/ab.py --rounds 2 --libs $L -- bench.py --mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline > gpurun_out/ab_wd2_c4.log 2>&1 || exit $?
python3 tools/ab_table.py gpurun_out/ab_wd2_share.log gpurun_out/ab_wd2_c4.log | tee gpurun_out/ab_wd2_table.txt
