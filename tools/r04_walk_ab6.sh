#!/bin/bash
# STEP-side A/B at one rank of the real C4 (interleaved, one box): the blocked
# filter capped at 2^24 bits (tools/build_variant.sh fb24 -DVS_FBITS_CAP=24u),
# half the membership buckets, no LDS prefilter.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
S="--mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum"
L="base=,fb24=volsync_amd/lib/var/fb24/libvsgpu.so"
timeout -k 10 300 python3 -u tools/ab.py --rounds 2 --libs $L -- bench.py $S > gpurun_out/ab6_fb.log 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --rounds 2 --libs base= -- bench.py $S --walk-opt bucket_bits=19 > gpurun_out/ab6_bb19.log 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --rounds 2 --libs base= -- bench.py $S --walk-opt walk_prefilter=0 > gpurun_out/ab6_nopf.log 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --rounds 2 --libs $L -- bench.py --mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline > gpurun_out/ab6_c4_fb.log 2>&1 || exit $?
python3 tools/ab_table.py gpurun_out/ab6_*.log | tee gpurun_out/ab6_table.txt
