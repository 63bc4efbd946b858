#!/bin/bash
# C2 A/B: SHA-256 producer/consumer roles fixed per wave (default) against
# alternating tile by tile (tools/build_variant.sh shaalt -DVS_SHA_ALTERNATE=1),
# interleaved on one box; then the C5 line under both.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
L="base=,shaalt=volsync_amd/lib/var/shaalt/libvsgpu.so"
timeout -k 10 500 python3 -u tools/ab.py --rounds 3 --libs $L -- bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_sha_c2.log 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --rounds 1 --libs $L -- bench.py --mode smallfiles --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_sha_c5.log 2>&1 || exit $?
python3 tools/ab_table.py gpurun_out/ab_sha_c2.log gpurun_out/ab_sha_c5.log | tee gpurun_out/ab_sha_table.txt
