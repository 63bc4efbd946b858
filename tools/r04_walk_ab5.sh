#!/bin/bash
# Wide flush stripe reads: unaligned ds_read_b128 (default) against five
# aligned dwords + v_alignbyte (tools/build_variant.sh aligned
# -DVS_WIDE_ALIGNED=1), interleaved on one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
L="base=,aligned=volsync_amd/lib/var/aligned/libvsgpu.so"
timeout -k 10 300 python3 -u tools/ab.py --rounds 2 --libs $L -- bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum > gpurun_out/ab5_share.log 2>&1 &&
timeout -k 10 300 python3 -u tools/ab.py --rounds 2 --libs $L -- bench.py --mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline > gpurun_out/ab5_c4.log 2>&1 || exit $?
python3 tools/ab_table.py gpurun_out/ab5_share.log gpurun_out/ab5_c4.log | tee gpurun_out/ab5_table.txt &&
bash tools/gpu.sh prof r04_c4 rs_walk --mode rsync --steps 3 --warmup 1 --no-file-sum
