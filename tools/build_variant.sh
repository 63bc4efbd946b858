#!/bin/bash
# Build an A/B variant of the product library with extra -D flags into
# volsync_amd/lib/var/<name>/libvsgpu.so (select it with VSGPU_LIB=...).
#   tools/build_variant.sh fp_base -DVS_FP_FASTOPS=0
set -e
name=$1
shift
root=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$root/volsync_amd/csrc" -j8 OUT="../lib/var/$name" \
  FLAGS="-O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950 -Wall -Wno-unused-function $*"
echo "$root/volsync_amd/lib/var/$name/libvsgpu.so"
