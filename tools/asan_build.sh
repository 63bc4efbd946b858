#!/bin/bash
# Sanitizer build of the host-side C/C++: the product
# library's host code (wire.cpp token/sum parsers, filesum_host.cpp, xfer.cpp,
# rabin_host.cpp and the host parts of every .hip file) and the C oracle, with
# AddressSanitizer + UndefinedBehaviorSanitizer, then the CPU test suite run
# against them.  Host only: the device code is built as usual (GPU sanitizers
# are not available on the pool), and nothing here runs on a GPU.
#   bash tools/asan_build.sh            build + pytest -m "not gpu" -> profiles/r05_asan/
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
cd "$root"
LLVM=/opt/rocm/lib/llvm
RT=$(ls $LLVM/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
SAN="-fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined"
HSAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer -Xarch_host -fno-sanitize-recover=undefined"
out=volsync_amd/lib/var/asan
make -s -C volsync_amd/csrc -j8 OUT="../lib/var/asan" CXX=$LLVM/bin/clang++ \
  FLAGS="-O1 -g -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950 -Wall -Wno-unused-function $HSAN" \
  HOST_FLAGS="-O1 -g -std=c++17 -fPIC -fvisibility=hidden -Wall -Wno-unknown-pragmas $SAN"
make -s -C oracle OUT=build_asan CC=$LLVM/bin/clang CFLAGS="-O1 -g -fPIC -Wall -std=c11 -D_GNU_SOURCE $SAN"
mkdir -p profiles/r05_asan
log=profiles/r05_asan/pytest_not_gpu.log
echo "runtime: $RT" > "$log"
echo "library: $out/libvsgpu.so  oracle: oracle/build_asan/liboracle.so  flags: $SAN" >> "$log"
set +e
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  VSGPU_LIB=$root/$out/libvsgpu.so VSGPU_ORACLE_LIB=$root/oracle/build_asan/liboracle.so \
  timeout -k 10 3000 python -m pytest tests/ -q -m "not gpu" -p no:cacheprovider "$@" >> "$log" 2>&1
rc=$?
tail -n 5 "$log"
grep -c "ERROR: AddressSanitizer\|runtime error:" "$log" | sed 's/^/sanitizer reports: /'
exit $rc
