// Host build of volsync_amd/csrc/strong.hpp for the CPU self-test
// (tests/test_strong_host.py).  Test infrastructure: checks the device
// restatement of rsync's strong sums against xxhash / hashlib without a GPU.
#include "../../volsync_amd/csrc/strong.hpp"

extern "C" void strong_host_checksum2(const uint8_t *p, uint64_t len, int csum_type,
                                      uint32_t seed, uint8_t *out16) {
    uint8_t o[16];
    vsstrong::checksum2(p, len, csum_type, seed, o);
    memcpy(out16, o, 16);
}
