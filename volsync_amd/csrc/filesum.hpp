// filesum.hpp -- the host half of rsync's whole-file checksum (R7) shared by
// the HIP sources and filesum_host.cpp (plain g++: no HIP headers here).
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace vsgpu {

// host: the XXH3 scramble chain over nb contribution rows (AVX-512 when the
// CPU has it); the last partial block, last stripe and merge from the file's
// last min(len, 1088) bytes -> sum_end's 16 bytes
void xxh3_init_acc(uint64_t acc[8]);
void xxh3_chain_rows(const uint64_t *C, uint64_t nb, uint64_t acc[8]);
void xxh3_file_finish(const uint8_t *last, uint64_t len, const uint64_t acc[8], int csum_type,
                      uint8_t out[16]);
const char *xxh3_chain_isa();

// the serial file sums (MD5, XXH64 with seed 0, XXH3 of <= 240 bytes), fed
// in file order in pieces of any size
struct SerialSum {
    int type;
    uint32_t nbuf, nsmall;
    uint64_t total;
    uint32_t md5[4];
    uint64_t v[4];
    uint8_t buf[64];
    uint8_t small[240];
};
void serial_sum_init(SerialSum &s, int type);
void serial_sum_update(SerialSum &s, const uint8_t *p, size_t n);
void serial_sum_final(SerialSum &s, uint8_t out[16]);

}  // namespace vsgpu
