// filesum_host.cpp -- the serial half of rsync's whole-file XXH3 (R7,
// checksum.c sum_update/sum_end over the file): the scramble chain over the
// per-block contributions the device computed (filesum.hip), and the tail.
//
// Per 1 KiB block and accumulator: acc = P32_1 * (u ^ (u >> 47) ^ secret),
// u = acc + contribution.  Each accumulator is a serial chain; the eight are
// independent, so one 512-bit register holds all of them and a block costs
// add -> shift -> ternary-xor -> multiply of latency.
//
// Plain host C++ (built with g++, not -x hip): strong.hpp's secret table is
// __constant__ in a HIP compile, whose host shadow is not the data.
#include <immintrin.h>
#include <stdint.h>

#include <cstring>

#include "strong.hpp"

namespace vsgpu {

using namespace vsstrong;

void xxh3_init_acc(uint64_t acc[8]) {
    Xxh3Long st;
    st.init();
    memcpy(acc, st.acc, 64);
}

namespace {

__attribute__((target("avx512f,avx512dq"))) void chain_avx512dq(const uint64_t *C, uint64_t nb,
                                                                 uint64_t acc[8]) {
    __m512i a = _mm512_loadu_si512(acc);
    const __m512i sec = _mm512_loadu_si512(kSecret64 + 16);
    const __m512i p = _mm512_set1_epi64(P32_1);
    for (uint64_t b = 0; b < nb; ++b) {
        const __m512i u = _mm512_add_epi64(a, _mm512_loadu_si512(C + 8 * b));
        const __m512i x = _mm512_ternarylogic_epi64(u, _mm512_srli_epi64(u, 47), sec, 0x96);
        a = _mm512_mullo_epi64(x, p);
    }
    _mm512_storeu_si512(acc, a);
}

// AVX-512F without DQ: x * P32_1 = lo32(x) * P + (hi32(x) * P << 32)
__attribute__((target("avx512f"))) void chain_avx512f(const uint64_t *C, uint64_t nb,
                                                      uint64_t acc[8]) {
    __m512i a = _mm512_loadu_si512(acc);
    const __m512i sec = _mm512_loadu_si512(kSecret64 + 16);
    const __m512i p = _mm512_set1_epi64(P32_1);
    for (uint64_t b = 0; b < nb; ++b) {
        const __m512i u = _mm512_add_epi64(a, _mm512_loadu_si512(C + 8 * b));
        const __m512i x = _mm512_ternarylogic_epi64(u, _mm512_srli_epi64(u, 47), sec, 0x96);
        const __m512i lo = _mm512_mul_epu32(x, p);
        const __m512i hi = _mm512_mul_epu32(_mm512_srli_epi64(x, 32), p);
        a = _mm512_add_epi64(lo, _mm512_slli_epi64(hi, 32));
    }
    _mm512_storeu_si512(acc, a);
}

void chain_scalar(const uint64_t *C, uint64_t nb, uint64_t acc[8]) {
    uint64_t a[8];
    for (int j = 0; j < 8; ++j) a[j] = acc[j];
    for (uint64_t b = 0; b < nb; ++b)
        for (int j = 0; j < 8; ++j) {
            const uint64_t u = a[j] + C[8 * b + j];
            a[j] = (u ^ (u >> 47) ^ kSecret64[16 + j]) * P32_1;
        }
    for (int j = 0; j < 8; ++j) acc[j] = a[j];
}

enum Isa { kScalar, kAvx512f, kAvx512dq };
Isa isa() {
    static const Isa v = [] {
        __builtin_cpu_init();
        if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq")) return kAvx512dq;
        if (__builtin_cpu_supports("avx512f")) return kAvx512f;
        return kScalar;
    }();
    return v;
}

}  // namespace

const char *xxh3_chain_isa() {
    switch (isa()) {
        case kAvx512dq: return "avx512dq";
        case kAvx512f: return "avx512f";
        default: return "scalar";
    }
}

void xxh3_chain_rows(const uint64_t *C, uint64_t nb, uint64_t acc[8]) {
    switch (isa()) {
        case kAvx512dq: chain_avx512dq(C, nb, acc); break;
        case kAvx512f: chain_avx512f(C, nb, acc); break;
        default: chain_scalar(C, nb, acc);
    }
}

// xxh3_long's end (strong.hpp): the stripes of the last partial block, the
// last stripe (ending at len), the merge.  `last` holds the file's last
// min(len, 1088) bytes; len > 240.
void xxh3_file_finish(const uint8_t *last, uint64_t len, const uint64_t acc[8], int csum_type,
                      uint8_t out[16]) {
    const uint64_t keep = len < 1088 ? len : 1088;
    const uint8_t *p = last - (len - keep);   // indexed by file offset (only the kept bytes)
    Xxh3Long st;
    memcpy(st.acc, acc, 64);
    const uint64_t nb = (len - 1) / 1024;
    const uint32_t ns = (uint32_t)(((len - 1) - nb * 1024) / 64);
    uint64_t d[8];
    for (uint32_t s = 0; s < ns; ++s) {
        load_stripe(d, p + nb * 1024 + 64 * s);
        st.stripe(d, 8 * s, 0);
    }
    load_stripe(d, p + len - 64);
    st.stripe(d, 192 - 64 - 7, 0);
    const uint64_t lo = st.merge(11, len * P64_1, 0);
    const uint64_t hi = csum_type == kXxh3_128 ? st.merge(192 - 64 - 11, ~(len * P64_2), 0) : 0;
    for (int i = 0; i < 8; ++i) {
        out[i] = (uint8_t)(lo >> (8 * i));
        out[8 + i] = (uint8_t)(hi >> (8 * i));
    }
}

}  // namespace vsgpu
