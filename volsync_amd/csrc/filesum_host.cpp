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

#include <algorithm>
#include <cstring>

#include "filesum.hpp"
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

// ---- the serial file sums: MD5, XXH64, XXH3 of <= 240 bytes -----------------
// MD5 and XXH64 are one dependency chain per 64 / 32 bytes (no parallel form),
// and a host core runs such a chain several times faster than a GPU lane, so
// the file's bytes are read back piece by piece (the same pinned D2H ring as
// the XXH3 contributions) and hashed here as they land.
void serial_sum_init(SerialSum &s, int type) {
    memset(&s, 0, sizeof s);
    s.type = type;
    s.md5[0] = 0x67452301u;
    s.md5[1] = 0xefcdab89u;
    s.md5[2] = 0x98badcfeu;
    s.md5[3] = 0x10325476u;
    s.v[0] = P64_1 + P64_2;   // XXH64, seed 0 (sum_init seeds no file sum)
    s.v[1] = P64_2;
    s.v[2] = 0;
    s.v[3] = 0 - P64_1;
}

namespace {
void md5_eat(SerialSum &s, const uint8_t *p) {
    uint32_t x[16];
    for (int i = 0; i < 16; ++i) x[i] = rd32(p + 4 * i);
    md5_block(s.md5, x);
}
void xxh64_eat(SerialSum &s, const uint8_t *p) {
    s.v[0] = xxh64_round(s.v[0], rd64(p));
    s.v[1] = xxh64_round(s.v[1], rd64(p + 8));
    s.v[2] = xxh64_round(s.v[2], rd64(p + 16));
    s.v[3] = xxh64_round(s.v[3], rd64(p + 24));
}
}  // namespace

void serial_sum_update(SerialSum &s, const uint8_t *p, size_t n) {
    const uint32_t bs = s.type == kMd5 ? 64 : 32;
    s.total += n;
    if (s.type != kMd5 && s.type != kXxh64) {   // XXH3 <= 240 bytes: kept whole
        const size_t k = std::min<size_t>(n, sizeof s.small - s.nsmall);
        memcpy(s.small + s.nsmall, p, k);
        s.nsmall += (uint32_t)k;
        return;
    }
    if (s.nbuf) {
        const size_t k = std::min<size_t>(n, bs - s.nbuf);
        memcpy(s.buf + s.nbuf, p, k);
        s.nbuf += (uint32_t)k;
        p += k;
        n -= k;
        if (s.nbuf < bs) return;
        if (s.type == kMd5) md5_eat(s, s.buf);
        else xxh64_eat(s, s.buf);
        s.nbuf = 0;
    }
    if (s.type == kMd5) {
        for (; n >= 64; p += 64, n -= 64) md5_eat(s, p);
    } else {
        for (; n >= 32; p += 32, n -= 32) xxh64_eat(s, p);
    }
    memcpy(s.buf, p, n);
    s.nbuf = (uint32_t)n;
}

void serial_sum_final(SerialSum &s, uint8_t out[16]) {
    memset(out, 0, 16);
    if (s.type == kMd5) {
        uint8_t pad[128];
        const uint64_t bits = s.total * 8;
        const uint32_t n = s.nbuf, padn = (n < 56 ? 64 : 128);
        memcpy(pad, s.buf, n);
        pad[n] = 0x80;
        memset(pad + n + 1, 0, padn - n - 1);
        for (int i = 0; i < 8; ++i) pad[padn - 8 + i] = (uint8_t)(bits >> (8 * i));
        md5_eat(s, pad);
        if (padn == 128) md5_eat(s, pad + 64);
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) out[4 * i + j] = (uint8_t)(s.md5[i] >> (8 * j));
        return;
    }
    if (s.type == kXxh64) {
        uint64_t h;
        if (s.total >= 32) {
            h = rotl64(s.v[0], 1) + rotl64(s.v[1], 7) + rotl64(s.v[2], 12) + rotl64(s.v[3], 18);
            for (int i = 0; i < 4; ++i) h = xxh64_merge(h, s.v[i]);
        } else {
            h = P64_5;
        }
        h += s.total;
        const uint8_t *p = s.buf;
        uint32_t left = s.nbuf;
        for (; left >= 8; p += 8, left -= 8) {
            h ^= xxh64_round(0, rd64(p));
            h = rotl64(h, 27) * P64_1 + P64_4;
        }
        if (left >= 4) {
            h ^= (uint64_t)rd32(p) * P64_1;
            h = rotl64(h, 23) * P64_2 + P64_3;
            p += 4;
            left -= 4;
        }
        for (; left; ++p, --left) {
            h ^= (*p) * P64_5;
            h = rotl64(h, 11) * P64_1;
        }
        h = xxh64_aval(h);
        for (int i = 0; i < 8; ++i) out[i] = (uint8_t)(h >> (8 * i));
        return;
    }
    uint8_t o[16];   // XXH3 of <= 240 bytes
    checksum2(s.small, s.nsmall, s.type, 0, o);
    memcpy(out, o, s.type == kXxh3_128 ? 16 : 8);
}

}  // namespace vsgpu
