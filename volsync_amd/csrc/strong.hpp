// strong.hpp -- rsync 3.2.3 strong block sums (get_checksum2) for one lane.
//
// the negotiated xfersum is XXH3-128 with the 32-bit
// checksum_seed for rsync 3.2.3 <-> 3.2.3 (stored LE low64 then LE high64),
// alternatives XXH3-64, XXH64 and MD5 (seed prepended as LE u32 when it is
// non-zero, proper_seed_order).  Only the first s2length bytes are compared.
// The xxhash algorithms restate the published xxHash 0.8 specification
// (XXH3_64bits_withSeed / XXH3_128bits_withSeed / XXH64; libxxhash 0.8.x,
// pinned in tests against the `xxhash` package); MD5 restates RFC 1321.
//
// Header-only and compiled twice: by hipcc for the device kernels (rsync.hip)
// and by g++ for the CPU self-test library under tests/native (which checks the
// restatement against xxhash / hashlib without a GPU).  Plain 64-bit integer
// code: on gfx950 a 64x64->128 product is v_mad_u64_u32 chains, no MFMA.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define VS_HD __host__ __device__ __forceinline__
#define VS_HM __host__ __device__ __forceinline__
#else
#define VS_HD static inline
#define VS_HM inline
#endif

namespace vsstrong {

enum : int { kMd5 = 5, kXxh64 = 6, kXxh3_64 = 7, kXxh3_128 = 8 };

constexpr uint32_t P32_1 = 0x9E3779B1u, P32_2 = 0x85EBCA77u, P32_3 = 0xC2B2AE3Du;
constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ull, P64_2 = 0xC2B2AE3D27D4EB4Full,
                   P64_3 = 0x165667B19E3779F9ull, P64_4 = 0x85EBCA77C2B2AE63ull,
                   P64_5 = 0x27D4EB2F165667C5ull;
constexpr uint64_t PMX_1 = 0x165667919E3779F9ull, PMX_2 = 0x9FB21C651E98DF25ull;

// XXH3 default secret (192 bytes) as little-endian u64 words
#if defined(__HIPCC__)
__device__ __constant__
#endif
static const uint64_t kSecret64[24] = {
    0xbe4ba423396cfeb8ull, 0x1cad21f72c81017cull, 0xdb979083e96dd4deull, 0x1f67b3b7a4a44072ull,
    0x78e5c0cc4ee679cbull, 0x2172ffcc7dd05a82ull, 0x8e2443f7744608b8ull, 0x4c263a81e69035e0ull,
    0xcb00c391bb52283cull, 0xa32e531b8b65d088ull, 0x4ef90da297486471ull, 0xd8acdea946ef1938ull,
    0x3f349ce33f76faa8ull, 0x1d4f0bc7c7bbdcf9ull, 0x3159b4cd4be0518aull, 0x647378d9c97e9fc8ull,
    0xc3ebd33483acc5eaull, 0xeb6313faffa081c5ull, 0x49daf0b751dd0d17ull, 0x9e68d429265516d3ull,
    0xfca1477d58be162bull, 0xce31d07ad1b8f88full, 0x280416958f3acb45ull, 0x7e404bbbcafbd7afull,
};

struct U128 {
    uint64_t lo, hi;
};

VS_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
VS_HD uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
VS_HD uint32_t swap32(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}
VS_HD uint64_t swap64(uint64_t x) {
    return ((uint64_t)swap32((uint32_t)x) << 32) | swap32((uint32_t)(x >> 32));
}
VS_HD uint64_t rd64(const uint8_t *p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}
VS_HD uint32_t rd32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
VS_HD U128 mul128(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return {a * b, __umul64hi(a, b)};
#else
    const unsigned __int128 r = (unsigned __int128)a * b;
    return {(uint64_t)r, (uint64_t)(r >> 64)};
#endif
}
VS_HD uint64_t fold64(uint64_t a, uint64_t b) {
    const U128 r = mul128(a, b);
    return r.lo ^ r.hi;
}

// secret word i (byte offset 8*i) of the default secret, or of the seeded
// custom secret (XXH3_initCustomSecret): even words + seed, odd words - seed
VS_HD uint64_t sec64(uint32_t i, uint64_t seed) {
    const uint64_t k = kSecret64[i];
    return (i & 1) ? k - seed : k + seed;
}
// unaligned 64-bit read of the default secret at byte offset b
VS_HD uint64_t ksec_at(uint32_t b) {
    const uint32_t w = b >> 3, r = (b & 7) * 8;
    if (!r) return kSecret64[w];
    return (kSecret64[w] >> r) | (kSecret64[w + 1] << (64 - r));
}
VS_HD uint32_t ksec32_at(uint32_t b) { return (uint32_t)ksec_at(b); }
// unaligned 64-bit read of the seeded custom secret at byte offset b
VS_HD uint64_t csec_at(uint32_t b, uint64_t seed) {
    const uint32_t w = b >> 3, r = (b & 7) * 8;
    const uint64_t a = sec64(w, seed);
    if (!r) return a;
    return (a >> r) | (sec64(w + 1, seed) << (64 - r));
}

// ---- XXH64 -------------------------------------------------------------------
VS_HD uint64_t xxh64_round(uint64_t acc, uint64_t in) {
    acc += in * P64_2;
    acc = rotl64(acc, 31);
    return acc * P64_1;
}
VS_HD uint64_t xxh64_merge(uint64_t acc, uint64_t v) {
    acc ^= xxh64_round(0, v);
    return acc * P64_1 + P64_4;
}
VS_HD uint64_t xxh64_aval(uint64_t h) {
    h ^= h >> 33;
    h *= P64_2;
    h ^= h >> 29;
    h *= P64_3;
    h ^= h >> 32;
    return h;
}
VS_HD uint64_t xxh64(const uint8_t *p, uint64_t len, uint64_t seed) {
    const uint8_t *const end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = seed + P64_1 + P64_2, v2 = seed + P64_2, v3 = seed, v4 = seed - P64_1;
        const uint8_t *const lim = end - 32;
        do {
            v1 = xxh64_round(v1, rd64(p));
            v2 = xxh64_round(v2, rd64(p + 8));
            v3 = xxh64_round(v3, rd64(p + 16));
            v4 = xxh64_round(v4, rd64(p + 24));
            p += 32;
        } while (p <= lim);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xxh64_merge(h, v1);
        h = xxh64_merge(h, v2);
        h = xxh64_merge(h, v3);
        h = xxh64_merge(h, v4);
    } else {
        h = seed + P64_5;
    }
    h += len;
    uint64_t left = len & 31;
    while (left >= 8) {
        h ^= xxh64_round(0, rd64(p));
        h = rotl64(h, 27) * P64_1 + P64_4;
        p += 8;
        left -= 8;
    }
    if (left >= 4) {
        h ^= (uint64_t)rd32(p) * P64_1;
        h = rotl64(h, 23) * P64_2 + P64_3;
        p += 4;
        left -= 4;
    }
    while (left > 0) {
        h ^= (*p) * P64_5;
        h = rotl64(h, 11) * P64_1;
        ++p;
        --left;
    }
    return xxh64_aval(h);
}

// ---- XXH3 common -------------------------------------------------------------
VS_HD uint64_t xxh3_aval(uint64_t h) {
    h ^= h >> 37;
    h *= PMX_1;
    h ^= h >> 32;
    return h;
}
VS_HD uint64_t rrmxmx(uint64_t h, uint64_t len) {
    h ^= rotl64(h, 49) ^ rotl64(h, 24);
    h *= PMX_2;
    h ^= (h >> 35) + len;
    h *= PMX_2;
    return h ^ (h >> 28);
}
// mix16B with the default secret at byte offset sb
VS_HD uint64_t mix16(const uint8_t *in, uint32_t sb, uint64_t seed) {
    return fold64(rd64(in) ^ (ksec_at(sb) + seed), rd64(in + 8) ^ (ksec_at(sb + 8) - seed));
}

// long-input accumulator state (hashLong, > 240 bytes): 8 lanes, stripes of
// 64 bytes, a scramble every 16 stripes; secret = seeded custom secret
struct Xxh3Long {
    uint64_t acc[8];
    VS_HM void init() {
        acc[0] = P32_3;
        acc[1] = P64_1;
        acc[2] = P64_2;
        acc[3] = P64_3;
        acc[4] = P64_4;
        acc[5] = P32_2;
        acc[6] = P64_5;
        acc[7] = P32_1;
    }
    // one 64-byte stripe; d = its 8 words, secret words at byte offset sb (8-aligned
    // for stripes n*8, 7 mod 8 for the last stripe: handled by csec_at)
    VS_HM void stripe(const uint64_t (&d)[8], uint32_t sb, uint64_t seed) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint64_t k = d[i] ^ csec_at(sb + 8 * i, seed);
            acc[i ^ 1] += d[i];
            acc[i] += (uint64_t)(uint32_t)k * (k >> 32);
        }
    }
    VS_HM void scramble(uint64_t seed) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            uint64_t a = acc[i];
            a ^= a >> 47;
            a ^= sec64(16 + i, seed);  // secret + 192 - 64
            acc[i] = a * P32_1;
        }
    }
    VS_HM uint64_t merge(uint32_t sb, uint64_t start, uint64_t seed) const {
        uint64_t r = start;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            r += fold64(acc[2 * i] ^ csec_at(sb + 16 * i, seed),
                        acc[2 * i + 1] ^ csec_at(sb + 16 * i + 8, seed));
        return xxh3_aval(r);
    }
};

VS_HD void load_stripe(uint64_t (&d)[8], const uint8_t *p) {
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = rd64(p + 8 * i);
}

VS_HD void xxh3_long(Xxh3Long &st, const uint8_t *p, uint64_t len, uint64_t seed) {
    st.init();
    const uint64_t nb = (len - 1) / 1024;
    uint64_t d[8];
    for (uint64_t b = 0; b < nb; ++b) {
        for (uint32_t s = 0; s < 16; ++s) {
            load_stripe(d, p + b * 1024 + s * 64);
            st.stripe(d, s * 8, seed);
        }
        st.scramble(seed);
    }
    const uint32_t ns = (uint32_t)(((len - 1) - nb * 1024) / 64);
    for (uint32_t s = 0; s < ns; ++s) {
        load_stripe(d, p + nb * 1024 + s * 64);
        st.stripe(d, s * 8, seed);
    }
    load_stripe(d, p + len - 64);
    st.stripe(d, 192 - 64 - 7, seed);
}

// ---- XXH3-64 with seed ---------------------------------------------------------
VS_HD uint64_t xxh3_64(const uint8_t *p, uint64_t len, uint64_t seed) {
    if (len <= 16) {
        if (len > 8) {
            const uint64_t f1 = (ksec_at(24) ^ ksec_at(32)) + seed;
            const uint64_t f2 = (ksec_at(40) ^ ksec_at(48)) - seed;
            const uint64_t lo = rd64(p) ^ f1, hi = rd64(p + len - 8) ^ f2;
            return xxh3_aval(len + swap64(lo) + hi + fold64(lo, hi));
        }
        if (len >= 4) {
            const uint64_t s = seed ^ ((uint64_t)swap32((uint32_t)seed) << 32);
            const uint32_t in1 = rd32(p), in2 = rd32(p + len - 4);
            const uint64_t f = (ksec_at(8) ^ ksec_at(16)) - s;
            return rrmxmx(((uint64_t)in2 + ((uint64_t)in1 << 32)) ^ f, len);
        }
        if (len > 0) {
            const uint32_t c = ((uint32_t)p[0] << 16) | ((uint32_t)p[len >> 1] << 24) |
                               (uint32_t)p[len - 1] | ((uint32_t)len << 8);
            const uint64_t f = (uint64_t)(ksec32_at(0) ^ ksec32_at(4)) + seed;
            return xxh64_aval((uint64_t)c ^ f);
        }
        return xxh64_aval(seed ^ (ksec_at(56) ^ ksec_at(64)));
    }
    if (len <= 128) {
        uint64_t acc = len * P64_1;
        if (len > 32) {
            if (len > 64) {
                if (len > 96) {
                    acc += mix16(p + 48, 96, seed);
                    acc += mix16(p + len - 64, 112, seed);
                }
                acc += mix16(p + 32, 64, seed);
                acc += mix16(p + len - 48, 80, seed);
            }
            acc += mix16(p + 16, 32, seed);
            acc += mix16(p + len - 32, 48, seed);
        }
        acc += mix16(p, 0, seed);
        acc += mix16(p + len - 16, 16, seed);
        return xxh3_aval(acc);
    }
    if (len <= 240) {
        const uint32_t rounds = (uint32_t)len / 16;
        uint64_t acc = len * P64_1;
        for (uint32_t i = 0; i < 8; ++i) acc += mix16(p + 16 * i, 16 * i, seed);
        acc = xxh3_aval(acc);
        for (uint32_t i = 8; i < rounds; ++i) acc += mix16(p + 16 * i, 16 * (i - 8) + 3, seed);
        acc += mix16(p + len - 16, 136 - 17, seed);
        return xxh3_aval(acc);
    }
    Xxh3Long st;
    xxh3_long(st, p, len, seed);
    return st.merge(11, len * P64_1, seed);
}

// ---- XXH3-128 with seed --------------------------------------------------------
VS_HD void mix32(U128 &acc, const uint8_t *a, const uint8_t *b, uint32_t sb, uint64_t seed) {
    acc.lo += mix16(a, sb, seed);
    acc.lo ^= rd64(b) + rd64(b + 8);
    acc.hi += mix16(b, sb + 16, seed);
    acc.hi ^= rd64(a) + rd64(a + 8);
}
VS_HD U128 fin128(U128 acc, uint64_t len, uint64_t seed) {
    U128 h;
    h.lo = acc.lo + acc.hi;
    h.hi = acc.lo * P64_1 + acc.hi * P64_4 + (len - seed) * P64_2;
    h.lo = xxh3_aval(h.lo);
    h.hi = 0 - xxh3_aval(h.hi);
    return h;
}

VS_HD U128 xxh3_128(const uint8_t *p, uint64_t len, uint64_t seed) {
    if (len <= 16) {
        if (len > 8) {
            const uint64_t fl = (ksec_at(32) ^ ksec_at(40)) - seed;
            const uint64_t fh = (ksec_at(48) ^ ksec_at(56)) + seed;
            const uint64_t ilo = rd64(p);
            uint64_t ihi = rd64(p + len - 8);
            U128 m = mul128(ilo ^ ihi ^ fl, P64_1);
            m.lo += (uint64_t)(len - 1) << 54;
            ihi ^= fh;
            m.hi += ihi + (uint64_t)(uint32_t)ihi * (uint64_t)(P32_2 - 1);
            m.lo ^= swap64(m.hi);
            U128 h = mul128(m.lo, P64_2);
            h.hi += m.hi * P64_2;
            return {xxh3_aval(h.lo), xxh3_aval(h.hi)};
        }
        if (len >= 4) {
            const uint64_t s = seed ^ ((uint64_t)swap32((uint32_t)seed) << 32);
            const uint32_t ilo = rd32(p), ihi = rd32(p + len - 4);
            const uint64_t i64 = (uint64_t)ilo + ((uint64_t)ihi << 32);
            const uint64_t f = (ksec_at(16) ^ ksec_at(24)) + s;
            U128 m = mul128(i64 ^ f, P64_1 + (len << 2));
            m.hi += m.lo << 1;
            m.lo ^= m.hi >> 3;
            m.lo ^= m.lo >> 35;
            m.lo *= PMX_2;
            m.lo ^= m.lo >> 28;
            m.hi = xxh3_aval(m.hi);
            return m;
        }
        if (len > 0) {
            const uint32_t cl = ((uint32_t)p[0] << 16) | ((uint32_t)p[len >> 1] << 24) |
                                (uint32_t)p[len - 1] | ((uint32_t)len << 8);
            const uint32_t ch = rotl32(swap32(cl), 13);
            const uint64_t fl = (uint64_t)(ksec32_at(0) ^ ksec32_at(4)) + seed;
            const uint64_t fh = (uint64_t)(ksec32_at(8) ^ ksec32_at(12)) - seed;
            return {xxh64_aval((uint64_t)cl ^ fl), xxh64_aval((uint64_t)ch ^ fh)};
        }
        return {xxh64_aval(seed ^ (ksec_at(64) ^ ksec_at(72))),
                xxh64_aval(seed ^ (ksec_at(80) ^ ksec_at(88)))};
    }
    if (len <= 128) {
        U128 acc{len * P64_1, 0};
        if (len > 32) {
            if (len > 64) {
                if (len > 96) mix32(acc, p + 48, p + len - 64, 96, seed);
                mix32(acc, p + 32, p + len - 48, 64, seed);
            }
            mix32(acc, p + 16, p + len - 32, 32, seed);
        }
        mix32(acc, p, p + len - 16, 0, seed);
        return fin128(acc, len, seed);
    }
    if (len <= 240) {
        const uint32_t rounds = (uint32_t)len / 32;
        U128 acc{len * P64_1, 0};
        for (uint32_t i = 0; i < 4; ++i) mix32(acc, p + 32 * i, p + 32 * i + 16, 32 * i, seed);
        acc.lo = xxh3_aval(acc.lo);
        acc.hi = xxh3_aval(acc.hi);
        for (uint32_t i = 4; i < rounds; ++i)
            mix32(acc, p + 32 * i, p + 32 * i + 16, 3 + 32 * (i - 4), seed);
        mix32(acc, p + len - 16, p + len - 32, 136 - 17 - 16, 0 - seed);
        return fin128(acc, len, seed);
    }
    Xxh3Long st;
    xxh3_long(st, p, len, seed);
    return {st.merge(11, len * P64_1, seed), st.merge(192 - 64 - 11, ~(len * P64_2), seed)};
}

// ---- MD5 (RFC 1321), rsync seed prefix ------------------------------------------
VS_HD void md5_block(uint32_t (&h)[4], const uint32_t (&x)[16]) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
#define VS_MD5_STEP(F, a, b, c, d, k, s, t)                       \
    {                                                             \
        a += F(b, c, d) + x[k] + (t);                             \
        a = rotl32(a, s) + b;                                     \
    }
#define VS_F(b, c, d) ((d) ^ ((b) & ((c) ^ (d))))
#define VS_G(b, c, d) ((c) ^ ((d) & ((b) ^ (c))))
#define VS_H(b, c, d) ((b) ^ (c) ^ (d))
#define VS_I(b, c, d) ((c) ^ ((b) | ~(d)))
    VS_MD5_STEP(VS_F, a, b, c, d, 0, 7, 0xd76aa478u)
    VS_MD5_STEP(VS_F, d, a, b, c, 1, 12, 0xe8c7b756u)
    VS_MD5_STEP(VS_F, c, d, a, b, 2, 17, 0x242070dbu)
    VS_MD5_STEP(VS_F, b, c, d, a, 3, 22, 0xc1bdceeeu)
    VS_MD5_STEP(VS_F, a, b, c, d, 4, 7, 0xf57c0fafu)
    VS_MD5_STEP(VS_F, d, a, b, c, 5, 12, 0x4787c62au)
    VS_MD5_STEP(VS_F, c, d, a, b, 6, 17, 0xa8304613u)
    VS_MD5_STEP(VS_F, b, c, d, a, 7, 22, 0xfd469501u)
    VS_MD5_STEP(VS_F, a, b, c, d, 8, 7, 0x698098d8u)
    VS_MD5_STEP(VS_F, d, a, b, c, 9, 12, 0x8b44f7afu)
    VS_MD5_STEP(VS_F, c, d, a, b, 10, 17, 0xffff5bb1u)
    VS_MD5_STEP(VS_F, b, c, d, a, 11, 22, 0x895cd7beu)
    VS_MD5_STEP(VS_F, a, b, c, d, 12, 7, 0x6b901122u)
    VS_MD5_STEP(VS_F, d, a, b, c, 13, 12, 0xfd987193u)
    VS_MD5_STEP(VS_F, c, d, a, b, 14, 17, 0xa679438eu)
    VS_MD5_STEP(VS_F, b, c, d, a, 15, 22, 0x49b40821u)
    VS_MD5_STEP(VS_G, a, b, c, d, 1, 5, 0xf61e2562u)
    VS_MD5_STEP(VS_G, d, a, b, c, 6, 9, 0xc040b340u)
    VS_MD5_STEP(VS_G, c, d, a, b, 11, 14, 0x265e5a51u)
    VS_MD5_STEP(VS_G, b, c, d, a, 0, 20, 0xe9b6c7aau)
    VS_MD5_STEP(VS_G, a, b, c, d, 5, 5, 0xd62f105du)
    VS_MD5_STEP(VS_G, d, a, b, c, 10, 9, 0x02441453u)
    VS_MD5_STEP(VS_G, c, d, a, b, 15, 14, 0xd8a1e681u)
    VS_MD5_STEP(VS_G, b, c, d, a, 4, 20, 0xe7d3fbc8u)
    VS_MD5_STEP(VS_G, a, b, c, d, 9, 5, 0x21e1cde6u)
    VS_MD5_STEP(VS_G, d, a, b, c, 14, 9, 0xc33707d6u)
    VS_MD5_STEP(VS_G, c, d, a, b, 3, 14, 0xf4d50d87u)
    VS_MD5_STEP(VS_G, b, c, d, a, 8, 20, 0x455a14edu)
    VS_MD5_STEP(VS_G, a, b, c, d, 13, 5, 0xa9e3e905u)
    VS_MD5_STEP(VS_G, d, a, b, c, 2, 9, 0xfcefa3f8u)
    VS_MD5_STEP(VS_G, c, d, a, b, 7, 14, 0x676f02d9u)
    VS_MD5_STEP(VS_G, b, c, d, a, 12, 20, 0x8d2a4c8au)
    VS_MD5_STEP(VS_H, a, b, c, d, 5, 4, 0xfffa3942u)
    VS_MD5_STEP(VS_H, d, a, b, c, 8, 11, 0x8771f681u)
    VS_MD5_STEP(VS_H, c, d, a, b, 11, 16, 0x6d9d6122u)
    VS_MD5_STEP(VS_H, b, c, d, a, 14, 23, 0xfde5380cu)
    VS_MD5_STEP(VS_H, a, b, c, d, 1, 4, 0xa4beea44u)
    VS_MD5_STEP(VS_H, d, a, b, c, 4, 11, 0x4bdecfa9u)
    VS_MD5_STEP(VS_H, c, d, a, b, 7, 16, 0xf6bb4b60u)
    VS_MD5_STEP(VS_H, b, c, d, a, 10, 23, 0xbebfbc70u)
    VS_MD5_STEP(VS_H, a, b, c, d, 13, 4, 0x289b7ec6u)
    VS_MD5_STEP(VS_H, d, a, b, c, 0, 11, 0xeaa127fau)
    VS_MD5_STEP(VS_H, c, d, a, b, 3, 16, 0xd4ef3085u)
    VS_MD5_STEP(VS_H, b, c, d, a, 6, 23, 0x04881d05u)
    VS_MD5_STEP(VS_H, a, b, c, d, 9, 4, 0xd9d4d039u)
    VS_MD5_STEP(VS_H, d, a, b, c, 12, 11, 0xe6db99e5u)
    VS_MD5_STEP(VS_H, c, d, a, b, 15, 16, 0x1fa27cf8u)
    VS_MD5_STEP(VS_H, b, c, d, a, 2, 23, 0xc4ac5665u)
    VS_MD5_STEP(VS_I, a, b, c, d, 0, 6, 0xf4292244u)
    VS_MD5_STEP(VS_I, d, a, b, c, 7, 10, 0x432aff97u)
    VS_MD5_STEP(VS_I, c, d, a, b, 14, 15, 0xab9423a7u)
    VS_MD5_STEP(VS_I, b, c, d, a, 5, 21, 0xfc93a039u)
    VS_MD5_STEP(VS_I, a, b, c, d, 12, 6, 0x655b59c3u)
    VS_MD5_STEP(VS_I, d, a, b, c, 3, 10, 0x8f0ccc92u)
    VS_MD5_STEP(VS_I, c, d, a, b, 10, 15, 0xffeff47du)
    VS_MD5_STEP(VS_I, b, c, d, a, 1, 21, 0x85845dd1u)
    VS_MD5_STEP(VS_I, a, b, c, d, 8, 6, 0x6fa87e4fu)
    VS_MD5_STEP(VS_I, d, a, b, c, 15, 10, 0xfe2ce6e0u)
    VS_MD5_STEP(VS_I, c, d, a, b, 6, 15, 0xa3014314u)
    VS_MD5_STEP(VS_I, b, c, d, a, 13, 21, 0x4e0811a1u)
    VS_MD5_STEP(VS_I, a, b, c, d, 4, 6, 0xf7537e82u)
    VS_MD5_STEP(VS_I, d, a, b, c, 11, 10, 0xbd3af235u)
    VS_MD5_STEP(VS_I, c, d, a, b, 2, 15, 0x2ad7d2bbu)
    VS_MD5_STEP(VS_I, b, c, d, a, 9, 21, 0xeb86d391u)
#undef VS_MD5_STEP
#undef VS_F
#undef VS_G
#undef VS_H
#undef VS_I
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
}

// MD5 of (seed as LE u32 if seed != 0) || buf[0:len) -> 16 bytes
VS_HD void md5_seeded(const uint8_t *p, uint64_t len, uint32_t seed, uint8_t (&out)[16]) {
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    const uint32_t pre = seed ? 4 : 0;
    const uint64_t total = len + pre;  // message bytes
    const uint64_t nblk = (total + 8) / 64 + 1;
    for (uint64_t b = 0; b < nblk; ++b) {
        uint32_t x[16];
        const uint64_t m0 = b * 64;  // message offset of this block
        if (m0 + 64 <= total && m0 >= pre) {
            // fast path: a whole block of data bytes
            const uint8_t *q = p + (m0 - pre);
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = rd32(q + 4 * i);
        } else {
            for (int i = 0; i < 16; ++i) {
                uint32_t w = 0;
                for (int j = 0; j < 4; ++j) {
                    const uint64_t m = m0 + 4 * i + j;
                    uint32_t byte;
                    if (m < pre)
                        byte = (seed >> (8 * m)) & 0xff;
                    else if (m < total)
                        byte = p[m - pre];
                    else if (m == total)
                        byte = 0x80;
                    else
                        byte = 0;
                    w |= byte << (8 * j);
                }
                x[i] = w;
            }
            if (b == nblk - 1) {
                const uint64_t bits = total * 8;
                x[14] = (uint32_t)bits;
                x[15] = (uint32_t)(bits >> 32);
            }
        }
        md5_block(h, x);
    }
    for (int i = 0; i < 4; ++i) {
        out[4 * i + 0] = (uint8_t)h[i];
        out[4 * i + 1] = (uint8_t)(h[i] >> 8);
        out[4 * i + 2] = (uint8_t)(h[i] >> 16);
        out[4 * i + 3] = (uint8_t)(h[i] >> 24);
    }
}

// get_checksum2: 16-byte strong sum in rsync's layout (xxh3/xxh64: LE value,
// zero padded; xxh128: LE low64, LE high64; md5: the digest)
VS_HD void checksum2(const uint8_t *p, uint64_t len, int csum_type, uint32_t seed,
                     uint8_t (&out)[16]) {
    uint64_t lo = 0, hi = 0;
    if (csum_type == kMd5) {
        md5_seeded(p, len, seed, out);
        return;
    }
    if (csum_type == kXxh3_128) {
        const U128 r = xxh3_128(p, len, seed);
        lo = r.lo;
        hi = r.hi;
    } else if (csum_type == kXxh3_64) {
        lo = xxh3_64(p, len, seed);
    } else {
        lo = xxh64(p, len, seed);
    }
    for (int i = 0; i < 8; ++i) {
        out[i] = (uint8_t)(lo >> (8 * i));
        out[8 + i] = (uint8_t)(hi >> (8 * i));
    }
}

}  // namespace vsstrong
