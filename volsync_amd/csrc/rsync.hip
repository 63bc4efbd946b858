// rsync.hip -- rsync 3.2.3 delta matching on gfx950.
//
//   R1 weak sum   get_checksum1 over signed bytes: s1 = sum b, s2 = sum (k-j) b_j,
//                 sum = (s1 & 0xffff) | (s2 << 16).  Four bytes per v_dot4c_i32_i8.
//   R2 strong sum get_checksum2 (strong.hpp: XXH3-128/64, XXH64, MD5).
//   R4 signatures one lane per destination block: weak + strong.
//   R5 table      blocks sorted by (sum1 ascending, index descending) -- the
//                 order in which match.c build_hash_table's chains present the
//                 blocks of one weak sum -- plus a bucket directory on the top
//                 bits of sum1 and a bit filter in front of it.
//   R6 scan       every source offset's weak sum: coarse prefix sums give a
//                 lane the window sum at its strip start, the lane then rolls
//                 (hash_search's s1/s2 update) and probes filter -> directory ->
//                 entries; offsets with a block of equal sum1 and length are
//                 appended as candidates.  Strong sums of candidates the greedy
//                 walk visits are computed in batches (rs_strong_kernel).
// HBM layout: source/basis bytes as given (16-byte aligned base); candidates
// (offset u64, sum u32) appended then radix-sorted by offset.  DESIGN.md 4.
#include <rocprim/device/device_radix_sort.hpp>

#include "internal.hpp"
#include "strong.hpp"

namespace vsgpu {

// ---- weak sums ------------------------------------------------------------------
// signed-byte dot products: sum of 4 bytes, and 4 bytes weighted by w (int8 lanes)
__device__ __forceinline__ int dot4(uint32_t word, uint32_t w, int acc) {
    return __builtin_amdgcn_sdot4((int)word, (int)w, acc, false);
}

// 16 bytes at p (any alignment), bounds-checked against [0, lim)
__device__ __forceinline__ void load16(const uint8_t *p, uint64_t pos, uint64_t lim,
                                       uint32_t (&w)[4]) {
    if (pos + 16 <= lim) {
        memcpy(w, p + pos, 16);
        return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t v = 0;
        for (int j = 0; j < 4; ++j) {
            const uint64_t q = pos + 4 * i + j;
            if (q < lim) v |= (uint32_t)p[q] << (8 * j);
        }
        w[i] = v;
    }
}

// 16 bytes at p (global address space, any alignment): the load counts only in
// vmcnt, so a prefetch stays in flight past LDS traffic
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gload16(const uint8_t *p) {
    typedef __attribute__((address_space(1))) const u32x4 g4;
    const u32x4 v = *(g4 *)(uintptr_t)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

// (sum b, sum u*b) over bytes [pos, pos+n) with u = position - pos (local weights)
__device__ void weak_parts(const uint8_t *p, uint64_t pos, uint64_t n, uint64_t lim,
                           uint32_t &sx, uint32_t &sux) {
    uint32_t a = 0, b = 0;
    uint64_t u = 0;
    for (; u + 16 <= n; u += 16) {
        uint32_t w[4];
        load16(p, pos + u, lim, w);
        int s = 0, t = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            s = dot4(w[i], 0x01010101u, s);
            // weights 4i .. 4i+3 for bytes 0..3 of word i (little endian)
            t = dot4(w[i], (uint32_t)(4 * i) * 0x01010101u + 0x03020100u, t);
        }
        b += (uint32_t)u * (uint32_t)s + (uint32_t)t;
        a += (uint32_t)s;
    }
    for (; u < n; ++u) {
        const uint32_t x = (uint32_t)(int32_t)(int8_t)p[pos + u];
        a += x;
        b += (uint32_t)u * x;
    }
    sx = a;
    sux = b;
}

// get_checksum1 of [pos, pos+n): s1 = sum x, s2 = sum (n - u) x = n*s1 - sum u*x
__device__ __forceinline__ uint32_t weak_sum(const uint8_t *p, uint64_t pos, uint64_t n,
                                             uint64_t lim) {
    uint32_t sx, sux;
    weak_parts(p, pos, n, lim, sx, sux);
    const uint32_t s2 = (uint32_t)n * sx - sux;
    return (sx & 0xffffu) | (s2 << 16);
}

// ---- R4 signatures: one lane per block ------------------------------------------
__global__ void rs_sig_kernel(RsSigArgs a) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.count) return;
    const uint64_t pos = i * a.blength;
    const uint64_t n = (i == a.count - 1 && a.remainder) ? a.remainder : a.blength;
    a.sum1[i] = weak_sum(a.data, pos, n, a.len);
    uint8_t s[16];
    vsstrong::checksum2(a.data + pos, n, a.csum_type, a.seed, s);
    for (uint32_t j = 0; j < a.s2length; ++j) a.sum2[i * a.s2length + j] = s[j];
}

// ---- cooperative XXH3 for long windows: 8 lanes per window ----------------------
// One lane per 128 KiB window streams 64 windows 128 KiB apart through every
// load instruction (64 pages per access).  XXH3's long-input state is 8
// independent 64-bit accumulators over 64-byte stripes, so lane i of an
// 8-lane group owns accumulator i and reads word i of every stripe: the
// group's 8 loads form one contiguous 64-byte access.  acc[i ^ 1] += d[i]
// (xxh3_long in strong.hpp) becomes acc[i] += d[i ^ 1] through a lane swap;
// the scramble is per accumulator.  The same loads feed get_checksum1 (signed
// byte sums via v_dot4), reduced over the group at the end.  Bit-identical to
// vsstrong::checksum2 / weak_sum (tests/test_gpu_rsync.py).
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}

// signed-byte sum and position-weighted sum of the 8 bytes of d at byte pos
__device__ __forceinline__ void weak8(uint64_t d, uint32_t pos, uint32_t &sx, uint32_t &sux) {
    const uint32_t lo = (uint32_t)d, hi = (uint32_t)(d >> 32);
    const uint32_t a = (uint32_t)dot4(lo, 0x01010101u, 0), b = (uint32_t)dot4(hi, 0x01010101u, 0);
    sx += a + b;
    sux += pos * a + (uint32_t)dot4(lo, 0x03020100u, 0) + (pos + 4) * b +
           (uint32_t)dot4(hi, 0x03020100u, 0);
}

__device__ __forceinline__ void coop_stripe(uint64_t &acc, uint64_t d, uint32_t sb, uint32_t i,
                                            uint64_t seed) {
    const uint64_t k = d ^ vsstrong::csec_at(sb + 8 * i, seed);
    acc += (uint64_t)(uint32_t)k * (k >> 32);
    acc += shfl_xor64(d, 1);
}

// window p[0, len), len > 240; i = lane within the 8-lane group.  Returns
// accumulator i; sx/sux = this lane's share of the weak-sum parts.
__device__ __forceinline__ uint64_t coop_long(const uint8_t *p, uint64_t len, uint64_t seed,
                                              uint32_t i, uint32_t &sx, uint32_t &sux) {
    using namespace vsstrong;
    const uint64_t init[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
    uint64_t acc = init[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) acc = (i == (uint32_t)j) ? init[j] : acc;
    sx = 0;
    sux = 0;
    const uint64_t nb = (len - 1) / 1024;
    const uint64_t sec_scr = sec64(16 + i, seed);
    for (uint64_t b = 0; b < nb; ++b) {
        const uint8_t *q = p + b * 1024 + 8 * i;
#pragma unroll 4
        for (uint32_t s = 0; s < 16; ++s) {
            const uint64_t d = rd64(q + 64 * s);
            weak8(d, (uint32_t)(b * 1024 + 64 * s + 8 * i), sx, sux);
            coop_stripe(acc, d, 8 * s, i, seed);
        }
        acc ^= acc >> 47;
        acc ^= sec_scr;
        acc *= P32_1;
    }
    const uint32_t ns = (uint32_t)(((len - 1) - nb * 1024) / 64);
    for (uint32_t s = 0; s < ns; ++s) {
        const uint64_t off = nb * 1024 + 64 * s + 8 * i;
        const uint64_t d = rd64(p + off);
        weak8(d, (uint32_t)off, sx, sux);
        coop_stripe(acc, d, 8 * s, i, seed);
    }
    // last stripe (overlaps): hashed whole, weak-summed from the first byte no
    // earlier stripe covered
    const uint64_t covered = (nb * 16 + ns) * 64;
    const uint64_t off = len - 64 + 8 * i;
    const uint64_t d = rd64(p + off);
    coop_stripe(acc, d, 192 - 64 - 7, i, seed);
    const uint64_t skip = covered > off ? min<uint64_t>(covered - off, 8) : 0;
    weak8(skip >= 8 ? 0 : d & (~0ull << (8 * skip)), (uint32_t)off, sx, sux);
    return acc;
}

// The same with 4 lanes per window: lane k owns accumulators 2k and 2k+1 and
// reads bytes [16k, 16k + 16) of every stripe with one 16-byte load, so
// acc[j ^ 1] += d[j] stays inside the lane (no swap) and a wave's load moves
// 1 KiB.  The signature pass (all windows full blocks) uses this layout.
__device__ __forceinline__ void coop4_stripe(uint64_t &a0, uint64_t &a1, uint64_t d0, uint64_t d1,
                                             uint32_t sb, uint32_t k, uint64_t seed) {
    const uint64_t x0 = d0 ^ vsstrong::csec_at(sb + 16 * k, seed);
    const uint64_t x1 = d1 ^ vsstrong::csec_at(sb + 16 * k + 8, seed);
    a0 += (uint64_t)(uint32_t)x0 * (x0 >> 32) + d1;
    a1 += (uint64_t)(uint32_t)x1 * (x1 >> 32) + d0;
}

__device__ __forceinline__ void ld16u(const uint8_t *p, uint64_t &d0, uint64_t &d1) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);   // unaligned dwordx4 (gfx950 unaligned mode)
    d0 = ((uint64_t)v.y << 32) | v.x;
    d1 = ((uint64_t)v.w << 32) | v.z;
}

// window p[0, len), len > 240; k = lane within the 4-lane group.  a0 / a1 =
// accumulators 2k / 2k+1; sx/sux = this lane's share of the weak-sum parts.
__device__ __forceinline__ void coop4_long(const uint8_t *p, uint64_t len, uint64_t seed, uint32_t k,
                                           uint64_t &a0, uint64_t &a1, uint32_t &sx, uint32_t &sux) {
    using namespace vsstrong;
    const uint64_t init[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
    a0 = init[0];
    a1 = init[1];
#pragma unroll
    for (int j = 1; j < 4; ++j) {
        a0 = (k == (uint32_t)j) ? init[2 * j] : a0;
        a1 = (k == (uint32_t)j) ? init[2 * j + 1] : a1;
    }
    sx = 0;
    sux = 0;
    const uint64_t nb = (len - 1) / 1024;
    const uint64_t scr0 = sec64(16 + 2 * k, seed), scr1 = sec64(17 + 2 * k, seed);
    for (uint64_t b = 0; b < nb; ++b) {
        const uint8_t *q = p + b * 1024 + 16 * k;
#pragma unroll 8
        for (uint32_t s = 0; s < 16; ++s) {
            uint64_t d0, d1;
            ld16u(q + 64 * s, d0, d1);
            const uint32_t pos = (uint32_t)(b * 1024 + 64 * s + 16 * k);
            weak8(d0, pos, sx, sux);
            weak8(d1, pos + 8, sx, sux);
            coop4_stripe(a0, a1, d0, d1, 8 * s, k, seed);
        }
        a0 ^= a0 >> 47;
        a0 ^= scr0;
        a0 *= P32_1;
        a1 ^= a1 >> 47;
        a1 ^= scr1;
        a1 *= P32_1;
    }
    const uint32_t ns = (uint32_t)(((len - 1) - nb * 1024) / 64);
    for (uint32_t s = 0; s < ns; ++s) {
        const uint64_t off = nb * 1024 + 64 * s + 16 * k;
        uint64_t d0, d1;
        ld16u(p + off, d0, d1);
        weak8(d0, (uint32_t)off, sx, sux);
        weak8(d1, (uint32_t)off + 8, sx, sux);
        coop4_stripe(a0, a1, d0, d1, 8 * s, k, seed);
    }
    // last stripe (overlaps): hashed whole, weak-summed from the first byte no
    // earlier stripe covered
    const uint64_t covered = (nb * 16 + ns) * 64;
    const uint64_t off = len - 64 + 16 * k;
    uint64_t d0, d1;
    ld16u(p + off, d0, d1);
    coop4_stripe(a0, a1, d0, d1, 192 - 64 - 7, k, seed);
    const uint64_t sk0 = covered > off ? min<uint64_t>(covered - off, 8) : 0;
    const uint64_t sk1 = covered > off + 8 ? min<uint64_t>(covered - off - 8, 8) : 0;
    weak8(sk0 >= 8 ? 0 : d0 & (~0ull << (8 * sk0)), (uint32_t)off, sx, sux);
    weak8(sk1 >= 8 ? 0 : d1 & (~0ull << (8 * sk1)), (uint32_t)off + 8, sx, sux);
}

__device__ __forceinline__ void coop4_finish(uint64_t a0, uint64_t a1, uint32_t sx, uint32_t sux,
                                             uint64_t len, int csum_type, uint64_t seed,
                                             uint32_t gbase, uint32_t &weak, uint64_t &lo,
                                             uint64_t &hi) {
#pragma unroll
    for (int m = 1; m < 4; m <<= 1) {
        sx += (uint32_t)__shfl_xor((int)sx, m, 64);
        sux += (uint32_t)__shfl_xor((int)sux, m, 64);
    }
    const uint32_t s2 = (uint32_t)len * sx - sux;
    weak = (sx & 0xffffu) | (s2 << 16);
    vsstrong::Xxh3Long st;
#pragma unroll
    for (int j = 0; j < 8; ++j) st.acc[j] = shfl64((j & 1) ? a1 : a0, (int)gbase + j / 2);
    lo = st.merge(11, len * vsstrong::P64_1, seed);
    hi = (csum_type == vsstrong::kXxh3_128) ? st.merge(192 - 64 - 11, ~(len * vsstrong::P64_2), seed)
                                            : 0;
}

// group-wide finish: weak sum and strong sum of the window (every lane returns them)
__device__ __forceinline__ void coop_finish(uint64_t acc, uint32_t sx, uint32_t sux, uint64_t len,
                                            int csum_type, uint64_t seed, uint32_t gbase,
                                            uint32_t &weak, uint64_t &lo, uint64_t &hi) {
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) {
        sx += (uint32_t)__shfl_xor((int)sx, m, 64);
        sux += (uint32_t)__shfl_xor((int)sux, m, 64);
    }
    const uint32_t s2 = (uint32_t)len * sx - sux;
    weak = (sx & 0xffffu) | (s2 << 16);
    vsstrong::Xxh3Long st;
#pragma unroll
    for (int j = 0; j < 8; ++j) st.acc[j] = shfl64(acc, (int)gbase + j);
    lo = st.merge(11, len * vsstrong::P64_1, seed);
    hi = (csum_type == vsstrong::kXxh3_128) ? st.merge(192 - 64 - 11, ~(len * vsstrong::P64_2), seed)
                                            : 0;
}

__device__ __forceinline__ void put_strong(uint8_t *out, uint32_t s2length, uint64_t lo, uint64_t hi) {
    for (uint32_t j = 0; j < s2length; ++j)
        out[j] = (uint8_t)(j < 8 ? lo >> (8 * j) : hi >> (8 * (j - 8)));
}

// signatures: 4 lanes per block (XXH3, every block > 240 bytes)
__global__ __launch_bounds__(256) void rs_sig_coop_kernel(RsSigArgs a) {
    const uint64_t g = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
    const uint32_t i = threadIdx.x & 3, gbase = (threadIdx.x & 63) & ~3u;
    const uint64_t b = g < a.count ? g : a.count - 1;  // whole groups stay active (shuffles)
    const uint64_t pos = b * a.blength;
    const uint64_t n = (b == a.count - 1 && a.remainder) ? a.remainder : a.blength;
    uint32_t sx, sux, weak;
    uint64_t lo, hi, a0, a1;
    coop4_long(a.data + pos, n, a.seed, i, a0, a1, sx, sux);
    coop4_finish(a0, a1, sx, sux, n, a.csum_type, a.seed, gbase, weak, lo, hi);
    if (g < a.count && i == 0) {
        a.sum1[g] = weak;
        put_strong(a.sum2 + g * a.s2length, a.s2length, lo, hi);
    }
}

// LN lanes per block (LN = 8 .. 64): lane (h, m) of a block's group reads
// 16 bytes at 16 (4 h + m) of every run of LN / 4 stripes, so one load
// instruction covers 64 / LN blocks' LN * 16-byte runs instead of sixteen
// 64-byte pieces; lane m's accumulators 2m, 2m + 1 sum the group's stripes
// (xor-shuffles over h) before each 1 KiB scramble, which every h repeats.
#ifndef VS_SIG_LANES
#define VS_SIG_LANES 8   // 4: rs_sig_coop_kernel; 8 .. 64: rs_sig_coopn_kernel
#endif
static_assert(VS_SIG_LANES >= 4 && VS_SIG_LANES <= 64 && (VS_SIG_LANES & (VS_SIG_LANES - 1)) == 0,
              "lanes per block");
template <uint32_t LN>
__device__ __forceinline__ void coopn_long(const uint8_t *p, uint64_t len, uint64_t seed, uint32_t ml,
                                           uint64_t &a0, uint64_t &a1, uint32_t &sx, uint32_t &sux) {
    using namespace vsstrong;
    constexpr uint32_t SP = LN / 4, NI = 16 / SP;
    const uint32_t m = ml & 3, h = ml >> 2;
    const uint64_t init[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
    a0 = init[0];
    a1 = init[1];
#pragma unroll
    for (int j = 1; j < 4; ++j) {
        a0 = (m == (uint32_t)j) ? init[2 * j] : a0;
        a1 = (m == (uint32_t)j) ? init[2 * j + 1] : a1;
    }
    sx = 0;
    sux = 0;
    const uint64_t nb = (len - 1) / 1024;
    const uint64_t scr0 = sec64(16 + 2 * m, seed), scr1 = sec64(17 + 2 * m, seed);
    uint64_t ks0[NI], ks1[NI];
#pragma unroll
    for (uint32_t i = 0; i < NI; ++i) {
        ks0[i] = sec64(SP * i + h + 2 * m, seed);
        ks1[i] = sec64(SP * i + h + 2 * m + 1, seed);
    }
    auto fold = [&](uint64_t &c0, uint64_t &c1) {
#pragma unroll
        for (uint32_t o = 4; o < LN; o <<= 1) {
            c0 += shfl_xor64(c0, (int)o);
            c1 += shfl_xor64(c1, (int)o);
        }
    };
    for (uint64_t b = 0; b < nb; ++b) {
        const uint8_t *q = p + b * 1024 + 16 * ml;
        uint64_t c0 = 0, c1 = 0;
#pragma unroll
        for (uint32_t i = 0; i < NI; ++i) {
            uint64_t d0, d1;
            ld16u(q + 64 * SP * i, d0, d1);
            const uint32_t pos = (uint32_t)(b * 1024 + 64 * SP * i + 16 * ml);
            weak8(d0, pos, sx, sux);
            weak8(d1, pos + 8, sx, sux);
            const uint64_t x0 = d0 ^ ks0[i], x1 = d1 ^ ks1[i];
            c0 += (uint64_t)(uint32_t)x0 * (x0 >> 32) + d1;
            c1 += (uint64_t)(uint32_t)x1 * (x1 >> 32) + d0;
        }
        fold(c0, c1);
        a0 += c0;
        a0 ^= a0 >> 47;
        a0 ^= scr0;
        a0 *= P32_1;
        a1 += c1;
        a1 ^= a1 >> 47;
        a1 ^= scr1;
        a1 *= P32_1;
    }
    // the partial block's ns stripes (no scramble)
    const uint32_t ns = (uint32_t)(((len - 1) - nb * 1024) / 64);
    {
        uint64_t c0 = 0, c1 = 0;
#pragma unroll
        for (uint32_t i = 0; i < NI; ++i) {
            const uint32_t s = SP * i + h;
            if (s < ns) {
                const uint64_t off = nb * 1024 + 64 * s + 16 * m;
                uint64_t d0, d1;
                ld16u(p + off, d0, d1);
                weak8(d0, (uint32_t)off, sx, sux);
                weak8(d1, (uint32_t)off + 8, sx, sux);
                const uint64_t x0 = d0 ^ ks0[i], x1 = d1 ^ ks1[i];
                c0 += (uint64_t)(uint32_t)x0 * (x0 >> 32) + d1;
                c1 += (uint64_t)(uint32_t)x1 * (x1 >> 32) + d0;
            }
        }
        fold(c0, c1);
        a0 += c0;
        a1 += c1;
    }
    // last stripe (overlaps): every h hashes it (the accumulators stay equal
    // across h); h = 0 weak-sums it from the first byte no earlier stripe covered
    const uint64_t covered = (nb * 16 + ns) * 64;
    const uint64_t off = len - 64 + 16 * m;
    uint64_t d0, d1;
    ld16u(p + off, d0, d1);
    coop4_stripe(a0, a1, d0, d1, 192 - 64 - 7, m, seed);
    if (h == 0) {
        const uint64_t sk0 = covered > off ? min<uint64_t>(covered - off, 8) : 0;
        const uint64_t sk1 = covered > off + 8 ? min<uint64_t>(covered - off - 8, 8) : 0;
        weak8(sk0 >= 8 ? 0 : d0 & (~0ull << (8 * sk0)), (uint32_t)off, sx, sux);
        weak8(sk1 >= 8 ? 0 : d1 & (~0ull << (8 * sk1)), (uint32_t)off + 8, sx, sux);
    }
}

template <uint32_t LN>
__global__ __launch_bounds__(256) void rs_sig_coopn_kernel(RsSigArgs a) {
    const uint64_t g = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / LN;
    const uint32_t ml = threadIdx.x & (LN - 1), gbase = (threadIdx.x & 63) & ~(LN - 1);
    const uint64_t b = g < a.count ? g : a.count - 1;  // whole groups stay active (shuffles)
    const uint64_t pos = b * a.blength;
    const uint64_t n = (b == a.count - 1 && a.remainder) ? a.remainder : a.blength;
    uint32_t sx, sux, weak;
    uint64_t lo, hi, a0, a1;
    coopn_long<LN>(a.data + pos, n, a.seed, ml, a0, a1, sx, sux);
    // the weak parts of lanes h > 0 join lanes h = 0; coop4_finish adds the four m
#pragma unroll
    for (uint32_t o = 4; o < LN; o <<= 1) {
        sx += (uint32_t)__shfl_xor((int)sx, (int)o, 64);
        sux += (uint32_t)__shfl_xor((int)sux, (int)o, 64);
    }
    coop4_finish(a0, a1, sx, sux, n, a.csum_type, a.seed, gbase, weak, lo, hi);
    if (g < a.count && ml == 0) {
        a.sum1[g] = weak;
        put_strong(a.sum2 + g * a.s2length, a.s2length, lo, hi);
    }
}

// candidate verification: 8 lanes per window (XXH3, every window > 240 bytes)
__global__ __launch_bounds__(256) void rs_strong_coop_kernel(const uint8_t *data,
                                                             const uint64_t *offs,
                                                             const uint32_t *lens, uint64_t n,
                                                             int csum_type, uint32_t seed,
                                                             uint32_t s2length, uint8_t *out) {
    const uint64_t g = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3;
    const uint32_t i = threadIdx.x & 7, gbase = (threadIdx.x & 63) & ~7u;
    const uint64_t w = g < n ? g : n - 1;
    const uint64_t len = lens[w];
    uint32_t sx, sux, weak;
    uint64_t lo, hi;
    const uint64_t acc = coop_long(data + offs[w], len, seed, i, sx, sux);
    coop_finish(acc, sx, sux, len, csum_type, seed, gbase, weak, lo, hi);
    if (g < n && i == 0) put_strong(out + g * s2length, s2length, lo, hi);
}

static bool coop_ok(int csum_type) {
    return csum_type == vsstrong::kXxh3_128 || csum_type == vsstrong::kXxh3_64;
}

hipError_t launch_rs_signatures(const RsSigArgs &a, hipStream_t s) {
    if (!a.count) return hipSuccess;
    if (coop_ok(a.csum_type) && a.blength > 240 && (a.remainder == 0 || a.remainder > 240)) {
        if (VS_SIG_LANES > 4)
            rs_sig_coopn_kernel<VS_SIG_LANES>
                <<<(uint32_t)((a.count * VS_SIG_LANES + 255) / 256), 256, 0, s>>>(a);
        else
            rs_sig_coop_kernel<<<(uint32_t)((a.count * 4 + 255) / 256), 256, 0, s>>>(a);
    } else
        rs_sig_kernel<<<(uint32_t)((a.count + 127) / 128), 128, 0, s>>>(a);
    return hipGetLastError();
}

// ---- strong sums of arbitrary windows (candidate verification) --------------------
__global__ void rs_strong_kernel(const uint8_t *data, const uint64_t *offs, const uint32_t *lens,
                                 uint64_t n, int csum_type, uint32_t seed, uint32_t s2length,
                                 uint8_t *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t s[16];
    vsstrong::checksum2(data + offs[i], lens[i], csum_type, seed, s);
    for (uint32_t j = 0; j < s2length; ++j) out[i * s2length + j] = s[j];
}

hipError_t launch_rs_strong(const uint8_t *data, const uint64_t *offs, const uint32_t *lens,
                            uint64_t n, int csum_type, uint32_t seed, uint32_t s2length,
                            uint8_t *out, uint32_t min_len, hipStream_t s) {
    if (!n) return hipSuccess;
    if (coop_ok(csum_type) && min_len > 240)
        rs_strong_coop_kernel<<<(uint32_t)((n * 8 + 255) / 256), 256, 0, s>>>(
            data, offs, lens, n, csum_type, seed, s2length, out);
    else
        rs_strong_kernel<<<(uint32_t)((n + 127) / 128), 128, 0, s>>>(data, offs, lens, n,
                                                                     csum_type, seed, s2length, out);
    return hipGetLastError();
}

// ---- R5 table: sort keys, directory, filter ----------------------------------------
__global__ void rs_keys_kernel(const uint32_t *sum1, uint32_t count, uint64_t *keys) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) keys[i] = ((uint64_t)sum1[i] << 32) | (uint32_t)~i;
}

// dir[b] = first sorted position whose bucket (sum1 >> (32 - dbits)) >= b, b in [0, 2^dbits]
__global__ void rs_dir_kernel(const uint64_t *tkey, uint32_t count, uint32_t dbits, uint32_t *dir,
                              uint32_t fbits, uint32_t *filt) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nb = 1ull << dbits;
    if (p > count) return;
    const uint64_t b = (p < count) ? (tkey[p] >> (64 - dbits)) : nb;
    const uint64_t bp = (p == 0) ? 0 : (tkey[p - 1] >> (64 - dbits)) + 1;
    for (uint64_t q = bp; q <= b; ++q) dir[q] = (uint32_t)p;
    if (p < count) {
        const uint32_t f = (uint32_t)(tkey[p] >> (64 - fbits));
        atomicOr(&filt[f >> 5], 1u << (f & 31));
        // LDS prefilter, stored after the filter
        uint32_t *filt_l = filt + ((1ull << fbits) / 32);
        const uint32_t fl = (uint32_t)(tkey[p] >> (64 - rs_lds_filter_bits(fbits)));
        atomicOr(&filt_l[fl >> 5], 1u << (fl & 31));
        // blocked filter over all 32 bits of sum1, stored after the prefilter
        unsigned long long *filt_b =
            (unsigned long long *)(filt_l + ((1ull << rs_lds_filter_bits(fbits)) / 32));
        const uint32_t s1 = (uint32_t)(tkey[p] >> 32);
        atomicOr(&filt_b[rs_bloom_word(s1, fbits)], (unsigned long long)rs_bloom_mask(s1));
    }
}

hipError_t launch_rs_table(const uint32_t *sum1, uint32_t count, uint64_t *keys, uint64_t *tkey,
                           void *tmp, size_t tmp_bytes, uint32_t dbits, uint32_t *dir,
                           uint32_t fbits, uint32_t *filt, hipStream_t s) {
    if (!count) return hipSuccess;
    rs_keys_kernel<<<(count + 255) / 256, 256, 0, s>>>(sum1, count, keys);
    hipError_t e = rocprim::radix_sort_keys(tmp, tmp_bytes, keys, tkey, (size_t)count, 0, 64, s);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(filt, 0, rs_filter_bytes(fbits), s);
    if (e != hipSuccess) return e;
    rs_dir_kernel<<<(count + 1 + 255) / 256, 256, 0, s>>>(tkey, count, dbits, dir, fbits, filt);
    return hipGetLastError();
}

// the key at sorted position p is a full-length block
__device__ __forceinline__ bool rs_key_full(uint64_t key, uint32_t count, uint32_t remainder) {
    return !(remainder && ~(uint32_t)key == count - 1);
}

__global__ void rs_bucket_kernel(const uint64_t *tkey, uint32_t count, uint32_t remainder,
                                 uint32_t bbits, uint32_t *bkt) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= count) return;
    const uint64_t k = tkey[p];
    if (!rs_key_full(k, count, remainder)) return;
    const uint32_t s = (uint32_t)(k >> 32);
    // the first full-length key of its sum's run: the run is sorted by
    // descending index, so the short block (the largest index) leads it
    if (p > 0 && (uint32_t)(tkey[p - 1] >> 32) == s) {
        const bool prev_full = rs_key_full(tkey[p - 1], count, remainder);
        if (prev_full || (p > 1 && (uint32_t)(tkey[p - 2] >> 32) == s)) return;
    }
    uint32_t *b = bkt + (uint64_t)rs_bucket(s, bbits) * kBucketWords;
    const uint32_t slot = atomicAdd(&b[0], 1u);
    if (slot < kBucketSlots) b[1 + slot] = s;
}

hipError_t launch_rs_buckets(const uint64_t *tkey, uint32_t count, uint32_t remainder,
                             uint32_t bbits, uint32_t *bkt, hipStream_t s) {
    if (!count) return hipSuccess;
    rs_bucket_kernel<<<(count + 255) / 256, 256, 0, s>>>(tkey, count, remainder, bbits, bkt);
    return hipGetLastError();
}

size_t rs_sort_tmp_bytes(uint64_t n_keys, bool pairs) {
    size_t b = 0;
    if (pairs)
        (void)rocprim::radix_sort_pairs(nullptr, b, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                        (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                        (size_t)n_keys, 0, 64);
    else
        (void)rocprim::radix_sort_keys(nullptr, b, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                       (size_t)n_keys, 0, 64);
    return b;
}

// ---- R6 coarse prefix sums of the source ------------------------------------------
// per kRsG-byte block j: px[j] = sum x, pt[j] = sum t*x (t absolute, mod 2^32).
// One wave per block: lane l sums bytes [64 l, 64 l + 64) with local weights,
// then sux = sum_l (sux_l + 64 l * sx_l) across the wave (coalesced reads).
__global__ __launch_bounds__(256) void rs_block_sums_kernel(const uint8_t *data, uint64_t len,
                                                            uint64_t nblk, uint32_t *px,
                                                            uint32_t *pt) {
    const uint64_t j = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    if (j >= nblk) return;
    const uint64_t pos = j * kRsG;
    const uint64_t n = min((uint64_t)kRsG, len - pos);
    const uint64_t lo = min((uint64_t)lane * 64, n), hi = min(lo + 64, n);
    uint32_t sx = 0, sux = 0;
    if (hi > lo) weak_parts(data, pos + lo, hi - lo, len, sx, sux);
    sux += (uint32_t)lo * sx;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        sx += (uint32_t)__shfl_xor((int)sx, o, 64);
        sux += (uint32_t)__shfl_xor((int)sux, o, 64);
    }
    if (lane == 0) {
        px[j] = sx;
        pt[j] = (uint32_t)pos * sx + sux;
    }
}

hipError_t launch_rs_prefix(const uint8_t *data, uint64_t len, uint32_t *px, uint32_t *pt,
                            uint32_t *px_scan, uint32_t *pt_scan, uint32_t *partials,
                            hipStream_t s) {
    const uint64_t nblk = (len + kRsG - 1) / kRsG;
    if (nblk) {
        rs_block_sums_kernel<<<(uint32_t)((nblk + 3) / 4), 256, 0, s>>>(data, len, nblk, px, pt);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipError_t e = launch_scan_u32(px, px_scan, nblk, partials, 0xffffffffu, s);
    if (e != hipSuccess) return e;
    return launch_scan_u32(pt, pt_scan, nblk, partials, 0xffffffffu, s);
}

// ---- R6 weak scan ----------------------------------------------------------------------
// prefix (sum x, sum t*x) of bytes [0, q)
__device__ __forceinline__ void prefix_at(const RsScanArgs &a, uint64_t q, uint32_t &sx,
                                          uint32_t &stx) {
    const uint64_t j = q / kRsG;
    const uint64_t q0 = j * kRsG;
    uint32_t x = a.px_scan[j], t = a.pt_scan[j];
    if (q > q0) {
        uint32_t bx, bux;
        weak_parts(a.data, q0, q - q0, a.len, bx, bux);
        x += bx;
        t += (uint32_t)q0 * bx + bux;
    }
    sx = x;
    stx = t;
}

// Both filter levels for 8 weak sums: the LDS prefilter tests first, then 8 unconditional
// HBM/L2 loads issued back to back (lanes that failed the prefilter read word
// 0, one shared address), so a lane waits for one round trip per 8 offsets
// instead of one per passing offset.  Bits j0..j0+7 of the result.
template <int J0, int N>
__device__ __forceinline__ uint32_t filter8(const RsScanArgs &a, const uint32_t *lfilt,
                                            const uint32_t (&sums)[N]) {
    uint32_t lp = 0, w[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t fl = sums[J0 + j] >> (32 - a.lbits);
        lp |= ((lfilt[fl >> 5] >> (fl & 31)) & 1u) << j;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t f = sums[J0 + j] >> (32 - a.fbits);
        sh[j] = f & 31;
        w[j] = *(((lp >> j) & 1u) ? a.filt + (f >> 5) : a.filt);
    }
    uint32_t hit = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) hit |= (((w[j] >> sh[j]) & (lp >> j)) & 1u) << (J0 + j);
    return hit;
}

// does a block with sum1 == sum and length k exist? (directory walk; the
// filters were applied by the caller)
__device__ __forceinline__ bool probe_dir(const RsScanArgs &a, uint32_t sum, bool full) {
    const uint32_t b = sum >> (32 - a.dbits);
    const uint32_t p0 = a.dir[b], p1 = a.dir[b + 1];
    for (uint32_t p = p0; p < p1; ++p) {
        const uint64_t key = a.tkey[p];
        const uint32_t s1 = (uint32_t)(key >> 32);
        if (s1 > sum) break;
        if (s1 < sum) continue;
        const uint32_t i = ~(uint32_t)key;
        const bool last_short = (i == a.count - 1) && a.remainder;
        if (full ? !last_short : last_short) return true;
    }
    return false;
}

__device__ __forceinline__ void emit(const RsScanArgs &a, uint64_t o, uint32_t sum) {
    const unsigned long long slot = atomicAdd((unsigned long long *)a.n_cand, 1ull);
    if (slot < a.cap) {
        a.cand_off[slot] = o;
        a.cand_sum[slot] = sum;
    }
}

// Candidates are collected per workgroup in LDS and appended to the global
// list with one atomic per workgroup and round: a single global counter bumped
// once per candidate serialises millions of same-address atomics.
//
// Filter in two levels: every offset's weak sum is first tested against a
// 2^20-bit prefilter held in LDS (the top 20 bits of the table's sums, built
// with the table), and only the offsets that pass gather from the 2^fbits-bit
// filter in HBM/L2 (filter8()).  With one random 4-byte gather per offset the
// L2-resident filter alone bound the scan (~186 GB/s at C4 shape).  The grid is
// persistent -- one workgroup per CU loads the prefilter once -- and each round
// of strips flushes the workgroup's candidates.
// 16 waves per CU: the gathers need the occupancy (512 threads: 332 ms, 1024:
// 235 ms at C4 shape, despite 80 B/lane of scratch in the rare probe path)
constexpr uint32_t kScanThreads = 1024;
constexpr uint32_t kLocCand = 2048;
constexpr uint32_t kLdsFiltWords = 1u << 15;  // 2^20 bits

__device__ __forceinline__ void scan_strip(const RsScanArgs &a, uint64_t k, const uint32_t *lfilt,
                                           uint64_t *loc_off, uint32_t *loc_sum,
                                           uint32_t *loc_n_p) {
    uint32_t &loc_n = *loc_n_p;
    const uint64_t o0 = k * kRsStrip;
    if (o0 < a.nfull) {
        const uint64_t o1 = min(o0 + kRsStrip, a.nfull);
        const uint64_t n = a.blength;
        // window sum at o0 from the coarse prefixes (o0 is a multiple of kRsG)
        uint32_t xa, ta, xb, tb;
        prefix_at(a, o0, xa, ta);
        prefix_at(a, o0 + n, xb, tb);
        uint32_t s1 = xb - xa;
        uint32_t s2 = (uint32_t)(n + o0) * s1 - (tb - ta);
        const uint8_t *d = a.data;
        const uint32_t nn = (uint32_t)n;
        uint64_t o = o0;
        if (o1 + n + 32 <= a.len) {
            // interior strip: unconditional 32-byte loads, the next group's
            // prefetched while this one's 32 filter gathers are in flight
            uint4 po0 = gload16(d + o), po1 = gload16(d + o + 16);
            uint4 pi0 = gload16(d + o + n), pi1 = gload16(d + o + n + 16);
            for (; o < o1; o += 32) {
                const uint32_t wo[8] = {po0.x, po0.y, po0.z, po0.w, po1.x, po1.y, po1.z, po1.w};
                const uint32_t wi[8] = {pi0.x, pi0.y, pi0.z, pi0.w, pi1.x, pi1.y, pi1.z, pi1.w};
                po0 = gload16(d + o + 32);
                po1 = gload16(d + o + 48);
                pi0 = gload16(d + o + n + 32);
                pi1 = gload16(d + o + n + 48);
                uint32_t sums[32];
#pragma unroll
                for (int j = 0; j < 32; ++j) {
                    sums[j] = (s1 & 0xffffu) | (s2 << 16);
                    const uint32_t xo = (uint32_t)__builtin_amdgcn_sbfe(wo[j >> 2], 8 * (j & 3), 8);
                    const uint32_t xi = (uint32_t)__builtin_amdgcn_sbfe(wi[j >> 2], 8 * (j & 3), 8);
                    s1 = s1 - xo + xi;
                    s2 = s2 - nn * xo + s1;
                }
                uint32_t hit = 0;
                hit = filter8<0>(a, lfilt, sums) | filter8<8>(a, lfilt, sums) |
                      filter8<16>(a, lfilt, sums) | filter8<24>(a, lfilt, sums);
                while (hit) {
                    const int j = __builtin_ctz(hit);
                    hit &= hit - 1;
                    if (o + j < o1 && o + j >= a.lo && probe_dir(a, sums[j], true)) {
                        const uint32_t slot = atomicAdd(&loc_n, 1u);
                        if (slot < kLocCand) {
                            loc_off[slot] = o + j;
                            loc_sum[slot] = sums[j];
                        } else {
                            emit(a, o + j, sums[j]);
                        }
                    }
                }
            }
        }
        for (; o < o1; o += 16) {
            uint32_t wo[4], wi[4];
            load16(d, o, a.len, wo);       // bytes leaving: o .. o+15
            load16(d, o + n, a.len, wi);   // bytes entering: o+n .. o+n+15
            uint32_t sums[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                sums[j] = (s1 & 0xffffu) | (s2 << 16);
                const uint32_t xo = (uint32_t)__builtin_amdgcn_sbfe(wo[j >> 2], 8 * (j & 3), 8);
                const uint32_t xi = (uint32_t)__builtin_amdgcn_sbfe(wi[j >> 2], 8 * (j & 3), 8);
                // hash_search's roll: s1 -= out; s2 -= k*out; s1 += in; s2 += s1
                s1 = s1 - xo + xi;
                s2 = s2 - nn * xo + s1;
            }
            uint32_t hit = 0;
            hit = filter8<0>(a, lfilt, sums) | filter8<8>(a, lfilt, sums);
            while (hit) {
                const int j = __builtin_ctz(hit);
                hit &= hit - 1;
                if (o + j < o1 && o + j >= a.lo && probe_dir(a, sums[j], true)) {
                    const uint32_t slot = atomicAdd(&loc_n, 1u);
                    if (slot < kLocCand) {
                        loc_off[slot] = o + j;
                        loc_sum[slot] = sums[j];
                    } else {
                        emit(a, o + j, sums[j]);  // local buffer full
                    }
                }
            }
        }
    }
}

__global__ __launch_bounds__(kScanThreads) void rs_scan_kernel(RsScanArgs a) {
    __shared__ uint32_t lfilt[kLdsFiltWords];
    __shared__ uint64_t loc_off[kLocCand];
    __shared__ uint32_t loc_sum[kLocCand];
    __shared__ uint32_t loc_n;
    __shared__ unsigned long long loc_base;
    const uint32_t lw = (1u << a.lbits) / 32;
    for (uint32_t i = threadIdx.x; i < lw; i += blockDim.x) lfilt[i] = a.filt_l[i];
    if (threadIdx.x == 0) loc_n = 0;
    __syncthreads();
    const uint64_t k0 = a.lo / kRsStrip;
    const uint64_t strips = (a.nfull + kRsStrip - 1) / kRsStrip - k0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < strips; base += stride) {
        const uint64_t k = base + threadIdx.x;
        if (k < strips) scan_strip(a, k0 + k, lfilt, loc_off, loc_sum, &loc_n);
        __syncthreads();
        const uint32_t m = min(loc_n, kLocCand);
        if (m) {
            if (threadIdx.x == 0)
                loc_base = atomicAdd((unsigned long long *)a.n_cand, (unsigned long long)m);
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
                const unsigned long long slot = loc_base + i;
                if (slot < a.cap) {
                    a.cand_off[slot] = loc_off[i];
                    a.cand_sum[slot] = loc_sum[i];
                }
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) loc_n = 0;
        __syncthreads();
    }
}

// the one shrunk-window offset that can match (the short last block), on one lane
__global__ void rs_scan_tail_kernel(RsScanArgs a, uint64_t o) {
    const uint32_t sum = weak_sum(a.data, o, a.remainder, a.len);
    if (probe_dir(a, sum, false)) emit(a, o, sum);
}

hipError_t launch_rs_scan(const RsScanArgs &a, int cus, hipStream_t s) {
    const uint64_t k0 = a.lo / kRsStrip;
    const uint64_t kend = (a.nfull + kRsStrip - 1) / kRsStrip;
    const uint64_t strips = (a.nfull > a.lo) ? kend - k0 : 0;
    if (a.lbits > 20) return hipErrorInvalidValue;  // prefilter larger than its LDS array
    if (strips) {
        // persistent: one workgroup per CU (the 152 KiB of LDS admit one)
        const uint64_t grid = std::min<uint64_t>((strips + kScanThreads - 1) / kScanThreads,
                                                 (uint64_t)std::max(cus, 1));
        rs_scan_kernel<<<(uint32_t)grid, kScanThreads, 0, s>>>(a);
    }
    if (a.tail >= 0 && a.remainder && a.count && (uint64_t)a.tail + a.remainder <= a.len)
        rs_scan_tail_kernel<<<1, 1, 0, s>>>(a, (uint64_t)a.tail);
    return hipGetLastError();
}

__device__ __forceinline__ bool sorted_has(const uint64_t *off, uint64_t n, uint64_t v) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (off[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo < n && off[lo] == v;
}

__global__ void rs_chained_kernel(const uint64_t *off, uint64_t n, uint64_t bl, uint8_t *flag) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const uint64_t o = off[c];
    flag[c] = (uint8_t)((o >= bl && sorted_has(off, n, o - bl)) || sorted_has(off, n, o + bl));
}

// Round-0 prediction of the candidates the walk will visit: a chained
// candidate, or one that no chained candidate in the block window before it
// covers (the walk, having matched that one, would jump past it).  Isolated
// weak collisions in edited regions are the second kind; hashing them up
// front saves a verification round and a second walk.  Only a prediction:
// the round loop in rsync_api.hip still guarantees rsync's decisions.
__global__ void rs_visit_kernel(const uint64_t *off, uint64_t n, uint64_t bl,
                                const uint8_t *chained, uint8_t *visit) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    uint8_t v = chained[c];
    if (!v) {
        const uint64_t o = off[c];
        bool covered = false;
        // ~count / 2^32 * blength weak collisions per window: a short scan;
        // past the cap assume covered (a missed prediction costs a round)
        for (uint64_t p = c, k = 0; p > 0 && off[p - 1] + bl > o; --p, ++k) {
            if (k == 256 || chained[p - 1]) {
                covered = true;
                break;
            }
        }
        v = !covered;
    }
    visit[c] = v;
}

hipError_t launch_rs_chained(const uint64_t *off, uint64_t n, uint64_t blength, uint8_t *flag,
                             hipStream_t s) {
    if (!n) return hipSuccess;
    const uint32_t grid = (uint32_t)((n + 255) / 256);
    rs_chained_kernel<<<grid, 256, 0, s>>>(off, n, blength, flag);
    rs_visit_kernel<<<grid, 256, 0, s>>>(off, n, blength, flag, flag + n);
    return hipGetLastError();
}

hipError_t launch_rs_sort_cands(void *tmp, size_t tmp_bytes, const uint64_t *off_in,
                                uint64_t *off_out, const uint32_t *sum_in, uint32_t *sum_out,
                                uint64_t n, int end_bit, hipStream_t s) {
    if (!n) return hipSuccess;
    return rocprim::radix_sort_pairs(tmp, tmp_bytes, off_in, off_out, sum_in, sum_out, (size_t)n, 0,
                                     (unsigned)end_bit, s);
}

}  // namespace vsgpu
