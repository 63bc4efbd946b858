// crypto.hip -- restic's blob encryption on the device (the
// pack stage after the blob ID: mover-restic/entry.sh:60-65).
//
// restic v0.13.1 internal/crypto Key.Seal(dst, nonce, plaintext, nil):
//   ciphertext = AES-256-CTR(EncryptionKey, IV = nonce)(plaintext), the IV
//     incremented as one 128-bit big-endian counter per 16-byte block
//     (Go cipher.NewCTR);
//   mac = Poly1305(ciphertext, r = MACKey.R, s = AES-128(MACKey.K, nonce)).
// The repository stores nonce || ciphertext || mac per blob.
//
// seal_ctr_kernel: AES-256 counter blocks with a T-table in LDS (one 1 KiB
//   table, rotations for the other three, 32 lane-private copies so a
//   ds_read_b32 from 32 lanes never conflicts), XORed into the bytes; lane l
//   of a wave takes blocks base + 64 j + l, so every load / store is a
//   coalesced 1 KiB per wave.
// seal_mac_kernel: one wave per blob.  Poly1305 is h = sum_i m_i r^(N-i+1)
//   mod 2^130 - 5; lane j Horner-evaluates blocks j+1, j+65, ... with r^64
//   and the lanes' sums are lifted by r^e_j (e_j = N - last_j + 1 <= 64) and
//   added -- r is the repository's key, so r^1..r^64 are computed once per
//   handle.  130-bit arithmetic in five 26-bit limbs (v_mad_u64_u32).
#include <cstdlib>
#include <cstring>
#include <vector>

#include "internal.hpp"

#define VS_API extern "C" __attribute__((visibility("default")))

namespace vsgpu {
namespace {

constexpr uint32_t kCopies = 32;   // lane-private copies of Te0 in LDS

__device__ __forceinline__ uint32_t rotl8(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 24); }
__device__ __forceinline__ uint32_t rotl16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
__device__ __forceinline__ uint32_t rotl24(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 8); }

// AES encryption of one block held as four little-endian column words, with
// round keys rk[4 * (nr + 1)] (LE column words) and the LDS T-table te
// (entry e of copy c at e * kCopies + c)
__device__ __forceinline__ void aes_encrypt(uint32_t (&s)[4], const uint32_t *rk, int nr,
                                            const uint32_t *te, uint32_t c) {
    uint32_t s0 = s[0] ^ rk[0], s1 = s[1] ^ rk[1], s2 = s[2] ^ rk[2], s3 = s[3] ^ rk[3];
#define TE(x) te[((x) & 0xffu) * kCopies + c]
    for (int r = 1; r < nr; ++r) {
        const uint32_t *k = rk + 4 * r;
        const uint32_t t0 = TE(s0) ^ rotl8(TE(s1 >> 8)) ^ rotl16(TE(s2 >> 16)) ^ rotl24(TE(s3 >> 24)) ^ k[0];
        const uint32_t t1 = TE(s1) ^ rotl8(TE(s2 >> 8)) ^ rotl16(TE(s3 >> 16)) ^ rotl24(TE(s0 >> 24)) ^ k[1];
        const uint32_t t2 = TE(s2) ^ rotl8(TE(s3 >> 8)) ^ rotl16(TE(s0 >> 16)) ^ rotl24(TE(s1 >> 24)) ^ k[2];
        const uint32_t t3 = TE(s3) ^ rotl8(TE(s0 >> 8)) ^ rotl16(TE(s1 >> 16)) ^ rotl24(TE(s2 >> 24)) ^ k[3];
        s0 = t0;
        s1 = t1;
        s2 = t2;
        s3 = t3;
    }
    // last round: SubBytes + ShiftRows + AddRoundKey; S[x] is byte 1 of Te0[x]
#define SB(x) ((TE(x) >> 8) & 0xffu)
    const uint32_t *k = rk + 4 * nr;
    s[0] = (SB(s0) | (SB(s1 >> 8) << 8) | (SB(s2 >> 16) << 16) | (SB(s3 >> 24) << 24)) ^ k[0];
    s[1] = (SB(s1) | (SB(s2 >> 8) << 8) | (SB(s3 >> 16) << 16) | (SB(s0 >> 24) << 24)) ^ k[1];
    s[2] = (SB(s2) | (SB(s3 >> 8) << 8) | (SB(s0 >> 16) << 16) | (SB(s1 >> 24) << 24)) ^ k[2];
    s[3] = (SB(s3) | (SB(s0 >> 8) << 8) | (SB(s1 >> 16) << 16) | (SB(s2 >> 24) << 24)) ^ k[3];
#undef SB
#undef TE
}

// counter block nonce + q (128-bit big-endian) as LE column words; the nonce
// as four little-endian words as loaded (n[0] = bytes 0..3)
__device__ __forceinline__ void ctr_block(const uint32_t (&n)[4], uint64_t q, uint32_t (&s)[4]) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = __builtin_bswap32(n[i]);
    // add q to the 128-bit big-endian value w[0..3] (w[3] least significant)
    uint64_t acc = (uint64_t)w[3] + (uint32_t)q;
    w[3] = (uint32_t)acc;
    acc = (acc >> 32) + (uint64_t)w[2] + (uint32_t)(q >> 32);
    w[2] = (uint32_t)acc;
    acc = (acc >> 32) + w[1];
    w[1] = (uint32_t)acc;
    w[0] = w[0] + (uint32_t)(acc >> 32);
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] = __builtin_bswap32(w[i]);
}

__device__ __forceinline__ void load_nonce(const uint8_t *nonces, uint64_t b, uint32_t (&n)[4]) {
    const uint4 v = *(const uint4 *)(nonces + 16 * b);   // 16-byte aligned (checked on the host)
    n[0] = v.x;
    n[1] = v.y;
    n[2] = v.z;
    n[3] = v.w;
}

__device__ __forceinline__ void load_te(uint32_t *te, const uint32_t *g) {
    for (uint32_t i = threadIdx.x; i < 256 * kCopies; i += blockDim.x) te[i] = g[i / kCopies];
}

// the blob holding global block g: the last b with prefix[b] <= g
__device__ __forceinline__ uint64_t find_blob(const uint64_t *prefix, uint64_t n, uint64_t g) {
    uint64_t lo = 0, hi = n;   // prefix[lo] <= g < prefix[hi]
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (prefix[mid] <= g) lo = mid;
        else hi = mid;
    }
    return lo;
}

// ---- Poly1305 in five 26-bit limbs ------------------------------------------
struct L5 {
    uint32_t v[5];
};
constexpr uint32_t kM26 = 0x3ffffff;

// h * r mod 2^130 - 5, h limbs < 2^27, r limbs < 2^26 (s = 5 r)
__device__ __forceinline__ L5 pmul(const L5 &h, const L5 &r) {
    const uint32_t s1 = r.v[1] * 5, s2 = r.v[2] * 5, s3 = r.v[3] * 5, s4 = r.v[4] * 5;
    const uint64_t h0 = h.v[0], h1 = h.v[1], h2 = h.v[2], h3 = h.v[3], h4 = h.v[4];
    uint64_t d0 = h0 * r.v[0] + h1 * s4 + h2 * s3 + h3 * s2 + h4 * s1;
    uint64_t d1 = h0 * r.v[1] + h1 * r.v[0] + h2 * s4 + h3 * s3 + h4 * s2;
    uint64_t d2 = h0 * r.v[2] + h1 * r.v[1] + h2 * r.v[0] + h3 * s4 + h4 * s3;
    uint64_t d3 = h0 * r.v[3] + h1 * r.v[2] + h2 * r.v[1] + h3 * r.v[0] + h4 * s4;
    uint64_t d4 = h0 * r.v[4] + h1 * r.v[3] + h2 * r.v[2] + h3 * r.v[1] + h4 * r.v[0];
    L5 o;
    d1 += d0 >> 26;
    o.v[0] = (uint32_t)d0 & kM26;
    d2 += d1 >> 26;
    o.v[1] = (uint32_t)d1 & kM26;
    d3 += d2 >> 26;
    o.v[2] = (uint32_t)d2 & kM26;
    d4 += d3 >> 26;
    o.v[3] = (uint32_t)d3 & kM26;
    const uint64_t c = d4 >> 26;
    o.v[4] = (uint32_t)d4 & kM26;
    const uint64_t t = (uint64_t)o.v[0] + c * 5;
    o.v[0] = (uint32_t)t & kM26;
    o.v[1] += (uint32_t)(t >> 26);
    return o;
}

// 16 message bytes (n < 16: the partial final block, 0x01 appended)
__device__ __forceinline__ void absorb(L5 &h, const uint8_t *p, uint32_t n) {
    uint32_t t[4] = {0, 0, 0, 0};
    uint32_t hib = 1u << 24;
    if (n == 16) {
        __builtin_memcpy(t, p, 16);
    } else {
        uint8_t b[16] = {0};
        for (uint32_t i = 0; i < n; ++i) b[i] = p[i];
        b[n] = 1;
        __builtin_memcpy(t, b, 16);
        hib = 0;
    }
    h.v[0] += t[0] & kM26;
    h.v[1] += ((t[0] >> 26) | (t[1] << 6)) & kM26;
    h.v[2] += ((t[1] >> 20) | (t[2] << 12)) & kM26;
    h.v[3] += ((t[2] >> 14) | (t[3] << 18)) & kM26;
    h.v[4] += (t[3] >> 8) | hib;
}

// absorb one block given as four little-endian words (n < 16: the partial
// final block, its bytes past n zero; 0x01 goes at byte n)
__device__ __forceinline__ void absorb_words(L5 &h, uint32_t (&t)[4], uint32_t n) {
    uint32_t hib = 1u << 24;
    if (n < 16) {
        t[n >> 2] |= 1u << (8 * (n & 3));
        hib = 0;
    }
    h.v[0] += t[0] & kM26;
    h.v[1] += ((t[0] >> 26) | (t[1] << 6)) & kM26;
    h.v[2] += ((t[1] >> 20) | (t[2] << 12)) & kM26;
    h.v[3] += ((t[2] >> 14) | (t[3] << 18)) & kM26;
    h.v[4] += (t[3] >> 8) | hib;
}

__device__ __forceinline__ L5 ld_l5(const uint32_t *p) {
    L5 r;
#pragma unroll
    for (int i = 0; i < 5; ++i) r.v[i] = p[i];
    return r;
}

__device__ __forceinline__ uint64_t wsum64(uint64_t v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, 64);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, 64);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}

// the tag: limb sums d (any size below 2^63) reduced mod 2^130 - 5, plus the
// four words of s, mod 2^128, written as 16 little-endian bytes
__device__ __forceinline__ void poly_final(uint64_t (&d)[5], const uint32_t (&s)[4], uint8_t *mac) {
    for (int pass = 0; pass < 3; ++pass) {
        for (int i = 0; i < 4; ++i) {
            d[i + 1] += d[i] >> 26;
            d[i] &= kM26;
        }
        d[0] += (d[4] >> 26) * 5;
        d[4] &= kM26;
    }
    d[1] += d[0] >> 26;
    d[0] &= kM26;
    uint32_t h0 = (uint32_t)d[0], h1 = (uint32_t)d[1], h2 = (uint32_t)d[2], h3 = (uint32_t)d[3],
             h4 = (uint32_t)d[4];
    // h - p = h + 5 - 2^130: keep it when it does not borrow
    uint32_t g0 = h0 + 5, cc = g0 >> 26;
    g0 &= kM26;
    uint32_t g1 = h1 + cc;
    cc = g1 >> 26;
    g1 &= kM26;
    uint32_t g2 = h2 + cc;
    cc = g2 >> 26;
    g2 &= kM26;
    uint32_t g3 = h3 + cc;
    cc = g3 >> 26;
    g3 &= kM26;
    const uint32_t g4 = h4 + cc - (1u << 26);
    if ((g4 >> 31) == 0) {
        h0 = g0;
        h1 = g1;
        h2 = g2;
        h3 = g3;
        h4 = g4;
    }
    // (h + s) mod 2^128, packing the limbs by addition so a limb that is not
    // fully normalised (h1 = 2^26) still lands right
    uint64_t f = (uint64_t)h0 + ((uint64_t)h1 << 26) + s[0];
    uint32_t o[4];
    o[0] = (uint32_t)f;
    f = (f >> 32) + ((uint64_t)h2 << 20) + s[1];
    o[1] = (uint32_t)f;
    f = (f >> 32) + ((uint64_t)h3 << 14) + s[2];
    o[2] = (uint32_t)f;
    f = (f >> 32) + ((uint64_t)h4 << 8) + s[3];
    o[3] = (uint32_t)f;
#pragma unroll
    for (int i = 0; i < 16; ++i) mac[i] = (uint8_t)(o[i >> 2] >> (8 * (i & 3)));
}

// h * r^e (e >= 1): r^u from the r^1..r^64 table (e = 64 t + u, u in 1..64),
// then r^(64 t) by the binary expansion of t over r^(64 * 2^j)
__device__ __forceinline__ L5 lift(L5 h, uint64_t e, const SealArgs &a) {
    const uint64_t u = ((e - 1) & 63) + 1;
    uint64_t t = (e - u) >> 6;
    h = pmul(h, ld_l5(a.rpow + (u - 1) * 5));
    for (int j = 0; t && j < kSealSq; ++j, t >>= 1)
        if (t & 1) h = pmul(h, ld_l5(a.rsq + j * 5));
    return h;
}

// The fused MAC's flush: each flushing lane lifts its Horner sum h (blocks
// last, last-64, ... of blob `blob`, 1-based `last`) to the blocks' final
// weights r^(N - i + 1) and adds the limbs into acc[blob]; when every
// flushing lane holds the same blob (a blob's end, a range's end) the wave
// adds them first and one lane issues the five atomics.  Called by the whole
// wave.
__device__ __forceinline__ void mac_flush(const SealArgs &a, const L5 &h, uint64_t blob,
                                          uint64_t last, bool fl, uint32_t lane) {
    const uint64_t m = __ballot(fl);
    if (!m) return;
    uint64_t v[5] = {0, 0, 0, 0, 0};
    if (fl) {
        const uint64_t N = a.prefix[blob + 1] - a.prefix[blob];
        const L5 x = lift(h, N - last + 1, a);
#pragma unroll
        for (int i = 0; i < 5; ++i) v[i] = x.v[i];
    }
    const int first = __builtin_ctzll(m);
    const uint64_t b0 = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(blob >> 32), first, 64) << 32) |
                        (uint32_t)__shfl((int)(uint32_t)blob, first, 64);
    if (__ballot(fl && blob != b0) == 0) {
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const uint64_t t = wsum64(v[i]);
            if (lane == (uint32_t)first) atomicAdd(a.acc + 5 * b0 + i, (unsigned long long)t);
        }
    } else if (fl) {
#pragma unroll
        for (int i = 0; i < 5; ++i) atomicAdd(a.acc + 5 * blob + i, (unsigned long long)v[i]);
    }
}

// ---- CTR: two T-tables with the byte index written by SDWA ------------------
// LDS row e (256 B) = [T0[e] x 32 lane copies | T1[e] = rotl8(T0[e]) x 32], so
// lookup (byte x, table k, lane copy c) is at x * 256 + k * 128 + c * 4: bank
// c, conflict-free within each 32-lane group.  Each lookup's address register
// holds k * 128 + c * 4 in byte 0 and zeros above; one v_mov_b32_sdwa
// writes the state byte into byte 1 and keeps the rest, so a lookup costs one
// single-source VALU instead of a bfe + lshl_or pair.  A column is
//   T0[a] ^ T1[b] ^ rotl16(T0[c] ^ T1[d]) ^ k   (one rotation, not three).
constexpr uint32_t kCtrWords = 256 * 64;   // 64 KiB

template <int B>
__device__ __forceinline__ void pick(uint32_t &a, uint32_t x) {
    if constexpr (B == 0)
        asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0" : "+v"(a) : "v"(x));
    else if constexpr (B == 1)
        asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1" : "+v"(a) : "v"(x));
    else if constexpr (B == 2)
        asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a) : "v"(x));
    else
        asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3" : "+v"(a) : "v"(x));
}

__device__ __forceinline__ uint32_t tl(const uint32_t *tab, uint32_t a) {
    return *(const uint32_t *)((const uint8_t *)tab + a);
}

template <int NB>
__device__ __forceinline__ void pick_all(uint32_t (&ix)[NB][16], const uint32_t (&s)[NB][4]) {
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            pick<0>(ix[b][4 * j], s[b][j]);
            pick<1>(ix[b][4 * j + 1], s[b][(j + 1) & 3]);
            pick<2>(ix[b][4 * j + 2], s[b][(j + 2) & 3]);
            pick<3>(ix[b][4 * j + 3], s[b][(j + 3) & 3]);
        }
}

// AES-256 of NB counter blocks per lane; rk: the 60 round-key words (uniform,
// read through the scalar cache)
template <int NB>
__device__ __forceinline__ void aes256_tab(uint32_t (&s)[NB][4], uint32_t (&ix)[NB][16],
                                           const uint32_t *tab, const uint32_t *__restrict__ rk) {
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int j = 0; j < 4; ++j) s[b][j] ^= rk[j];
#pragma unroll
    for (int r = 1; r < 14; ++r) {
        pick_all<NB>(ix, s);
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                s[b][j] = tl(tab, ix[b][4 * j]) ^ tl(tab, ix[b][4 * j + 1]) ^
                          rotl16(tl(tab, ix[b][4 * j + 2]) ^ tl(tab, ix[b][4 * j + 3])) ^ rk[4 * r + j];
    }
    // last round: S[x] is byte 1 of T0[x] and byte 2 of T1[x] (T0 = 2s,s,s,3s)
    pick_all<NB>(ix, s);
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            s[b][j] = (((tl(tab, ix[b][4 * j]) >> 8) & 0xffu) | ((tl(tab, ix[b][4 * j + 1]) >> 8) & 0xff00u) |
                       (tl(tab, ix[b][4 * j + 2]) & 0xff0000u) | (tl(tab, ix[b][4 * j + 3]) & 0xff000000u)) ^
                      rk[56 + j];
}

// Each wave seals a contiguous range of 128-block steps (2 blocks per lane:
// lane l takes blocks g0 + l and g0 + 64 + l, so each access is 1 KiB
// contiguous per wave); the blob index follows the range forward and the
// per-lane search runs only for steps that straddle a blob boundary.
// kCtrPer blocks per lane per step (ILP); two workgroups per CU (64 KiB of
// tables each), WPE waves per SIMD
template <int kCtrPer, int kThreads, int WPE, bool MAC = false, bool OPEN = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
void seal_ctr_kernel(SealArgs a) {
    static_assert(!OPEN || MAC, "Open verifies the MAC over its input in the same pass");
    static_assert(!MAC || kCtrPer == 1, "the fused MAC takes one block per lane per step");
    __shared__ uint32_t tab[kCtrWords];
    for (uint32_t i = threadIdx.x; i < kCtrWords; i += blockDim.x) {
        const uint32_t t = a.te0[i >> 6];
        tab[i] = (i & 32) ? rotl8(t) : t;
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, c4 = (lane & 31) * 4;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    constexpr uint32_t kStep = 64 * kCtrPer;
    const uint64_t steps = (a.total_blocks + kStep - 1) / kStep;
    const uint64_t per = (steps + nw - 1) / nw;
    const uint64_t s0 = wave * per, s1 = min(s0 + per, steps);
    if (s0 >= s1) return;
    uint32_t ix[kCtrPer][16];
#pragma unroll
    for (int b = 0; b < (int)kCtrPer; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) ix[b][i] = c4 + (i & 1) * 128;
    uint64_t blob = find_blob(a.prefix, a.n, s0 * kStep);
    // fused MAC (MAC): this lane's Horner sum over the ciphertext blocks it
    // sealed of blob mb (blocks 64 apart, the last one 1-based mlast)
    L5 mh{{0, 0, 0, 0, 0}};
    uint64_t mb = ~0ull, mlast = 0;
    L5 r64{{0, 0, 0, 0, 0}};
    if constexpr (MAC) r64 = ld_l5(a.rpow + 63 * 5);
    for (uint64_t st = s0; st < s1; ++st) {
        const uint64_t g0 = st * kStep;
        const uint64_t glast = min(g0 + kStep - 1, a.total_blocks - 1);
        while (a.prefix[blob + 1] <= g0) ++blob;
        const bool one = a.prefix[blob + 1] > glast;
        uint32_t s[kCtrPer][4];
        uint64_t off[kCtrPer], oof[kCtrPer];
        uint32_t nb[kCtrPer];
        uint64_t lb = blob, lq = 0;   // this lane's blob and block (MAC, kCtrPer == 1)
        if (one) {
            // the usual case: the whole step lies in one blob, so its
            // metadata is wave-uniform (scalar loads)
            const uint64_t pb = a.prefix[blob], ob = a.off[blob];
            const uint64_t oo = a.out_off ? a.out_off[blob] : ob;
            const uint32_t len = a.len[blob];
            uint32_t nn[4];
            load_nonce(a.nonces, blob, nn);
#pragma unroll
            for (int b = 0; b < (int)kCtrPer; ++b) {
                const uint64_t g = g0 + 64 * b + lane;
                const uint64_t q = g - pb;
                off[b] = ob + 16 * q;
                oof[b] = oo + 16 * q;
                nb[b] = g < a.total_blocks ? (uint32_t)min<uint64_t>(16, len - 16 * q) : 0;
                ctr_block(nn, q, s[b]);
                lq = q;
            }
        } else {
#pragma unroll
            for (int b = 0; b < (int)kCtrPer; ++b) {
                const uint64_t g = g0 + 64 * b + lane;
                const uint64_t gi = min(g, a.total_blocks - 1);
                const uint64_t bi = find_blob(a.prefix, a.n, gi);
                const uint64_t q = gi - a.prefix[bi];
                off[b] = a.off[bi] + 16 * q;
                oof[b] = (a.out_off ? a.out_off[bi] : a.off[bi]) + 16 * q;
                const uint32_t len = a.len[bi];
                nb[b] = g < a.total_blocks ? (uint32_t)min<uint64_t>(16, len - 16 * q) : 0;
                uint32_t nn[4];
                load_nonce(a.nonces, bi, nn);
                ctr_block(nn, q, s[b]);
                lb = bi;
                lq = q;
            }
        }
        // plaintext loaded before the rounds so its latency hides behind them
        uint4 v[kCtrPer];
#pragma unroll
        for (int b = 0; b < (int)kCtrPer; ++b)
            if (nb[b] == 16) __builtin_memcpy(&v[b], a.in + off[b], 16);
        aes256_tab<kCtrPer>(s, ix, tab, a.rk256);
#pragma unroll
        for (int b = 0; b < (int)kCtrPer; ++b) {
            uint32_t ct[4] = {0, 0, 0, 0};   // the ciphertext block, zero-padded (MAC)
            if (nb[b] == 16) {
                if constexpr (OPEN) {   // Open: the MAC covers the input (ciphertext)
                    ct[0] = v[b].x;
                    ct[1] = v[b].y;
                    ct[2] = v[b].z;
                    ct[3] = v[b].w;
                }
                v[b].x ^= s[b][0];
                v[b].y ^= s[b][1];
                v[b].z ^= s[b][2];
                v[b].w ^= s[b][3];
                __builtin_memcpy(a.out + oof[b], &v[b], 16);
                if constexpr (!OPEN) {
                    ct[0] = v[b].x;
                    ct[1] = v[b].y;
                    ct[2] = v[b].z;
                    ct[3] = v[b].w;
                }
            } else {
                for (uint32_t i = 0; i < nb[b]; ++i) {
                    const uint8_t x = a.in[off[b] + i];
                    const uint8_t c = x ^ (uint8_t)(s[b][i >> 2] >> (8 * (i & 3)));
                    a.out[oof[b] + i] = c;
                    ct[i >> 2] |= (uint32_t)(OPEN ? x : c) << (8 * (i & 3));
                }
            }
            if constexpr (MAC) {
                // a lane whose block starts another blob hands its sum over
                const bool act = nb[b] > 0;
                mac_flush(a, mh, mb, mlast, act && lb != mb && mb != ~0ull, lane);
                if (act) {
                    if (lb != mb) {
                        mh = L5{{0, 0, 0, 0, 0}};
                        mb = lb;
                    } else {
                        mh = pmul(mh, r64);
                    }
                    absorb_words(mh, ct, nb[b]);
                    mlast = lq + 1;
                }
            }
        }
    }
    if constexpr (MAC) mac_flush(a, mh, mb, mlast, mb != ~0ull, lane);
}

// fused MAC, last step: per blob, the limb sums reduced mod 2^130 - 5, plus
// s = AES-128(MACKey.K, nonce), mod 2^128
__global__ __launch_bounds__(256) void seal_fin_kernel(SealArgs a) {
    __shared__ uint32_t te[256 * kCopies];
    __shared__ uint32_t rk[44];
    load_te(te, a.te0);
    if (threadIdx.x < 44) rk[threadIdx.x] = a.rk128[threadIdx.x];
    __syncthreads();
    const uint32_t c = threadIdx.x & (kCopies - 1);
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < a.n;
         b += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t d[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) d[i] = a.acc[5 * b + i];
        uint32_t s[4];
        load_nonce(a.nonces, b, s);
        aes_encrypt(s, rk, 10, te, c);
        uint8_t tag[16];
        poly_final(d, s, tag);
        if (a.mode == kSealMacs) {
            for (int i = 0; i < 16; ++i) a.macs[16 * b + i] = tag[i];
        } else if (a.mode == kSealRecords) {
            // the record around the ciphertext: nonce before it, tag after it
            uint8_t *ct = a.out + a.out_off[b];
            for (int i = 0; i < 16; ++i) ct[(uint64_t)a.len[b] + i] = tag[i];
            for (int i = 0; i < 16; ++i) ct[i - 16] = a.nonces[16 * b + i];
        } else {
            uint32_t diff = 0;
            for (int i = 0; i < 16; ++i) diff |= tag[i] ^ a.macs[16 * b + i];
            a.bad[b] = diff != 0;
            if (diff) atomicAdd(a.n_bad, 1ull);
        }
    }
}

// Open's inputs gathered from stored records, one thread per blob
__global__ __launch_bounds__(256) void open_gather_kernel(const uint8_t *in, const uint64_t *rec_off,
                                                          const uint32_t *len, uint64_t n,
                                                          uint8_t *nonces, uint8_t *macs,
                                                          uint64_t *ct_off) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n) return;
    const uint8_t *r = in + rec_off[b];
    uint4 nn, mm;
    __builtin_memcpy(&nn, r, 16);
    __builtin_memcpy(&mm, r + 16 + len[b], 16);
    *(uint4 *)(nonces + 16 * b) = nn;
    *(uint4 *)(macs + 16 * b) = mm;
    ct_off[b] = rec_off[b] + 16;
}

__global__ __launch_bounds__(256) void put_u32_kernel(uint8_t *out, const uint64_t *pos,
                                                      const uint32_t *val, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int k = 0; k < 4; ++k) out[pos[i] + k] = (uint8_t)(val[i] >> (8 * k));
}

__global__ __launch_bounds__(256) void seal_mac_kernel(SealArgs a) {
    __shared__ uint32_t te[256 * kCopies];
    __shared__ uint32_t rk[44];
    load_te(te, a.te0);
    if (threadIdx.x < 44) rk[threadIdx.x] = a.rk128[threadIdx.x];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, c = lane & (kCopies - 1);
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    L5 R64, Re;
#pragma unroll
    for (int i = 0; i < 5; ++i) R64.v[i] = a.rpow[63 * 5 + i];
    for (uint64_t b = wave; b < a.n; b += nw) {
        const uint8_t *ct = a.out + a.off[b];
        const uint32_t len = a.len[b];
        const uint32_t N = (len + 15) / 16;
        L5 h{{0, 0, 0, 0, 0}};
        uint32_t last = 0;
        for (uint32_t i = lane; i < N; i += 64) {
            h = pmul(h, R64);
            absorb(h, ct + 16 * (uint64_t)i, min(16u, len - 16 * i));
            last = i + 1;   // 1-based index of this lane's last block
        }
        // lift by r^(N - last + 1) (1..64) and add the lanes
        uint64_t sumv[5] = {0, 0, 0, 0, 0};
        if (last) {
            const uint32_t e = N - last + 1;
#pragma unroll
            for (int i = 0; i < 5; ++i) Re.v[i] = a.rpow[(e - 1) * 5 + i];
            const L5 t = pmul(h, Re);
#pragma unroll
            for (int i = 0; i < 5; ++i) sumv[i] = t.v[i];
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) sumv[i] = wsum64(sumv[i]);
        // s = AES-128(MACKey.K, nonce): every lane computes it (uniform)
        uint32_t s[4];
        load_nonce(a.nonces, b, s);
        aes_encrypt(s, rk, 10, te, c);
        if (lane == 0) {
            uint64_t d[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) d[i] = sumv[i];
            poly_final(d, s, a.macs + 16 * b);
        }
    }
}

// ---- host: tables, key schedules, r powers ----------------------------------
uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }
uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    while (b) {
        if (b & 1) p ^= a;
        a = xtime(a);
        b >>= 1;
    }
    return p;
}
void sbox(uint8_t (&S)[256]) {
    // S[x] = affine(x^-1) over GF(2^8) with the AES polynomial (FIPS-197 5.1.1)
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = 0;
        if (x)
            for (int y = 1; y < 256; ++y)
                if (gmul((uint8_t)x, (uint8_t)y) == 1) {
                    inv = (uint8_t)y;
                    break;
                }
        uint8_t b = inv, r = inv;
        for (int i = 1; i < 5; ++i) {
            b = (uint8_t)((b << 1) | (b >> 7));
            r ^= b;
        }
        S[x] = r ^ 0x63;
    }
}
// FIPS-197 5.2 key expansion, round keys as LE column words
void expand(const uint8_t *key, int nk, const uint8_t (&S)[256], uint32_t *out) {
    const int nr = nk + 6, total = 4 * (nr + 1);
    std::vector<uint8_t> w((size_t)total * 4);
    memcpy(w.data(), key, (size_t)nk * 4);
    uint8_t rcon = 1;
    for (int i = nk; i < total; ++i) {
        uint8_t t[4];
        memcpy(t, &w[(size_t)(i - 1) * 4], 4);
        if (i % nk == 0) {
            const uint8_t t0 = t[0];
            t[0] = (uint8_t)(S[t[1]] ^ rcon);
            t[1] = S[t[2]];
            t[2] = S[t[3]];
            t[3] = S[t0];
            rcon = xtime(rcon);
        } else if (nk > 6 && i % nk == 4) {
            for (int k = 0; k < 4; ++k) t[k] = S[t[k]];
        }
        for (int k = 0; k < 4; ++k) w[(size_t)i * 4 + k] = w[(size_t)(i - nk) * 4 + k] ^ t[k];
    }
    for (int i = 0; i < total; ++i)
        out[i] = (uint32_t)w[4 * i] | ((uint32_t)w[4 * i + 1] << 8) | ((uint32_t)w[4 * i + 2] << 16) |
                 ((uint32_t)w[4 * i + 3] << 24);
}
// 130-bit host arithmetic for the r powers (limbs as the device uses them)
struct H5 {
    uint64_t v[5];
};
H5 hmul(const H5 &h, const H5 &r) {
    const uint64_t s1 = r.v[1] * 5, s2 = r.v[2] * 5, s3 = r.v[3] * 5, s4 = r.v[4] * 5;
    uint64_t d0 = h.v[0] * r.v[0] + h.v[1] * s4 + h.v[2] * s3 + h.v[3] * s2 + h.v[4] * s1;
    uint64_t d1 = h.v[0] * r.v[1] + h.v[1] * r.v[0] + h.v[2] * s4 + h.v[3] * s3 + h.v[4] * s2;
    uint64_t d2 = h.v[0] * r.v[2] + h.v[1] * r.v[1] + h.v[2] * r.v[0] + h.v[3] * s4 + h.v[4] * s3;
    uint64_t d3 = h.v[0] * r.v[3] + h.v[1] * r.v[2] + h.v[2] * r.v[1] + h.v[3] * r.v[0] + h.v[4] * s4;
    uint64_t d4 = h.v[0] * r.v[4] + h.v[1] * r.v[3] + h.v[2] * r.v[2] + h.v[3] * r.v[1] + h.v[4] * r.v[0];
    H5 o;
    d1 += d0 >> 26;
    o.v[0] = d0 & kM26;
    d2 += d1 >> 26;
    o.v[1] = d1 & kM26;
    d3 += d2 >> 26;
    o.v[2] = d2 & kM26;
    d4 += d3 >> 26;
    o.v[3] = d3 & kM26;
    o.v[4] = d4 & kM26;
    o.v[0] += (d4 >> 26) * 5;
    o.v[1] += o.v[0] >> 26;
    o.v[0] &= kM26;
    return o;
}

}  // namespace
}  // namespace vsgpu

using namespace vsgpu;

struct vs_seal {
    int device = 0;
    int cus = 256;
    DevBuf te0, rk256, rk128, rpow, prefix, acc;
    uint64_t *pinned = nullptr;   // the prefix total, read back
    // after the last run's kernels, on its stream: the next run (maybe on
    // another stream) waits for it before it rewrites prefix / acc
    hipEvent_t done = nullptr;
    bool ran = false;
    bool timing = false;
    bool fused = true;            // VS_OPT_SEAL_FUSED
    std::vector<hipEvent_t> ev;   // 3 per timed run: before CTR, between, after MAC
    // Open / pack scratch
    DevBuf o_nonce, o_mac, o_ctoff, o_cnt;
    DevBuf p_off, p_len, p_ctoff, p_nonce, p_hdr, p_hoff, p_hlen, p_hct, p_hnonce, p_tpos, p_tval,
        p_pack_off, p_pack_len, p_ids;
    DevBuf i_json, i_file;        // the index file (vs_restic_index)
    Stager stage;
};

VS_API int vs_seal_open(int device, const uint8_t enc_key[32], const uint8_t mac_k[16],
                        const uint8_t mac_r[16], vs_seal **out) {
    if (!out || !enc_key || !mac_k || !mac_r) return fail(VS_ERR_ARG, "bad arguments");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        return fail(VS_ERR_NO_DEVICE, "no HIP device available (no CPU fallback)");
    }
    if (device < 0 || device >= ndev) return fail(VS_ERR_ARG, "device index out of range");
    VS_TRY(enter_device(device));
    vs_seal *h = new vs_seal();
    h->device = device;
    if (hipDeviceGetAttribute(&h->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
        h->cus = 256;
    uint8_t S[256];
    sbox(S);
    uint32_t te[256];
    for (int x = 0; x < 256; ++x) {
        const uint8_t s = S[x], s2 = xtime(s), s3 = (uint8_t)(s2 ^ s);
        te[x] = (uint32_t)s2 | ((uint32_t)s << 8) | ((uint32_t)s << 16) | ((uint32_t)s3 << 24);
    }
    uint32_t rk256[60], rk128[44];
    expand(enc_key, 8, S, rk256);
    expand(mac_k, 4, S, rk128);
    // r clamped (RFC 8439; restic masks MACKey.R the same way), then r^1..r^64
    uint8_t rb[16];
    memcpy(rb, mac_r, 16);
    rb[3] &= 15;
    rb[7] &= 15;
    rb[11] &= 15;
    rb[15] &= 15;
    rb[4] &= 252;
    rb[8] &= 252;
    rb[12] &= 252;
    uint32_t t[4];
    memcpy(t, rb, 16);
    H5 r{{t[0] & kM26, ((t[0] >> 26) | (t[1] << 6)) & kM26, ((t[1] >> 20) | (t[2] << 12)) & kM26,
          ((t[2] >> 14) | (t[3] << 18)) & kM26, (t[3] >> 8)}};
    // r^1..r^64, then r^(64 * 2^j) for j < kSealSq (the fused MAC's lifts)
    std::vector<uint32_t> rp((64 + kSealSq) * 5);
    H5 p = r, r64 = r;
    for (int k = 0; k < 64; ++k) {
        for (int i = 0; i < 5; ++i) rp[(size_t)k * 5 + i] = (uint32_t)p.v[i];
        r64 = p;
        p = hmul(p, r);
    }
    for (int j = 0; j < kSealSq; ++j) {
        for (int i = 0; i < 5; ++i) rp[(size_t)(64 + j) * 5 + i] = (uint32_t)r64.v[i];
        r64 = hmul(r64, r64);
    }
    auto init = [&]() -> int {
        VS_TRY(h->te0.ensure(sizeof te));
        VS_TRY(h->rk256.ensure(sizeof rk256));
        VS_TRY(h->rk128.ensure(sizeof rk128));
        VS_TRY(h->rpow.ensure(rp.size() * 4));
        if (!(h->pinned = (uint64_t *)pinned_alloc(64)))
            return fail(VS_ERR_NOMEM, "pinned read-back word");
        VS_HIP(hipEventCreateWithFlags(&h->done, hipEventDisableTiming));
        // the key tables live in this frame: staged like any host memory the
        // library does not own (xfer.cpp)
        Stager st;
        int r = st.h2d(h->te0.p, te, sizeof te, nullptr);
        if (!r) r = st.h2d(h->rk256.p, rk256, sizeof rk256, nullptr);
        if (!r) r = st.h2d(h->rk128.p, rk128, sizeof rk128, nullptr);
        if (!r) r = st.h2d(h->rpow.p, rp.data(), rp.size() * 4, nullptr);
        st.release();   // waits for the copies
        return r;
    };
    const int rc = init();
    if (rc < 0) {
        const std::string msg = vs_last_error();
        vs_seal_close(h);
        set_error(msg);
        return rc;
    }
    *out = h;
    return 0;
}

// one launch of the seal / open engine over n device blobs (a carries the
// mode and the per-mode pointers); ordered after the handle's last run
static int seal_run(vs_seal *h, SealArgs a, const uint32_t *dev_len, size_t n, hipStream_t s) {
    if (h->ran) VS_HIP(hipStreamWaitEvent(s, h->done, 0));
    VS_TRY(h->prefix.ensure((n + 1) * 8));
    VS_HIP(launch_seal_prefix(dev_len, n, h->prefix.as<uint64_t>(), h->pinned, s));
    a.len = dev_len;
    a.n = n;
    a.prefix = h->prefix.as<uint64_t>();
    a.total_blocks = h->pinned[0];
    a.te0 = h->te0.as<uint32_t>();
    a.rk256 = h->rk256.as<uint32_t>();
    a.rk128 = h->rk128.as<uint32_t>();
    a.rpow = h->rpow.as<uint32_t>();
    a.rsq = a.rpow + 64 * 5;
    a.fused = h->fused;
    VS_TRY(h->acc.ensure(n * 5 * 8));
    a.acc = h->acc.as<unsigned long long>();
    hipEvent_t e[3] = {nullptr, nullptr, nullptr};
    if (h->timing) {
        for (auto &x : e) VS_HIP(hipEventCreate(&x));
        h->ev.insert(h->ev.end(), e, e + 3);
    }
    VS_HIP(launch_seal(a, h->cus, s, e));
    VS_HIP(hipEventRecord(h->done, s));
    h->ran = true;
    return 0;
}

VS_API int vs_seal_run_device(vs_seal *h, const void *dev_in, const uint64_t *dev_off,
                              const uint32_t *dev_len, size_t n, const uint8_t *dev_nonces,
                              uint8_t *dev_out, uint8_t *dev_macs, void *hip_stream) {
    if (!h || (n && (!dev_in || !dev_off || !dev_len || !dev_nonces || !dev_out || !dev_macs)))
        return fail(VS_ERR_ARG, "bad arguments");
    if (!n) return 0;
    if ((uintptr_t)dev_nonces & 15) return fail(VS_ERR_ARG, "nonces must be 16-byte aligned");
    VS_TRY(enter_device(h->device));
    SealArgs a{};
    a.in = (const uint8_t *)dev_in;
    a.out = dev_out;
    a.off = dev_off;
    a.nonces = dev_nonces;
    a.macs = dev_macs;
    a.mode = kSealMacs;
    return seal_run(h, a, dev_len, n, (hipStream_t)hip_stream);
}

VS_API int vs_seal_records_device(vs_seal *h, const void *dev_in, const uint64_t *dev_off,
                                  const uint32_t *dev_len, size_t n, const uint8_t *dev_nonces,
                                  uint8_t *dev_out, const uint64_t *dev_ct_off, void *hip_stream) {
    if (!h || (n && (!dev_in || !dev_off || !dev_len || !dev_nonces || !dev_out || !dev_ct_off)))
        return fail(VS_ERR_ARG, "bad arguments");
    if (!n) return 0;
    if ((uintptr_t)dev_nonces & 15) return fail(VS_ERR_ARG, "nonces must be 16-byte aligned");
    VS_TRY(enter_device(h->device));
    SealArgs a{};
    a.in = (const uint8_t *)dev_in;
    a.out = dev_out;
    a.off = dev_off;
    a.out_off = dev_ct_off;
    a.nonces = dev_nonces;
    a.mode = kSealRecords;
    return seal_run(h, a, dev_len, n, (hipStream_t)hip_stream);
}

VS_API int vs_open_run_device(vs_seal *h, const void *dev_in, const uint64_t *dev_rec_off,
                              const uint32_t *dev_len, size_t n, uint8_t *dev_out,
                              const uint64_t *dev_out_off, uint32_t *dev_bad, uint64_t *n_bad,
                              void *hip_stream) {
    if (n_bad) *n_bad = 0;
    if (!h || (n && (!dev_in || !dev_rec_off || !dev_len || !dev_out || !dev_bad)))
        return fail(VS_ERR_ARG, "bad arguments");
    if (!n) return 0;
    VS_TRY(enter_device(h->device));
    const hipStream_t s = (hipStream_t)hip_stream;
    if (h->ran) VS_HIP(hipStreamWaitEvent(s, h->done, 0));   // the scratch below
    VS_TRY(h->o_nonce.ensure(n * 16));
    VS_TRY(h->o_mac.ensure(n * 16));
    VS_TRY(h->o_ctoff.ensure(n * 8));
    VS_TRY(h->o_cnt.ensure(8));
    VS_HIP(launch_open_gather((const uint8_t *)dev_in, dev_rec_off, dev_len, n,
                              h->o_nonce.as<uint8_t>(), h->o_mac.as<uint8_t>(),
                              h->o_ctoff.as<uint64_t>(), s));
    VS_HIP(hipMemsetAsync(h->o_cnt.p, 0, 8, s));
    SealArgs a{};
    a.in = (const uint8_t *)dev_in;
    a.out = dev_out;
    a.off = h->o_ctoff.as<uint64_t>();
    a.out_off = dev_out_off ? dev_out_off : a.off;
    a.nonces = h->o_nonce.as<uint8_t>();
    a.macs = h->o_mac.as<uint8_t>();
    a.bad = dev_bad;
    a.n_bad = h->o_cnt.as<unsigned long long>();
    a.mode = kOpen;
    VS_TRY(seal_run(h, a, dev_len, n, s));
    if (n_bad) {
        VS_HIP(hipMemcpyAsync(h->pinned + 1, h->o_cnt.p, 8, hipMemcpyDeviceToHost, s));
        VS_HIP(hipStreamSynchronize(s));
        *n_bad = h->pinned[1];
    }
    return 0;
}

// restic v0.13.1 internal/repository: one packer per blob type; a blob is
// appended (Packer.Add) to its type's open pack, which is finalised once it
// holds >= min_pack_size bytes; Flush finalises the data pack, then the tree
// pack.  Finalize writes the header (per blob: type, record length, ID),
// sealed with the pack's own nonce, and its length as a 4-byte LE trailer.
struct PackPlan {
    std::vector<vs_pack> packs;
    std::vector<uint32_t> order;   // blob indices in pack order
    std::vector<uint64_t> ct_off;  // [blob] where its ciphertext goes
    uint64_t total = 0;
};

static void plan_packs(const uint32_t *len, const uint8_t *types, size_t n, uint64_t min_pack,
                       PackPlan &pl) {
    std::vector<uint32_t> cur[2];
    uint64_t size[2] = {0, 0};
    pl.ct_off.assign(n, 0);
    auto close = [&](int t) {
        if (cur[t].empty()) return;
        vs_pack p{};
        p.offset = pl.total;
        p.first_blob = (uint32_t)pl.order.size();
        p.n_blobs = (uint32_t)cur[t].size();
        uint64_t o = pl.total;
        for (const uint32_t i : cur[t]) {
            pl.order.push_back(i);
            pl.ct_off[i] = o + 16;
            o += (uint64_t)len[i] + 32;
        }
        o += 37ull * cur[t].size() + 32 + 4;   // sealed header + its length
        p.length = o - pl.total;
        pl.total = o;
        pl.packs.push_back(p);
        cur[t].clear();
        size[t] = 0;
    };
    for (size_t i = 0; i < n; ++i) {
        const int t = types[i] ? 1 : 0;
        cur[t].push_back((uint32_t)i);
        size[t] += (uint64_t)len[i] + 32;
        if (size[t] >= min_pack) close(t);
    }
    close(0);
    close(1);
}

VS_API int vs_restic_pack(vs_seal *h, vs_sha *sha, const void *dev_in, const uint64_t *off,
                          const uint32_t *len, const uint8_t *types, const uint8_t *ids, size_t n,
                          const uint8_t *blob_nonces, const uint8_t *hdr_nonces,
                          uint64_t min_pack_size, uint8_t *dev_out, uint64_t out_cap,
                          vs_pack *packs, size_t pack_cap, size_t *n_packs, uint64_t *out_len,
                          uint8_t *pack_ids, void *hip_stream) {
    if (!h || !n_packs || !out_len || (n && (!off || !len || !types || !ids)))
        return fail(VS_ERR_ARG, "bad arguments");
    for (size_t i = 0; i < n; ++i)
        if (types[i] > 1) return fail(VS_ERR_ARG, "blob type must be 0 (data) or 1 (tree)");
    PackPlan pl;
    plan_packs(len, types, n, std::max<uint64_t>(min_pack_size, 1), pl);
    *n_packs = pl.packs.size();
    *out_len = pl.total;
    if (packs) memcpy(packs, pl.packs.data(), std::min(pack_cap, pl.packs.size()) * sizeof(vs_pack));
    if (!dev_out) return 0;   // size query
    if (!sha || !dev_in || !blob_nonces || !hdr_nonces || !pack_ids || !packs)
        return fail(VS_ERR_ARG, "null pointer");
    if (out_cap < pl.total) return fail(VS_ERR_ARG, "pack output buffer too small");
    if (pack_cap < pl.packs.size()) return fail(VS_ERR_ARG, "pack descriptor array too small");
    if (!n) return 0;
    VS_TRY(enter_device(h->device));
    const hipStream_t s = (hipStream_t)hip_stream;
    if (h->ran) VS_HIP(hipStreamWaitEvent(s, h->done, 0));
    const size_t np = pl.packs.size();
    // 1. the blobs' records: nonce || AES-256-CTR ciphertext || Poly1305 tag
    VS_TRY(h->p_off.ensure(n * 8));
    VS_TRY(h->p_len.ensure(n * 4));
    VS_TRY(h->p_ctoff.ensure(n * 8));
    VS_TRY(h->p_nonce.ensure(n * 16));
    VS_TRY(h->stage.h2d(h->p_off.p, off, n * 8, s));
    VS_TRY(h->stage.h2d(h->p_len.p, len, n * 4, s));
    VS_TRY(h->stage.h2d(h->p_ctoff.p, pl.ct_off.data(), n * 8, s));
    VS_TRY(h->stage.h2d(h->p_nonce.p, blob_nonces, n * 16, s));
    {
        SealArgs a{};
        a.in = (const uint8_t *)dev_in;
        a.out = dev_out;
        a.off = h->p_off.as<uint64_t>();
        a.out_off = h->p_ctoff.as<uint64_t>();
        a.nonces = h->p_nonce.as<uint8_t>();
        a.mode = kSealRecords;
        VS_TRY(seal_run(h, a, h->p_len.as<uint32_t>(), n, s));
    }
    // 2. the headers (pack.go makeHeader: type, Length = record length, ID),
    // each sealed as one blob with its pack's nonce, after the records
    std::vector<uint8_t> hdr;
    std::vector<uint64_t> hoff(np), hct(np), tpos(np), poff(np), plen(np);
    std::vector<uint32_t> hlen(np), tval(np);
    for (size_t p = 0; p < np; ++p) {
        const vs_pack &pk = pl.packs[p];
        hoff[p] = hdr.size();
        for (uint32_t k = 0; k < pk.n_blobs; ++k) {
            const uint32_t i = pl.order[pk.first_blob + k];
            const uint32_t rl = len[i] + 32;
            hdr.push_back(types[i]);
            for (int b = 0; b < 4; ++b) hdr.push_back((uint8_t)(rl >> (8 * b)));
            hdr.insert(hdr.end(), ids + 32 * (size_t)i, ids + 32 * (size_t)i + 32);
        }
        hlen[p] = 37u * pk.n_blobs;
        const uint64_t end = pk.offset + pk.length;
        hct[p] = end - 4 - 16 - hlen[p];
        tpos[p] = end - 4;
        tval[p] = hlen[p] + 32;
        poff[p] = pk.offset;
        plen[p] = pk.length;
    }
    VS_TRY(h->p_hdr.ensure(hdr.size()));
    VS_TRY(h->p_hoff.ensure(np * 8));
    VS_TRY(h->p_hlen.ensure(np * 4));
    VS_TRY(h->p_hct.ensure(np * 8));
    VS_TRY(h->p_hnonce.ensure(np * 16));
    VS_TRY(h->p_tpos.ensure(np * 8));
    VS_TRY(h->p_tval.ensure(np * 4));
    VS_TRY(h->p_pack_off.ensure(np * 8));
    VS_TRY(h->p_pack_len.ensure(np * 4));
    VS_TRY(h->p_ids.ensure(np * 32));
    for (size_t p = 0; p < np; ++p)
        if (plen[p] > 0xffffffffull) return fail(VS_ERR_ARG, "a pack over 4 GiB");
    std::vector<uint32_t> plen32(plen.begin(), plen.end());
    VS_TRY(h->stage.h2d(h->p_hdr.p, hdr.data(), hdr.size(), s));
    VS_TRY(h->stage.h2d(h->p_hoff.p, hoff.data(), np * 8, s));
    VS_TRY(h->stage.h2d(h->p_hlen.p, hlen.data(), np * 4, s));
    VS_TRY(h->stage.h2d(h->p_hct.p, hct.data(), np * 8, s));
    VS_TRY(h->stage.h2d(h->p_hnonce.p, hdr_nonces, np * 16, s));
    VS_TRY(h->stage.h2d(h->p_tpos.p, tpos.data(), np * 8, s));
    VS_TRY(h->stage.h2d(h->p_tval.p, tval.data(), np * 4, s));
    VS_TRY(h->stage.h2d(h->p_pack_off.p, poff.data(), np * 8, s));
    VS_TRY(h->stage.h2d(h->p_pack_len.p, plen32.data(), np * 4, s));
    {
        SealArgs a{};
        a.in = h->p_hdr.as<uint8_t>();
        a.out = dev_out;
        a.off = h->p_hoff.as<uint64_t>();
        a.out_off = h->p_hct.as<uint64_t>();
        a.nonces = h->p_hnonce.as<uint8_t>();
        a.mode = kSealRecords;
        VS_TRY(seal_run(h, a, h->p_hlen.as<uint32_t>(), np, s));
    }
    VS_HIP(launch_put_u32(dev_out, h->p_tpos.as<uint64_t>(), h->p_tval.as<uint32_t>(), np, s));
    // 3. pack IDs: SHA-256 of each whole pack file
    VS_TRY(vs_sha256_run_device(sha, dev_out, h->p_pack_off.as<uint64_t>(),
                                h->p_pack_len.as<uint32_t>(), np, h->p_ids.as<uint8_t>(), s));
    VS_TRY(h->stage.d2h(pack_ids, h->p_ids.p, np * 32, s));
    VS_HIP(hipEventRecord(h->done, s));
    return 0;
}

// restic v0.13.1 internal/index Index.Encode (json.NewEncoder(w).Encode of
// jsonIndex{Packs: []packJSON{ID, Blobs: []blobJSON{ID, Type, Offset,
// Length}}}, "supersedes" omitted when empty): blob offsets and lengths are
// those of the records in the pack (Length = plaintext + 32, the stored
// length), types marshal as "data" / "tree", IDs as lower-case hex.  restic
// lists blobs in its index hash map's order, which a per-process random seed
// shuffles; this writes packs in finalize order and blobs in pack order, one
// of the orders restic's DecodeIndex reads back the same.
static void index_json(const PackPlan &pl, const uint32_t *len, const uint8_t *types,
                       const uint8_t *ids, const uint8_t *pack_ids, std::string &js) {
    static const char *hex = "0123456789abcdef";
    auto put_id = [&](const uint8_t *id) {
        js += '"';
        for (int b = 0; b < 32; ++b) {
            js += hex[id[b] >> 4];
            js += hex[id[b] & 15];
        }
        js += '"';
    };
    js = "{\"packs\":[";
    for (size_t p = 0; p < pl.packs.size(); ++p) {
        const vs_pack &pk = pl.packs[p];
        if (p) js += ',';
        js += "{\"id\":";
        put_id(pack_ids + 32 * p);
        js += ",\"blobs\":[";
        uint64_t off = 0;
        for (uint32_t k = 0; k < pk.n_blobs; ++k) {
            const uint32_t i = pl.order[pk.first_blob + k];
            const uint64_t rl = (uint64_t)len[i] + 32;
            if (k) js += ',';
            js += "{\"id\":";
            put_id(ids + 32 * (size_t)i);
            js += types[i] ? ",\"type\":\"tree\"" : ",\"type\":\"data\"";
            js += ",\"offset\":" + std::to_string(off) + ",\"length\":" + std::to_string(rl) + "}";
            off += rl;
        }
        js += "]}";
    }
    js += "]}\n";
}

VS_API int vs_restic_index(vs_seal *h, vs_sha *sha, const uint32_t *len, const uint8_t *types,
                           const uint8_t *ids, size_t n, uint64_t min_pack_size,
                           const uint8_t *pack_ids, const uint8_t nonce[16], uint8_t *json_out,
                           size_t json_cap, size_t *json_n, uint8_t *file_out, uint8_t file_id[32]) {
    if (!json_n || (n && (!len || !types || !ids || !pack_ids)))
        return fail(VS_ERR_ARG, "bad arguments");
    for (size_t i = 0; i < n; ++i)
        if (types[i] > 1) return fail(VS_ERR_ARG, "blob type must be 0 (data) or 1 (tree)");
    PackPlan pl;
    plan_packs(len, types, n, std::max<uint64_t>(min_pack_size, 1), pl);
    std::string js;
    index_json(pl, len, types, ids, pack_ids, js);
    *json_n = js.size();
    if (json_out) {
        if (json_cap < js.size()) return fail(VS_ERR_ARG, "index JSON buffer too small");
        memcpy(json_out, js.data(), js.size());
    }
    if (!file_out) return 0;   // the plaintext only
    if (!h || !sha || !nonce || !file_id) return fail(VS_ERR_ARG, "null handle or output");
    if (js.size() > 0xffffffffull - 32) return fail(VS_ERR_ARG, "index over 4 GiB");
    // repository.SaveUnpacked: Key.Seal(nonce) -> nonce || ciphertext || tag,
    // stored under the SHA-256 of those bytes
    VS_TRY(enter_device(h->device));
    const hipStream_t s = nullptr;
    if (h->ran) VS_HIP(hipStreamWaitEvent(s, h->done, 0));
    const uint64_t flen = js.size() + 32;
    VS_TRY(h->i_json.ensure(js.size() + 16));
    VS_TRY(h->i_file.ensure(flen + 16));
    VS_TRY(h->p_hoff.ensure(8));
    VS_TRY(h->p_hlen.ensure(4));
    VS_TRY(h->p_hct.ensure(8));
    VS_TRY(h->p_hnonce.ensure(16));
    VS_TRY(h->p_ids.ensure(32));
    const uint64_t zero = 0, ct = 16;
    const uint32_t jl = (uint32_t)js.size(), fl = (uint32_t)flen;
    VS_TRY(h->stage.h2d(h->i_json.p, js.data(), js.size(), s));
    VS_TRY(h->stage.h2d(h->p_hoff.p, &zero, 8, s));
    VS_TRY(h->stage.h2d(h->p_hlen.p, &jl, 4, s));
    VS_TRY(h->stage.h2d(h->p_hct.p, &ct, 8, s));
    VS_TRY(h->stage.h2d(h->p_hnonce.p, nonce, 16, s));
    {
        SealArgs a{};
        a.in = h->i_json.as<uint8_t>();
        a.out = h->i_file.as<uint8_t>();
        a.off = h->p_hoff.as<uint64_t>();
        a.out_off = h->p_hct.as<uint64_t>();
        a.nonces = h->p_hnonce.as<uint8_t>();
        a.mode = kSealRecords;
        VS_TRY(seal_run(h, a, h->p_hlen.as<uint32_t>(), 1, s));
    }
    // the file's ID by the SHA-256 engine (offset 0, flen bytes)
    VS_TRY(h->p_pack_len.ensure(4));
    VS_TRY(h->stage.h2d(h->p_pack_len.p, &fl, 4, s));
    VS_TRY(vs_sha256_run_device(sha, h->i_file.p, h->p_hoff.as<uint64_t>(),
                                h->p_pack_len.as<uint32_t>(), 1, h->p_ids.as<uint8_t>(), s));
    VS_TRY(h->stage.d2h(file_out, h->i_file.p, flen, s));
    VS_TRY(h->stage.d2h(file_id, h->p_ids.p, 32, s));
    VS_HIP(hipEventRecord(h->done, s));
    return 0;
}

VS_API int vs_seal_set_option(vs_seal *h, int option, int64_t value) {
    if (!h) return fail(VS_ERR_ARG, "null handle");
    if (option != VS_OPT_SEAL_FUSED) return fail(VS_ERR_ARG, "unknown vs_seal option");
    if (h->ran) VS_HIP(hipEventSynchronize(h->done));
    h->fused = value != 0;
    return 0;
}

VS_API int vs_seal_set_timing(vs_seal *h, int on) {
    if (!h) return fail(VS_ERR_ARG, "bad arguments");
    h->timing = on != 0;
    return 0;
}

VS_API int vs_seal_kernel_ms(vs_seal *h, double ms[2], int *runs) {
    if (!h || !ms || !runs) return fail(VS_ERR_ARG, "bad arguments");
    ms[0] = ms[1] = 0;
    *runs = (int)(h->ev.size() / 3);
    for (size_t i = 0; i + 2 < h->ev.size(); i += 3) {
        float a = 0, b = 0;
        VS_HIP(hipEventSynchronize(h->ev[i + 2]));
        VS_HIP(hipEventElapsedTime(&a, h->ev[i], h->ev[i + 1]));
        VS_HIP(hipEventElapsedTime(&b, h->ev[i + 1], h->ev[i + 2]));
        ms[0] += a;
        ms[1] += b;
    }
    for (hipEvent_t x : h->ev) (void)hipEventDestroy(x);
    h->ev.clear();
    return 0;
}

VS_API void vs_seal_close(vs_seal *h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)hipDeviceSynchronize();
    for (hipEvent_t x : h->ev) (void)hipEventDestroy(x);
    for (DevBuf *b : {&h->te0, &h->rk256, &h->rk128, &h->rpow, &h->prefix, &h->acc, &h->o_nonce,
                      &h->o_mac, &h->o_ctoff, &h->o_cnt, &h->p_off, &h->p_len, &h->p_ctoff,
                      &h->p_nonce, &h->p_hdr, &h->p_hoff, &h->p_hlen, &h->p_hct, &h->p_hnonce,
                      &h->p_tpos, &h->p_tval, &h->p_pack_off, &h->p_pack_len, &h->p_ids})
        b->release();
    h->stage.release();
    pinned_free(h->pinned);
    if (h->done) (void)hipEventDestroy(h->done);
    delete h;
}

namespace vsgpu {

namespace {
constexpr uint32_t kScanThreads = 1024, kScanPer = 16;

// prefix[i] = 16-byte blocks of blobs [0, i) for i <= n, in one workgroup:
// tiles of 16 K blobs, 16 consecutive blobs per thread, a workgroup scan of
// the thread sums in LDS carried from tile to tile.  n is a blob count
// (~45 K for a 64 GiB volume), so a single workgroup is microseconds.
__global__ __launch_bounds__(kScanThreads) void seal_prefix_kernel(const uint32_t *len, uint64_t n,
                                                                   uint64_t *prefix) {
    __shared__ uint64_t part[kScanThreads];
    const uint32_t t = threadIdx.x;
    uint64_t carry = 0;
    for (uint64_t base = 0; base <= n; base += (uint64_t)kScanThreads * kScanPer) {
        const uint64_t i0 = base + (uint64_t)t * kScanPer;
        uint64_t v[kScanPer], sum = 0;
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; ++k) {
            v[k] = (i0 + k < n) ? (len[i0 + k] + 15u) / 16u : 0;
            sum += v[k];
        }
        part[t] = sum;
        __syncthreads();
        for (uint32_t d = 1; d < kScanThreads; d <<= 1) {   // inclusive Hillis-Steele
            const uint64_t x = t >= d ? part[t - d] : 0;
            __syncthreads();
            part[t] += x;
            __syncthreads();
        }
        uint64_t run = carry + part[t] - sum;   // exclusive prefix of this thread's first blob
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; ++k) {
            if (i0 + k <= n) prefix[i0 + k] = run;
            run += v[k];
        }
        carry += part[kScanThreads - 1];
        __syncthreads();
    }
}
}  // namespace

hipError_t launch_open_gather(const uint8_t *in, const uint64_t *rec_off, const uint32_t *len,
                              uint64_t n, uint8_t *nonces, uint8_t *macs, uint64_t *ct_off,
                              hipStream_t s) {
    if (!n) return hipSuccess;
    open_gather_kernel<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(in, rec_off, len, n, nonces, macs,
                                                                 ct_off);
    return hipGetLastError();
}

hipError_t launch_put_u32(uint8_t *out, const uint64_t *pos, const uint32_t *val, uint64_t n,
                          hipStream_t s) {
    if (!n) return hipSuccess;
    put_u32_kernel<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(out, pos, val, n);
    return hipGetLastError();
}

// prefix[i] = blocks of blobs [0, i), prefix[n] = *total (read back: waits)
hipError_t launch_seal_prefix(const uint32_t *len, uint64_t n, uint64_t *prefix, uint64_t *total,
                              hipStream_t s) {
    seal_prefix_kernel<<<1, kScanThreads, 0, s>>>(len, n, prefix);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = hipMemcpyAsync(total, prefix + n, 8, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(s);
}

hipError_t launch_seal(const SealArgs &a, int cus, hipStream_t s, hipEvent_t *ev) {
    // default: the MAC fused into the CTR pass (no re-read of the ciphertext),
    // 768-thread workgroups at 6 waves per SIMD; VS_OPT_SEAL_FUSED = 0 selects
    // the separate CTR + MAC kernels (A/B and tests)
    const bool fused = a.fused || a.mode != kSealMacs;
    if (fused) {
        hipError_t e = hipMemsetAsync(a.acc, 0, a.n * 5 * 8, s);
        if (e != hipSuccess) return e;
        if (ev[0]) (void)hipEventRecord(ev[0], s);
        if (a.total_blocks) {
            const uint64_t steps = (a.total_blocks + 63) / 64;
            const uint64_t grid = std::min<uint64_t>((steps + 11) / 12, (uint64_t)std::max(cus, 1) * 2);
            if (a.mode == kOpen)
                seal_ctr_kernel<1, 768, 6, true, true><<<(uint32_t)grid, 768, 0, s>>>(a);
            else
                seal_ctr_kernel<1, 768, 6, true><<<(uint32_t)grid, 768, 0, s>>>(a);
        }
        if (ev[1]) (void)hipEventRecord(ev[1], s);
        const uint64_t fg = std::min<uint64_t>((a.n + 255) / 256, (uint64_t)std::max(cus, 1) * 4);
        seal_fin_kernel<<<(uint32_t)std::max<uint64_t>(fg, 1), 256, 0, s>>>(a);
        if (ev[2]) (void)hipEventRecord(ev[2], s);
        return hipGetLastError();
    }
    if (ev[0]) (void)hipEventRecord(ev[0], s);
    if (a.total_blocks) {
        // 1 block per lane, 1024 threads, 8 waves per SIMD: 22.0 ms per 16 GiB
        // of blobs against 22.6 / 22.8 ms for 2 / 3 blocks per lane at 512
        // threads (r02).  LDS-issue bound (2 cycles per ds_read_b32, 224
        // lookups per block): SQ_LDS_IDX_ACTIVE is ~65 % of the cycles.
        const uint64_t steps = (a.total_blocks + 63) / 64;
        const uint64_t grid = std::min<uint64_t>((steps + 15) / 16, (uint64_t)std::max(cus, 1) * 2);
        seal_ctr_kernel<1, 1024, 8><<<(uint32_t)grid, 1024, 0, s>>>(a);
    }
    if (ev[1]) (void)hipEventRecord(ev[1], s);
    const uint64_t mg = std::min<uint64_t>((a.n + 3) / 4, (uint64_t)std::max(cus, 1) * 8);
    seal_mac_kernel<<<(uint32_t)std::max<uint64_t>(mg, 1), 256, 0, s>>>(a);
    if (ev[2]) (void)hipEventRecord(ev[2], s);
    return hipGetLastError();
}

}  // namespace vsgpu
