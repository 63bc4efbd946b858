// sha256.hip -- batched SHA-256 blob IDs on gfx950: the time-sliced
// producer/consumer hash engine.
//
// restic's blob ID is sha256.Sum256 of the chunk plaintext
// (restic v0.13.1 internal/restic/id.go Hash, Go crypto/sha256 after
// /root/reference/mover-restic/patch-sources.sh:16-27), computed for every
// chunk in Repository.SaveBlob.
//
// A blob's Merkle-Damgard chain is sequential, so parallelism is across
// blobs ("chains").  Two facts shape the kernel:
//   * a wave alone on its SIMD issues one VALU instruction per 4 cycles, so a
//     chain's latency is its per-lane instruction count: the longest chunk
//     (MaxSize = 8 MiB = 131072 blocks) is the critical path of a volume;
//   * chains of one volume (~44 K at 64 GiB) fill only a fraction of the
//     256 CU x 4 SIMD x 2 waves x 64 lanes the chip can keep busy.
// Hence:
//   * producer/consumer split: per 64 chains a workgroup of two waves; the
//     producer loads message blocks and expands the schedule W[0..63] + K into
//     an LDS double buffer, the consumer runs only the 64 rounds (14 VALU per
//     round + 16 ds_read_b128 per block instead of ~1460 VALU per block), so a
//     chain advances ~1.6x faster than with one lane doing both;
//   * time slicing: a launch advances every active chain by at most `budget`
//     blocks and writes the midstate of unfinished chains to the next active
//     list, so the chains of consecutive volumes share launches on one stream
//     (no hardware-queue serialisation) and the chip stays full in steady
//     state.
// Chains are processed in tiles of 64 taken longest-first from a work queue;
// v_bitop3_b32 does Ch / Maj / three-way XORs, v_alignbit_b32 the rotates and
// v_perm_b32 the big-endian, byte-misaligned message words.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <thread>

#include "internal.hpp"

namespace vsgpu {

static constexpr uint32_t kK256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
    0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
    0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
    0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
    0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
    0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
    0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
    0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};

static constexpr uint32_t kIV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                    0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) {
    return __builtin_amdgcn_alignbit(x, x, n);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
    return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);  // e ? f : g
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

// Blocks (data + padding) still to compress for a chain whose next unread
// byte is ptr and whose data ends at end.  end - ptr < 0 only while the
// second padding block (tail >= 56 bytes) is pending.
__device__ __forceinline__ uint32_t blocks_left(uint64_t ptr, uint64_t end) {
    const int64_t d = (int64_t)(end - ptr);
    if (d < 0) return 1;
    const uint64_t b = ((uint64_t)d >> 6) + (((uint64_t)d & 63) < 56 ? 1u : 2u);
    return b > 0xffffffffull ? 0xffffffffu : (uint32_t)b;
}

// Block data reaches the producer by cooperative, coalesced loads.  A chain's
// bytes are read as aligned 16-byte segments: block j of a slice starting at
// ptr covers the segments at A + 64 j + 16 s, s = 0..4, with A = ptr & ~15
// (ptr & 15 is the same for every block of a chain); segment 4 of block j is
// segment 0 of block j+1, so a block needs segments 1..4.  For those, lane m
// of load instruction i (i = 0..3) fetches segment 1 + m % 4 of chain
// 16 i + m / 4: one instruction touches 16 chains (16 pages) instead of 64,
// which is what the address-translation path can sustain.  The segments are
// staged in the free LDS slot and each lane reads back its own chain's four.
// A segment with no byte of the blob is read from `safe` (the blob's last
// segment, or the digest slot of an empty blob): every load is
// unconditional and in mapped memory; message() masks bytes past the end.
// Global address space: the loads count only in vmcnt, so the prefetch stays
// in flight across the LDS barrier.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;

__device__ __forceinline__ uint4 load_seg(uint64_t a, uint64_t end, uint64_t safe) {
    const u32x4 v = *(gu32x4 *)(uintptr_t)(a < end ? a : safe);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Raw little-endian words d[0..16] of a block from its five segments s0 and
// s[0..3]: d[k] = word k + q of that 80-byte window, q = (ptr & 15) >> 2.
__device__ __forceinline__ void window_words(uint32_t (&d)[17], const uint4 &s0,
                                             const uint4 (&s)[4], uint32_t q) {
    const uint32_t win[20] = {s0.x,   s0.y,   s0.z,   s0.w,   s[0].x, s[0].y, s[0].z,
                              s[0].w, s[1].x, s[1].y, s[1].z, s[1].w, s[2].x, s[2].y,
                              s[2].z, s[2].w, s[3].x, s[3].y, s[3].z, s[3].w};
    // bit selects (v_bitop3), not a ternary on q: the compiler turns that into
    // a dynamically indexed private array, i.e. scratch memory
    const uint32_t m1 = 0u - (q & 1u), m2 = 0u - ((q >> 1) & 1u);
    uint32_t t[19];
#pragma unroll
    for (int i = 0; i < 19; ++i) t[i] = ch(m1, win[i + 1], win[i]);
#pragma unroll
    for (int k = 0; k < 17; ++k) d[k] = ch(m2, t[k + 2], t[k]);
}

// Big-endian message words W[0..15] of the block at ptr from its raw words.
__device__ __forceinline__ void message(uint32_t (&w)[16], const uint32_t (&d)[17], uint64_t ptr,
                                        uint64_t end, uint64_t len) {
    const uint32_t r = (uint32_t)(ptr & 3);
    const uint32_t sel = (r << 24) | ((r + 1) << 16) | ((r + 2) << 8) | (r + 3);
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = __builtin_amdgcn_perm(d[k + 1], d[k], sel);
    const int64_t left = (int64_t)(end - ptr);
    if (left < 64) {
        // padding: [tail bytes, 0x80, zeros] (+ big-endian bit length)
        const int tl = left > 0 ? (int)left : 0;
        const bool mark = left >= 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int v = min(max(tl - 4 * k, 0), 4);  // tail bytes in word k
            const uint32_t keep = (v == 4) ? 0xffffffffu : ~(0xffffffffu >> (8 * v));
            const uint32_t m80 = (mark && v < 4 && tl >= 4 * k) ? (0x80u << (24 - 8 * v)) : 0u;
            w[k] = (w[k] & keep) | m80;
        }
        if (left < 56) {
            const uint64_t bits = len << 3;
            w[14] = (uint32_t)(bits >> 32);
            w[15] = (uint32_t)bits;
        }
    }
}

// W slot layouts: split tiles (64 chains, word group q of lane l at uint4
// q*64 + l: conflict-free ds_write_b128 / ds_read_b128); latency tiles (16
// chains at q*16 + lane, K added here, so a lane that reads a zero slot gets
// exactly 0); isolated latency tiles (the same, one word early: uint4 q holds
// words 4q+1 .. 4q+4 and word 0 ends uint4 15, so an eight-round group of
// compress_quad_iso reads exactly two uint4s).
enum { kSlotSplit = 0, kSlotQuad = 1, kSlotQuadEarly = 2 };

// Producer: W[t] (+ K[t]) for t = 0..63 into an LDS slot of layout L.
template <int L, int CS = 16>   // CS: chains per slot (latency layouts)
__device__ __forceinline__ void schedule_to_lds(uint32_t (&w)[16], uint4 *slot, uint32_t lane) {
    uint32_t k0 = 0, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int t = 4 * q + i;
            uint32_t wt;
            if (t < 16) {
                wt = w[t];
            } else {
                const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
                const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
                const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
                wt = w[t & 15] = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
            }
            o[i] = L == kSlotSplit ? wt : wt + kK256[t];
        }
        if constexpr (L == kSlotQuadEarly) {
            if (q == 0) k0 = o[0];
            else slot[(q - 1) * CS + lane] = make_uint4(c1, c2, c3, o[0]);
            c1 = o[1];
            c2 = o[2];
            c3 = o[3];
        } else {
            slot[q * (L == kSlotQuad ? CS : 64) + lane] = make_uint4(o[0], o[1], o[2], o[3]);
        }
    }
    if constexpr (L == kSlotQuadEarly) slot[15 * CS + lane] = make_uint4(c1, c2, c3, k0);
}

#define VS_SHA_ROUND(a, b, c, d, e, f, g, h, wk)                                   \
    {                                                                              \
        const uint32_t t1_ = h + xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)) +       \
                             ch(e, f, g) + (wk);                                   \
        const uint32_t t2_ = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)) + maj(a, b, c); \
        d += t1_;                                                                  \
        h = t1_ + t2_;                                                             \
    }

// Consumer: the 64 rounds of one block from the LDS slot.
__device__ __forceinline__ void compress_lds(uint32_t (&st)[8], const uint4 *slot, uint32_t lane) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int q = 0; q < 16; q += 2) {
        const uint4 v = slot[q * 64 + lane];
        const uint4 u = slot[(q + 1) * 64 + lane];
        // + K[t] here rather than in the producer: a scalar operand of the
        // v_add3 the round needs anyway
        VS_SHA_ROUND(a, b, c, d, e, f, g, h, v.x + kK256[4 * q + 0])
        VS_SHA_ROUND(h, a, b, c, d, e, f, g, v.y + kK256[4 * q + 1])
        VS_SHA_ROUND(g, h, a, b, c, d, e, f, v.z + kK256[4 * q + 2])
        VS_SHA_ROUND(f, g, h, a, b, c, d, e, v.w + kK256[4 * q + 3])
        VS_SHA_ROUND(e, f, g, h, a, b, c, d, u.x + kK256[4 * q + 4])
        VS_SHA_ROUND(d, e, f, g, h, a, b, c, u.y + kK256[4 * q + 5])
        VS_SHA_ROUND(c, d, e, f, g, h, a, b, u.z + kK256[4 * q + 6])
        VS_SHA_ROUND(b, c, d, e, f, g, h, a, u.w + kK256[4 * q + 7])
    }
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
    st[4] += e;
    st[5] += f;
    st[6] += g;
    st[7] += h;
}
#undef VS_SHA_ROUND

// Latency (quad) consumer: four lanes per chain, so one wave's instruction
// stream advances a chain with 10 VALU and a select per round instead of the
// split form's 14 (compress_quad_iso below drops the select).  Lane roles
// in a quad: 0 runs the e-path (cur = e, history f, g, h), 1 the a-path
// (cur = a, history b, c, d), 2 and 3 hold zeros.  Per round, with per-lane
// rotation amounts and masks:
//   S = Sigma1(e) | Sigma0(a)            (3 v_alignbit by per-lane amounts + xor3)
//   X = e | ~(a ^ b)                      (one v_bitop3: o ^ (m & ~p))
//   C = Ch(X, p1, p2) = Ch(e,f,g) | Maj(a,b,c)   (Maj(a,b,c) = Ch(~(a^b), b, c))
//   Z = h + (K + W) | 0                   (DPP: lane 1 reads lane 2's zero)
//   T = S + C + Z = T1 | T2
//   new = DPP-swap(T1 | d) + T = d + T1 (e') | T1 + T2 (a')
// K + W comes from the producer; lanes 1-3 read a zero slot instead.
struct QuadLane {
    uint32_t s1, s2, s3;  // rotation amounts: Sigma1 (6, 11, 25) / Sigma0 (2, 13, 22)
    uint32_t m;           // 0 / ~0: the Maj transform in lane 1
    bool l1;              // the a-path lane
};

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}

// z: this round's h + (K + W) | 0, computed one round ahead (from p2, the
// next round's p3) so it fills the wait states between the select and the
// DPP add that reads it
#define VS_QUAD_ROUND(cur, p1, p2, p3, z, kwn)                                               \
    {                                                                                        \
        const uint32_t s_ = xor3(__builtin_amdgcn_alignbit(cur, cur, ql.s1),                \
                                 __builtin_amdgcn_alignbit(cur, cur, ql.s2),                 \
                                 __builtin_amdgcn_alignbit(cur, cur, ql.s3));                \
        const uint32_t x_ = __builtin_amdgcn_bitop3_b32(cur, p1, ql.m, 0xD2);               \
        const uint32_t c_ = ch(x_, p1, p2);                                                  \
        const uint32_t t_ = s_ + c_ + z;                                                     \
        const uint32_t a_ = ql.l1 ? p3 : t_;                                                 \
        z = dpp_u32<0xA8>(p2) + (kwn); /* quad_perm [0,2,2,2] */                            \
        p3 = dpp_u32<0xB1>(a_) + t_;   /* quad_perm [1,0,3,2] */                            \
    }

// Isolated latency tiles (a CU each) use a second form: one
// DPP add per round and no select.  Lane 0 folds d into its sum (T = T1 + d =
// e'), lane 1 carries -d (T = T2 - d), and the new value is T + the quad's
// lane-2 zero (lane 0) / lane 0's T (lane 1):
//   Z = h + (K + W) + d | -d | 0          (one round ahead: v_xad + DPP add)
//   new = DPP[2,0,2,2](T) + T = e' | T1 + T2 | 0
// Lane 1 reads a slot of ones for K + W, so (~c) + 1 = -c exactly.  Eight
// rounds per asm statement (hipcc reassociates Z into T, 13 VALU, or pads
// wait states, when it schedules the round itself): 10 VALU per round and no
// s_nop.  Measured alone on a SIMD (tools/probe/quad_round.hip): 47.9 cycles
// per round against the select form's 64.8.  The K + W slot is one word early
// (kSlotQuadEarly) so a group reads exactly two uint4s.  Wait states inside:
// the DPP read of T follows its v_add3 by two instructions; the DPP read of p2
// is of a value written three rounds before (s_nop 1 opens a block's first
// group, whose p2 comes from hipcc's code).
#define VS_QA(cur, p1, p2, p3, k)                                                           \
    "v_alignbit_b32 %[r1], %[" #cur "], %[" #cur "], %[s1]\n\t"                            \
    "v_alignbit_b32 %[r2], %[" #cur "], %[" #cur "], %[s2]\n\t"                            \
    "v_alignbit_b32 %[r3], %[" #cur "], %[" #cur "], %[s3]\n\t"                            \
    "v_bitop3_b32 %[xx], %[" #cur "], %[" #p1 "], %[m] bitop3:0xd2\n\t"                    \
    "v_bitop3_b32 %[r1], %[r1], %[r2], %[r3] bitop3:0x96\n\t"                              \
    "v_bitop3_b32 %[xx], %[xx], %[" #p1 "], %[" #p2 "] bitop3:0xca\n\t"                    \
    "v_add3_u32 %[tt], %[r1], %[xx], %[z]\n\t"                                             \
    "v_xad_u32 %[yy], %[" #p2 "], %[m], %[" #k "]\n\t"                                      \
    "v_add_u32_dpp %[z], %[" #p2 "], %[yy] quad_perm:[1,2,2,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t" \
    "v_add_u32_dpp %[" #p3 "], %[tt], %[tt] quad_perm:[2,0,2,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"

// extra arguments: unused inputs (they make hipcc issue those loads earlier)
#define VS_QUAD8(pre, A, B, ...)                                                             \
    {                                                                                        \
        uint32_t r1, r2, r3, xx, tt, yy;                                                     \
        asm(pre VS_QA(x0, x1, x2, x3, k0) VS_QA(x3, x0, x1, x2, k1) VS_QA(x2, x3, x0, x1, k2) \
                VS_QA(x1, x2, x3, x0, k3) VS_QA(x0, x1, x2, x3, k4) VS_QA(x3, x0, x1, x2, k5) \
                    VS_QA(x2, x3, x0, x1, k6) VS_QA(x1, x2, x3, x0, k7)                       \
            : [x0] "+v"(x0), [x1] "+v"(x1), [x2] "+v"(x2), [x3] "+v"(x3), [z] "+v"(z),       \
              [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3), [xx] "=&v"(xx), [tt] "=&v"(tt), \
              [yy] "=&v"(yy)                                                                 \
            : [k0] "v"(A.x), [k1] "v"(A.y), [k2] "v"(A.z), [k3] "v"(A.w), [k4] "v"(B.x),      \
              [k5] "v"(B.y), [k6] "v"(B.z), [k7] "v"(B.w), [m] "v"(ql.m), [s1] "v"(ql.s1),   \
              [s2] "v"(ql.s2), [s3] "v"(ql.s3), ##__VA_ARGS__);                              \
    }

// One block in the isolated form, its first K + W words (kz = word 0, a, b =
// words 1..8) already in registers; returns the next block's (from kwn).
template <int CS = 16>   // chains per K + W slot
__device__ __forceinline__ void compress_quad_iso(uint32_t (&x)[4], const uint4 *kw, const uint4 *kwn,
                                                  const QuadLane &ql, uint32_t &kz, uint4 &a, uint4 &b) {
    uint32_t x0 = x[0], x1 = x[1], x2 = x[2], x3 = x[3];
    uint32_t z = dpp_u32<0xA9>(x3) + ((x3 ^ ql.m) + kz);
    // the next block's first words ride as unused inputs of groups 6 and 7,
    // so hipcc issues their loads a group ahead and they land while a group
    // runs (left to itself it sinks them below the last group and waits)
    const uint4 pa = kwn[0], pb = kwn[CS];
    const uint32_t pz = kwn[15 * CS].w;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        uint4 na = pa, nb = pb;
        if (g < 7) {
            na = kw[(2 * g + 2) * CS];
            nb = kw[(2 * g + 3) * CS];
        }
        if (g == 0)
            VS_QUAD8("s_nop 1\n\t", a, b)
        else if (g == 6)
            VS_QUAD8("", a, b, "v"(pa.x), "v"(pa.y), "v"(pa.z), "v"(pa.w), "v"(pz))
        else if (g == 7)
            VS_QUAD8("", a, b, "v"(pb.x), "v"(pb.y), "v"(pb.z), "v"(pb.w))
        else
            VS_QUAD8("", a, b)
        a = na;
        b = nb;
    }
    kz = pz;
    x[0] += x0;
    x[1] += x1;
    x[2] += x2;
    x[3] += x3;
}

__device__ __forceinline__ void compress_quad(uint32_t (&x)[4], const uint4 *kw, const QuadLane &ql) {
    uint32_t x0 = x[0], x1 = x[1], x2 = x[2], x3 = x[3];
    uint4 v = kw[0];
    uint32_t z = dpp_u32<0xA8>(x3) + v.x;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const uint4 u = q < 15 ? kw[(q + 1) * 16] : make_uint4(0, 0, 0, 0);
        VS_QUAD_ROUND(x0, x1, x2, x3, z, v.y)
        VS_QUAD_ROUND(x3, x0, x1, x2, z, v.z)
        VS_QUAD_ROUND(x2, x3, x0, x1, z, v.w)
        VS_QUAD_ROUND(x1, x2, x3, x0, z, u.x)
        v = u;
    }
    x[0] += x0;
    x[1] += x1;
    x[2] += x2;
    x[3] += x3;
}
#undef VS_QUAD_ROUND
#undef VS_QA
#undef VS_QUAD8

// End of a chain's turn in a slice: write the digest of a finished chain, or
// append the midstate of an unfinished one to the next active list
// (wave-aggregated: one atomic per wave).
__device__ __forceinline__ void retire(const ShaSliceArgs &a, const ShaChain &ch0,
                                       const uint32_t (&st)[8], bool valid, uint32_t mine,
                                       uint32_t left, uint32_t lane) {
    const bool finished = valid && mine == left;
    const bool survive = valid && !finished;
    if (finished) {
        uint4 *out = (uint4 *)ch0.out;
        out[0] = make_uint4(__builtin_bswap32(st[0]), __builtin_bswap32(st[1]),
                            __builtin_bswap32(st[2]), __builtin_bswap32(st[3]));
        out[1] = make_uint4(__builtin_bswap32(st[4]), __builtin_bswap32(st[5]),
                            __builtin_bswap32(st[6]), __builtin_bswap32(st[7]));
    }
    const uint64_t bal = __ballot(survive);
    if (bal) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(a.n_next, (uint32_t)__popcll(bal));
        base = __builtin_amdgcn_readfirstlane(base);
        if (survive) {
            const uint32_t pos = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
            ShaChain nc = ch0;
            nc.ptr = ch0.ptr + 64ull * mine;
#pragma unroll
            for (int i = 0; i < 8; ++i) nc.st[i] = st[i];
            a.next[pos] = nc;
        }
    }
}

// One slice over the active chains.  Workgroup = 2 waves:
// wave 0 produces, wave 1 consumes; both hold the same 64 chains (lane l of
// each wave = chain l of the tile) and step through the same block loop, one
// workgroup barrier per block.
// Producer side of a tile (the W of each block into the LDS slots); QUAD: the
// compact latency-mode layout with K added (schedule_to_lds).
template <bool QUAD>
__device__ __forceinline__ void produce_tile(uint4 (&wk)[2][16 * 64], const ShaChain &ch0, uint32_t mine,
                                             uint32_t steps, uint32_t lane) {
    const uint64_t p = ch0.ptr, e = ch0.end, L = ch0.len;
    const uint64_t A = p & ~15ull;
    const uint64_t safe =
        L ? ((e - 1) & ~15ull) : ((uint64_t)(uintptr_t)ch0.out & ~15ull);
    const uint32_t q = (uint32_t)(p & 15) >> 2;
    // the chain this lane loads for in instruction i, and its segment offset
    uint64_t LA[4], LE[4], LS[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int src = 16 * i + (int)(lane >> 2);
        LA[i] = (uint64_t)__shfl((long long)A, src, 64);
        LE[i] = (uint64_t)__shfl((long long)e, src, 64);
        LS[i] = (uint64_t)__shfl((long long)safe, src, 64);
    }
    const uint64_t so = 16 + 16 * (lane & 3);
    // staged segments: chain c, segment t at uint4 index 5 c + t (80-byte
    // stride: conflict-free ds_write_b128 / ds_read_b128)
    const uint32_t wr = 5 * (lane >> 2) + (lane & 3);
    uint4 R[4], c = load_seg(A, e, safe), S[4];
    uint32_t d[17], w[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) R[i] = load_seg(LA[i] + so, LE[i], LS[i]);
    // block 0 -> slot 0
#pragma unroll
    for (int i = 0; i < 4; ++i) wk[0][80 * i + wr] = R[i];
#pragma unroll
    for (int t = 0; t < 4; ++t) S[t] = wk[0][5 * lane + t];
#pragma unroll
    for (int i = 0; i < 4; ++i) R[i] = load_seg(LA[i] + 64 + so, LE[i], LS[i]);
    window_words(d, c, S, q);
    c = S[3];
    if (mine > 0) {
        message(w, d, p, e, L);
        schedule_to_lds<QUAD ? kSlotQuad : kSlotSplit>(w, wk[0], lane);
    }
    __syncthreads();
    for (uint32_t j = 0; j < steps; ++j) {
        // produce block j+1 while the consumer runs block j; its segments
        // arrived during step j-1, block j+2's are fetched now
        uint4 *slot = wk[(j + 1) & 1];
        const uint64_t nb = 64ull * (j + 2) + so;
#pragma unroll
        for (int i = 0; i < 4; ++i) slot[80 * i + wr] = R[i];
#pragma unroll
        for (int i = 0; i < 4; ++i) R[i] = load_seg(LA[i] + nb, LE[i], LS[i]);
#pragma unroll
        for (int t = 0; t < 4; ++t) S[t] = slot[5 * lane + t];
        window_words(d, c, S, q);
        c = S[3];
        if (j + 1 < mine) {
            message(w, d, p + 64ull * (j + 1), e, L);
            schedule_to_lds<QUAD ? kSlotQuad : kSlotSplit>(w, slot, lane);
        }
        __syncthreads();
    }
}

// Isolated latency tiles run in their own kernel,
// sha_iso_kernel: a workgroup holds a CU alone (the launch asks for the CU's
// whole 160 KiB of LDS) and kIsoChains chains.  Wave 0 produces, each other
// wave consumes 16 chains in compress_quad_iso, on a SIMD of its own.  The
// producer uses all 64 lanes: lane 4c + k builds block 4m + k of chain c (and
// 16 + c), so one pass over the message schedule per chain yields a batch of
// four blocks (16 lanes of work per block, as in a shared-CU tile, took as
// long as the consumer's block).  The W ring: 16 slots of kIsoChains chains,
// block j in slot j % 16 at a 64 B-padded stride (the four blocks of a pass land in
// different banks).  One barrier per batch: the consumers run batch m while
// the producer builds batch m + 2 into the slots of batch m - 2, so batch
// m + 1 is complete and a consumer reads each next block's first K + W during
// the current one; a batch's segments are loaded one batch ahead.
// consumer waves per isolated tile: two (a SIMD each) put the tail on half
// as many CUs and leave the rest to the bulk -- C2 alone 200.4-201.5 ->
// 198.5-199.0 ms, a C3 rank 226.5-233.8 -> 223.1-227.9 against the round's
// one-consumer form (profiles/r06_iso32)
#ifndef VS_SHA_ISO_CONSUMERS
#define VS_SHA_ISO_CONSUMERS 2
#endif
constexpr uint32_t kIsoWaves = 1 + VS_SHA_ISO_CONSUMERS;   // producer + consumers
constexpr uint32_t kIsoChains = 16 * VS_SHA_ISO_CONSUMERS;  // chains per isolated tile
// the producer builds batch m + kIsoLead while the consumers run batch m; with
// a lead of 2 batch m + 1 is complete, so a consumer reads each next block's
// first K + W during the current one (three consumers' ring fits only a lead
// of 1: the first block of a batch then waits for its words after the barrier)
constexpr uint32_t kIsoLead = VS_SHA_ISO_CONSUMERS > 2 ? 1 : 2;
constexpr uint32_t kRingSlots = 8 * kIsoLead;
constexpr uint32_t kIsoRingStride = kIsoChains * 16 + 4;  // uint4 per ring slot
constexpr uint32_t kIsoLdsBytes = 160 * 1024;             // the CU's whole LDS
static_assert((kRingSlots * kIsoRingStride + 2 * 16 * kIsoChains + 1) * sizeof(uint4) <= kIsoLdsBytes,
              "W ring exceeds the CU's LDS");

struct IsoSrc {  // one chain's byte source in produce_iso
    uint64_t p, e, L, A, safe;
    uint32_t q, mine;
    uint4 S0, S[4];
    __device__ __forceinline__ void init(const ShaChain &ch, uint32_t m) {
        p = ch.ptr;
        e = ch.end;
        L = ch.len;
        A = p & ~15ull;
        safe = L ? ((e - 1) & ~15ull) : ((uint64_t)(uintptr_t)ch.out & ~15ull);
        q = (uint32_t)(p & 15) >> 2;
        mine = m;
    }
    __device__ __forceinline__ void load(uint32_t blk) {
        const uint64_t b = A + 64ull * blk;
        S0 = load_seg(b, e, safe);
#pragma unroll
        for (int s = 0; s < 4; ++s) S[s] = load_seg(b + 16 * (s + 1), e, safe);
    }
};

__device__ __forceinline__ void produce_iso(uint4 *ring, const ShaChain (&ch)[VS_SHA_ISO_CONSUMERS],
                                            const uint32_t (&mine)[VS_SHA_ISO_CONSUMERS], uint32_t steps,
                                            uint32_t lane) {
    constexpr int NC = VS_SHA_ISO_CONSUMERS;
    const uint32_t k = lane & 3, c = lane >> 2;
    IsoSrc x[NC];
#pragma unroll
    for (int i = 0; i < NC; ++i) x[i].init(ch[i], mine[i]);
    uint32_t d[17], w[16];
    auto build = [&](const IsoSrc &xs, uint32_t m, uint32_t cc) {
        const uint32_t blk = 4 * m + k;
        if (blk < xs.mine) {
            window_words(d, xs.S0, xs.S, xs.q);
            message(w, d, xs.p + 64ull * blk, xs.e, xs.L);
            schedule_to_lds<kSlotQuadEarly, kIsoChains>(w, ring + (blk % kRingSlots) * kIsoRingStride, cc);
        }
    };
    // build i happens before barrier i - (kIsoLead - 1): batches 0 .. lead-1
    // precede the consumers' first block, then batch m + lead while they run
    // batch m; 1 + ceil(steps / 4) barriers, as the consumers
    const uint32_t nb = (steps + 3) / 4;
#pragma unroll
    for (int i = 0; i < NC; ++i) x[i].load(k);
    for (uint32_t i = 0; i < nb + kIsoLead; ++i) {
        if (i < nb) {
#pragma unroll
            for (int j = 0; j < NC; ++j) build(x[j], i, 16 * j + c);
#pragma unroll
            for (int j = 0; j < NC; ++j) x[j].load(4 * (i + 1) + k);
        }
        if (i + 1 >= kIsoLead) __syncthreads();
    }
}

// VS_SHA_TRACE builds (A/B diagnostics only): every tile of sha_slice_kernel
// records {kind | tile, HW_ID, XCC_ID, start, end} (s_memrealtime, 100 MHz)
// from its consumer wave, read back with vs_debug_sha_trace
#ifndef VS_SHA_TRACE
#define VS_SHA_TRACE 0
#endif
#if VS_SHA_TRACE
constexpr uint32_t kTraceCap = 1u << 16;
__device__ uint64_t g_sha_trace[kTraceCap * 4];
__device__ uint32_t g_sha_trace_n;
// word 0: quad << 63 | shader-clock cycles of the tile (s_memtime) << 20 | tile
__device__ __forceinline__ void trace_tile(bool quad, uint32_t t, uint64_t t0, uint64_t c0, uint32_t lane) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    const uint64_t cyc = (uint64_t)__builtin_amdgcn_s_memtime() - c0;
    if (lane == 0) {
        const uint32_t k = atomicAdd(&g_sha_trace_n, 1u);
        if (k < kTraceCap) {
            g_sha_trace[4 * k + 0] = ((uint64_t)quad << 63) | ((cyc < (1ull << 43) ? cyc : (1ull << 43) - 1) << 20) | (t & 0xfffffu);
            g_sha_trace[4 * k + 1] = ((uint64_t)xcc << 32) | hw;
            g_sha_trace[4 * k + 2] = t0;
            g_sha_trace[4 * k + 3] = t1;
        }
    }
}
#endif

#ifndef VS_SHA_QUAD_PPRIO
// latency tiles' producers at the consumers' priority: measured slower in a
// mixed drain (C3 rank single pass 334-371 against 321-327 ms,
// profiles/r06_first/ab_single_c3r3.log), so off
#define VS_SHA_QUAD_PPRIO 0
#endif
// Tiles [0, qt) hold chains [a.quad_lo, a.quad_chains) of the order (the
// longest; an isolated drain's sha_iso_kernel takes the first a.quad_lo), 16
// per tile, consumed in latency mode (compress_quad; the producer's lanes
// 16..63 idle); the later tiles hold 64 chains each in split mode.
// VS_SHA_MINW (A/B builds): at least this many waves per SIMD, i.e. a
// register budget that fits beside a co-resident fingerprint workgroup
#ifdef VS_SHA_MINW
__global__ __launch_bounds__(128, VS_SHA_MINW) void sha_slice_kernel(ShaSliceArgs a) {
#else
__global__ __launch_bounds__(128) void sha_slice_kernel(ShaSliceArgs a) {
#endif
    __shared__ uint4 wk[2][16 * 64];  // 2 x 16 KiB: W of one block of 64 chains
    // the tile broadcast borrows W slot 1's first word: between tiles no block
    // is in flight, and the next tile's producer writes slot 1 only after the
    // barrier that follows block 0.  The kernel's LDS is then exactly 32 KiB,
    // so a workgroup fits beside a 128 KiB fingerprint workgroup on one CU.
    uint32_t &tile_sh = wk[1][0].x;
    // the K + W that quad lanes 1-3 read: zeros in a part of buffer 0 that
    // quad tiles never write (their W takes entries 0..255, the staged
    // segments 0..318); a workgroup's tiles come in tile-counter order, so it
    // runs every quad tile it gets before its first split tile
    uint4 *const zero_kw = &wk[0][512];
    const uint32_t lane = threadIdx.x & 63;
    const bool producer = __builtin_amdgcn_readfirstlane(threadIdx.x) < 64;  // wave-uniform
    const uint32_t n = *a.n_cur;
    const uint32_t nq = min(a.quad_chains, n);
    const uint32_t q0 = min(a.quad_lo, nq);
    const uint32_t qt = (nq - q0 + 15) / 16;
    const uint32_t ntiles = qt + (n - nq + 63) / 64;
    if (qt) {
        for (uint32_t i = threadIdx.x; i < 16 * 16; i += blockDim.x) zero_kw[i] = make_uint4(0, 0, 0, 0);
        __syncthreads();
    }
    if (!producer) __builtin_amdgcn_s_setprio(2);  // the rounds are the critical path
    for (;;) {
        if (threadIdx.x == 0) tile_sh = atomicAdd(a.tile_ctr, 1u);
        __syncthreads();
        const uint32_t t = tile_sh;
        __syncthreads();
        if (t >= ntiles) break;
        const bool quad = t < qt;  // wave-uniform
        const uint32_t my = quad ? (producer ? lane : lane >> 2) : lane;
        const uint32_t idx = quad ? q0 + t * 16 + my : nq + (t - qt) * 64 + my;
        const bool valid = quad ? (my < 16 && idx < nq) : idx < n;
        const uint32_t ci = valid ? (a.order ? a.order[idx] : idx) : 0u;
        const ShaChain ch0 = a.cur[ci];
        const uint32_t left = valid ? blocks_left(ch0.ptr, ch0.end) : 0u;
        const uint32_t mine = min(left, a.budget);
        // steps = max over the tile's lanes (identical in both waves)
        uint32_t steps = mine;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) steps = max(steps, (uint32_t)__shfl_xor((int)steps, o, 64));
        steps = __builtin_amdgcn_readfirstlane(steps);
        if (steps == 0) continue;
#if VS_SHA_TRACE
        const uint64_t t_tile = __builtin_amdgcn_s_memrealtime();
        const uint64_t c_tile = __builtin_amdgcn_s_memtime();
#endif
        if (producer) {
            if (quad) {
                // a latency tile's producer feeds the drain's critical path:
                // beside busy split tiles it would otherwise need ~6000
                // cycles per block against the quad consumer's ~3800
                if (VS_SHA_QUAD_PPRIO) __builtin_amdgcn_s_setprio(3);
                produce_tile<true>(wk, ch0, mine, steps, lane);
                if (VS_SHA_QUAD_PPRIO) __builtin_amdgcn_s_setprio(0);
            } else {
                produce_tile<false>(wk, ch0, mine, steps, lane);
            }
        } else if (quad) {
            __builtin_amdgcn_s_setprio(3);  // the drain's critical path
            const uint32_t role = lane & 3, c = lane >> 2;
            QuadLane ql;
            ql.s1 = role == 0 ? 6 : role == 1 ? 2 : 0;
            ql.s2 = role == 0 ? 11 : role == 1 ? 13 : 0;
            ql.s3 = role == 0 ? 25 : role == 1 ? 22 : 0;
            ql.m = role == 1 ? 0xffffffffu : 0u;
            ql.l1 = role == 1;
            // lane 0: e f g h, lane 1: a b c d, lanes 2-3: zeros
            uint32_t x[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = role == 0 ? ch0.st[4 + i] : role == 1 ? ch0.st[i] : 0u;
            __syncthreads();
            for (uint32_t j = 0; j < steps; ++j) {
                if (j < mine) compress_quad(x, role == 0 ? &wk[j & 1][c] : &zero_kw[c], ql);
                __syncthreads();
            }
            uint32_t st[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                st[i] = (uint32_t)__shfl((int)x[i], (int)(lane | 1), 64);
                st[4 + i] = x[i];
            }
            retire(a, ch0, st, valid && role == 0, mine, left, lane);
#if VS_SHA_TRACE
            trace_tile(true, t, t_tile, c_tile, lane);
#endif
            __builtin_amdgcn_s_setprio(2);
        } else {
            uint32_t st[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) st[i] = ch0.st[i];
            __syncthreads();
            for (uint32_t j = 0; j < steps; ++j) {
                if (j < mine) compress_lds(st, wk[j & 1], lane);
                __syncthreads();
            }
            retire(a, ch0, st, valid, mine, left, lane);
#if VS_SHA_TRACE
            trace_tile(false, t, t_tile, c_tile, lane);
#endif
        }
    }
}

// An isolated drain's latency tiles (see produce_iso): a.quad_chains chains
// of the order, kIsoChains per workgroup of kIsoWaves waves, each launched
// with the CU's whole LDS so it holds the CU alone; a.resident counts the
// workgroups that have started (the host launches the split tiles only then).
__global__ __launch_bounds__(64 * kIsoWaves) void sha_iso_kernel(ShaSliceArgs a) {
    extern __shared__ uint4 iso_lds[];
    uint4 *const ring = iso_lds;
    uint4 *const zero_kw = ring + kRingSlots * kIsoRingStride;  // lanes 2-3's K + W
    uint4 *const one_kw = zero_kw + 16 * kIsoChains;             // lane 1's (-d = ~d + 1)
    uint32_t *const tile_w = (uint32_t *)(one_kw + 16 * kIsoChains);   // [0] tile, [1] steps
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t n = *a.n_cur;
    const uint32_t nq = min(a.quad_chains, n);
    const uint32_t ntiles = (nq + kIsoChains - 1) / kIsoChains;
    if (threadIdx.x == 0) __hip_atomic_fetch_add(a.resident, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    for (uint32_t i = threadIdx.x; i < 16 * kIsoChains; i += blockDim.x) {
        zero_kw[i] = make_uint4(0, 0, 0, 0);
        one_kw[i] = make_uint4(1, 1, 1, 1);
    }
    if (wave) __builtin_amdgcn_s_setprio(3);  // the drain's critical path
    // chain cc of tile t (uniform per lane group of four)
    auto chain = [&](uint32_t t, uint32_t cc, ShaChain &ch, uint32_t &left, bool &valid) {
        const uint32_t idx = t * kIsoChains + cc;
        valid = idx < nq;
        ch = a.cur[valid ? (a.order ? a.order[idx] : idx) : 0u];
        left = valid ? blocks_left(ch.ptr, ch.end) : 0u;
    };
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) tile_w[0] = atomicAdd(a.tile_ctr, 1u);
        __syncthreads();
        const uint32_t t = tile_w[0];
        if (t >= ntiles) break;
        constexpr int NC = VS_SHA_ISO_CONSUMERS;
        ShaChain pc[NC];      // the producer's chains (lane: c, 16 + c, ...)
        uint32_t pm[NC];
        ShaChain c0;
        uint32_t l0;
        bool v0;
        const uint32_t c = lane >> 2;
        if (wave == 0) {
            uint32_t m = 0;
#pragma unroll
            for (int i = 0; i < NC; ++i) {
                chain(t, 16 * i + c, pc[i], l0, v0);
                pm[i] = min(l0, a.budget);
                m = max(m, pm[i]);
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
            if (threadIdx.x == 0) tile_w[1] = m;
        } else {
            chain(t, 16 * (wave - 1) + c, c0, l0, v0);
        }
        __syncthreads();
        const uint32_t steps = __builtin_amdgcn_readfirstlane(tile_w[1]);
        if (steps == 0) continue;
#if VS_SHA_TRACE
        const uint64_t t_tile = __builtin_amdgcn_s_memrealtime();
        const uint64_t c_tile = __builtin_amdgcn_s_memtime();
#endif
        if (wave == 0) {
            produce_iso(ring, pc, pm, steps, lane);
            continue;
        }
        const uint32_t mine = min(l0, a.budget);
        const uint32_t role = lane & 3, cc = 16 * (wave - 1) + c;
        QuadLane ql;
        ql.s1 = role == 0 ? 6 : role == 1 ? 2 : 0;
        ql.s2 = role == 0 ? 11 : role == 1 ? 13 : 0;
        ql.s3 = role == 0 ? 25 : role == 1 ? 22 : 0;
        ql.m = role == 1 ? 0xffffffffu : 0u;
        ql.l1 = role == 1;
        // lane 0: e f g h, lane 1: a b c d, lanes 2-3: zeros
        uint32_t x[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = role == 0 ? c0.st[4 + i] : role == 1 ? c0.st[i] : 0u;
        __syncthreads();
        // a batch of four blocks per barrier, straight-line: every lane runs
        // all four and keeps the blocks it owns; each block's first K + W words
        // are read during the block before.  Per-lane base and slot stride (0
        // for lanes 1-3): no branch
        const uint4 *kbase = role == 0 ? &ring[cc] : role == 1 ? &one_kw[cc] : &zero_kw[cc];
        const uint32_t kstride = role == 0 ? kIsoRingStride : 0u;
        auto kwp = [&](uint32_t j) { return kbase + (j % kRingSlots) * kstride; };
        uint32_t kz = kwp(0)[15 * kIsoChains].w;
        uint4 qa = kwp(0)[0], qb = kwp(0)[kIsoChains];
        for (uint32_t j0 = 0; j0 < steps; j0 += 4) {
#pragma unroll
            for (uint32_t kk = 0; kk < 4; ++kk) {
                const uint32_t j = j0 + kk;
                uint32_t y[4] = {x[0], x[1], x[2], x[3]};
                // (lead 1: the next batch is being written, so the last block
                // re-reads its own words and the next batch's come after the barrier)
                compress_quad_iso<kIsoChains>(y, kwp(j), kwp(kIsoLead > 1 || kk < 3 ? j + 1 : j), ql, kz, qa, qb);
                const bool on = j < mine;
#pragma unroll
                for (int i = 0; i < 4; ++i) x[i] = on ? y[i] : x[i];
            }
            __syncthreads();
            if (kIsoLead == 1) {
                kz = kwp(j0 + 4)[15 * kIsoChains].w;
                qa = kwp(j0 + 4)[0];
                qb = kwp(j0 + 4)[kIsoChains];
            }
        }
        uint32_t st[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            st[i] = (uint32_t)__shfl((int)x[i], (int)(lane | 1), 64);
            st[4 + i] = x[i];
        }
        retire(a, c0, st, v0 && role == 0, mine, l0, lane);
#if VS_SHA_TRACE
        trace_tile(true, 2 * t + wave - 1, t_tile, c_tile, lane);
#endif
    }
}

// Throughput mode: with enough active chains to give every
// SIMD several waves, a chain's latency no longer matters and the split's
// LDS round trip and barrier only cost throughput.  Each wave then owns a tile
// of 64 chains and does everything itself: the same cooperative segment loads
// as the producer (staged through a wave-private LDS area), message expansion
// in a rolling 16-word register window, and the 64 rounds.
__device__ __forceinline__ void compress_regs(uint32_t (&st)[8], uint32_t (&w)[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
#define VS_SHA_ROUND(a, b, c, d, e, f, g, h, wk)                                   \
    {                                                                              \
        const uint32_t t1_ = h + xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)) +       \
                             ch(e, f, g) + (wk);                                   \
        const uint32_t t2_ = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)) + maj(a, b, c); \
        d += t1_;                                                                  \
        h = t1_ + t2_;                                                             \
    }
#define VS_W(t)                                                                              \
    ((t) < 16 ? w[(t)&15]                                                                    \
              : (w[(t)&15] = w[(t)&15] +                                                     \
                             xor3(rotr(w[((t)-15) & 15], 7), rotr(w[((t)-15) & 15], 18),    \
                                  w[((t)-15) & 15] >> 3) +                                   \
                             w[((t)-7) & 15] +                                               \
                             xor3(rotr(w[((t)-2) & 15], 17), rotr(w[((t)-2) & 15], 19),     \
                                  w[((t)-2) & 15] >> 10)))
#pragma unroll
    for (int t = 0; t < 64; t += 8) {
        VS_SHA_ROUND(a, b, c, d, e, f, g, h, VS_W(t + 0) + kK256[t + 0])
        VS_SHA_ROUND(h, a, b, c, d, e, f, g, VS_W(t + 1) + kK256[t + 1])
        VS_SHA_ROUND(g, h, a, b, c, d, e, f, VS_W(t + 2) + kK256[t + 2])
        VS_SHA_ROUND(f, g, h, a, b, c, d, e, VS_W(t + 3) + kK256[t + 3])
        VS_SHA_ROUND(e, f, g, h, a, b, c, d, VS_W(t + 4) + kK256[t + 4])
        VS_SHA_ROUND(d, e, f, g, h, a, b, c, VS_W(t + 5) + kK256[t + 5])
        VS_SHA_ROUND(c, d, e, f, g, h, a, b, VS_W(t + 6) + kK256[t + 6])
        VS_SHA_ROUND(b, c, d, e, f, g, h, a, VS_W(t + 7) + kK256[t + 7])
    }
#undef VS_W
#undef VS_SHA_ROUND
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
    st[4] += e;
    st[5] += f;
    st[6] += g;
    st[7] += h;
}

// Cross-lane exchange through a wave-private LDS area: the LDS unit executes
// one wave's ds_write / ds_read in issue order, so only compiler reordering
// must be prevented.  (A wave-scope fence would also wait for the in-flight
// prefetch loads -- vmcnt(0) -- and serialise every block on HBM latency.)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

constexpr int kWideWaves = 4;  // waves per workgroup, each independent
__global__ __launch_bounds__(64 * kWideWaves, 3) void sha_slice_wide_kernel(ShaSliceArgs a) {
    __shared__ uint4 stage_all[kWideWaves][5 * 64];  // 5 KiB per wave
    const uint32_t lane = threadIdx.x & 63;
    uint4 *stage = stage_all[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];
    const uint32_t n = *a.n_cur;
    const uint32_t ntiles = (n + 63) / 64;
    for (;;) {
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(a.tile_ctr, 1u);
        t = __builtin_amdgcn_readfirstlane(t);
        if (t >= ntiles) break;
        const uint32_t idx = t * 64 + lane;
        const bool valid = idx < n;
        const uint32_t ci = valid ? (a.order ? a.order[idx] : idx) : 0u;
        const ShaChain ch0 = a.cur[ci];
        const uint32_t left = valid ? blocks_left(ch0.ptr, ch0.end) : 0u;
        const uint32_t mine = min(left, a.budget);
        uint32_t steps = mine;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) steps = max(steps, (uint32_t)__shfl_xor((int)steps, o, 64));
        steps = __builtin_amdgcn_readfirstlane(steps);
        if (steps == 0) continue;
        const uint64_t p = ch0.ptr, e = ch0.end, L = ch0.len;
        const uint64_t A = p & ~15ull;
        const uint64_t safe = L ? ((e - 1) & ~15ull) : ((uint64_t)(uintptr_t)ch0.out & ~15ull);
        const uint32_t q = (uint32_t)(p & 15) >> 2;
        uint64_t LA[4], LE[4], LS[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int src = 16 * i + (int)(lane >> 2);
            LA[i] = (uint64_t)__shfl((long long)A, src, 64);
            LE[i] = (uint64_t)__shfl((long long)e, src, 64);
            LS[i] = (uint64_t)__shfl((long long)safe, src, 64);
        }
        const uint64_t so = 16 + 16 * (lane & 3);
        const uint32_t wr = 5 * (lane >> 2) + (lane & 3);
        uint32_t st[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) st[i] = ch0.st[i];
        uint4 R[4], c = load_seg(A, e, safe), S[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) R[i] = load_seg(LA[i] + so, LE[i], LS[i]);
        for (uint32_t j = 0; j < steps; ++j) {
            // block j's segments arrived during block j-1; fetch block j+1's now
#pragma unroll
            for (int i = 0; i < 4; ++i) stage[80 * i + wr] = R[i];
            const uint64_t nb = 64ull * (j + 1) + so;
#pragma unroll
            for (int i = 0; i < 4; ++i) R[i] = load_seg(LA[i] + nb, LE[i], LS[i]);
            wave_lds_sync();
#pragma unroll
            for (int k = 0; k < 4; ++k) S[k] = stage[5 * lane + k];
            wave_lds_sync();
            uint32_t d[17], w[16];
            window_words(d, c, S, q);
            c = S[3];
            if (j < mine) {
                message(w, d, p + 64ull * j, e, L);
                compress_regs(st, w);
            }
        }
        retire(a, ch0, st, valid, mine, left, lane);
    }
}

// ---- engine bookkeeping kernels ------------------------------------------------
__global__ void sha_append_chunks_kernel(ShaChain *list, const uint32_t *n_cur, const uint8_t *data,
                                         const uint64_t *starts, const uint64_t *ends, uint64_t n,
                                         uint8_t *ids) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t s = starts[i];
    const uint64_t e = (ends[i] & kPosMask) + 1;
    ShaChain c;
    c.ptr = (uint64_t)(uintptr_t)(data + s);
    c.end = (uint64_t)(uintptr_t)(data + e);
    c.len = e - s;
    c.out = ids + 32 * i;
#pragma unroll
    for (int k = 0; k < 8; ++k) c.st[k] = kIV[k];
    list[*n_cur + i] = c;
}

__global__ void sha_append_blobs_kernel(ShaChain *list, const uint32_t *n_cur, const uint8_t *data,
                                        const uint64_t *off, const uint32_t *lens, uint64_t n,
                                        uint8_t *ids) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    ShaChain c;
    c.ptr = (uint64_t)(uintptr_t)(data + off[i]);
    c.end = c.ptr + lens[i];
    c.len = lens[i];
    c.out = ids + 32 * i;
#pragma unroll
    for (int k = 0; k < 8; ++k) c.st[k] = kIV[k];
    list[*n_cur + i] = c;
}

__global__ void sha_count_add_kernel(uint32_t *n_cur, uint32_t add) { *n_cur += add; }

// longest-first order of the active list: bucket = 4095 - f(blocks this slice),
// f monotone, exact below 1024 blocks, 1/64 relative precision above
constexpr uint32_t kShaBuckets = 4096;
__device__ __forceinline__ uint32_t sha_key(const ShaChain &c, uint32_t budget) {
    const uint32_t b = min(blocks_left(c.ptr, c.end), budget);
    uint32_t f;
    if (b < 1024) {
        f = b;
    } else {
        const uint32_t l = 31 - __clz(b);  // >= 10
        f = 1024 + ((l - 10) << 6) + ((b >> (l - 6)) & 63);
    }
    return kShaBuckets - 1 - min(f, kShaBuckets - 1);
}

// Budgeted slices put most chains in one bucket (remaining >= budget), so both
// kernels aggregate their atomics: the histogram in LDS per workgroup, the
// scatter per run of equal keys within a wave (one atomic per distinct key).
__global__ __launch_bounds__(256) void sha_hist_kernel(const ShaChain *list, const uint32_t *n_cur,
                                                       uint32_t budget, uint32_t *hist) {
    __shared__ uint32_t h[kShaBuckets];
    for (uint32_t i = threadIdx.x; i < kShaBuckets; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint32_t n = *n_cur;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        atomicAdd(&h[sha_key(list[i], budget)], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kShaBuckets; i += blockDim.x)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

__global__ __launch_bounds__(256) void sha_scatter_kernel(const ShaChain *list,
                                                          const uint32_t *n_cur, uint32_t budget,
                                                          uint32_t *cursor, uint32_t *order) {
    const uint32_t n = *n_cur;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t stride = gridDim.x * blockDim.x;
    // whole waves iterate together (ballots below)
    for (uint32_t base = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < n; base += stride) {
        const uint32_t i = base + lane;
        const bool valid = i < n;
        const uint32_t key = valid ? sha_key(list[i], budget) : 0xffffffffu;
        uint64_t todo = __ballot(valid);
        while (todo) {
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)todo) - 1;
            const uint32_t k = (uint32_t)__shfl((int)key, (int)leader, 64);
            const uint64_t grp = __ballot(valid && key == k);
            uint32_t pos = 0;
            if (lane == leader) pos = atomicAdd(&cursor[k], (uint32_t)__popcll(grp));
            pos = (uint32_t)__shfl((int)pos, (int)leader, 64);
            if (valid && key == k) order[pos + (uint32_t)__popcll(grp & ((1ull << lane) - 1))] = i;
            todo &= ~grp;
        }
    }
}

// ---- ShaEngine (host) ------------------------------------------------------------
// the fewest remaining blocks a chain in bucket key k can have (sha_key inverse)
static uint64_t bucket_blocks(uint32_t k) {
    const uint32_t f = kShaBuckets - 1 - k;
    if (f < 1024) return f;
    const uint32_t l = 10 + ((f - 1024) >> 6), m = (f - 1024) & 63;
    return (64ull + m) << (l - 6);
}

int ShaEngine::init(int dev) {
    device = dev;
    if (!hist_h) VS_HIP(hipHostMalloc((void **)&hist_h, kShaBuckets * 4, hipHostMallocDefault));
    VS_TRY(ctl.ensure(64));
    VS_TRY(hist.ensure((2 * kShaBuckets + 16) * 4));
    VS_HIP(hipMemset(ctl.p, 0, 64));
    VS_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (!live_h) VS_HIP(hipHostMalloc((void **)&live_h, 4, hipHostMallocDefault));
    // the isolated drain's stream and counter now, not inside the first
    // latency-bound drain (creating them took ~30 ms there: profiles/r06_val1)
    if (isolate) (void)iso_setup();
    return 0;
}

void ShaEngine::release() {
    if (iso_q) {
        (void)hipStreamSynchronize(iso_q);
        (void)hipStreamDestroy(iso_q);
        iso_q = nullptr;
    }
    for (auto &e : iso_ev)
        if (e) (void)hipEventDestroy(e), e = nullptr;
    if (iso_res_h) (void)hipHostFree(iso_res_h);
    iso_res_h = iso_res_d = nullptr;
    for (DevBuf *b : {&list[0], &list[1], &order, &hist, &ctl}) b->release();
    groups.clear();
    ub = 0;
    cap = 0;
    if (live_h) (void)hipHostFree(live_h);
    live_h = nullptr;
    if (hist_h) (void)hipHostFree(hist_h);
    hist_h = nullptr;
}

uint32_t *ShaEngine::count(int which) { return ctl.as<uint32_t>() + which; }

// capacity for n_new more chains on top of every chain that may still be active
int ShaEngine::reserve(uint64_t n_new, hipStream_t s) {
    const uint64_t need = ub + n_new;
    if (need > 0xffffffffull) return fail(VS_ERR_ARG, "too many active SHA-256 chains");
    if (need <= cap) return 0;
    uint64_t ncap = std::max<uint64_t>(need + need / 2, 4096);
    // growing: wait for queued slices, carry the current list over
    VS_HIP(hipStreamSynchronize(s));
    DevBuf nl[2], no;
    VS_TRY(nl[0].ensure(ncap * sizeof(ShaChain)));
    VS_TRY(nl[1].ensure(ncap * sizeof(ShaChain)));
    VS_TRY(no.ensure(ncap * 4));
    if (cap) VS_HIP(hipMemcpy(nl[cur].p, list[cur].p, cap * sizeof(ShaChain), hipMemcpyDeviceToDevice));
    list[0].release();
    list[1].release();
    order.release();
    list[0] = nl[0];
    list[1] = nl[1];
    order = no;
    cap = ncap;
    return 0;
}

int ShaEngine::append_chunks(const uint8_t *data, const uint64_t *starts, const uint64_t *ends,
                             uint64_t n, uint8_t *ids, uint32_t max_blocks, hipStream_t s) {
    if (!n) return 0;
    VS_TRY(reserve(n, s));
    sha_append_chunks_kernel<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(
        list[cur].as<ShaChain>(), count(cur), data, starts, ends, n, ids);
    sha_count_add_kernel<<<1, 1, 0, s>>>(count(cur), (uint32_t)n);
    VS_HIP(hipGetLastError());
    ub += n;
    groups.push_back({n, max_blocks});
    return 0;
}

int ShaEngine::append_blobs(const uint8_t *data, const uint64_t *off, const uint32_t *lens,
                            uint64_t n, uint8_t *ids, hipStream_t s) {
    if (!n) return 0;
    VS_TRY(reserve(n, s));
    sha_append_blobs_kernel<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(
        list[cur].as<ShaChain>(), count(cur), data, off, lens, n, ids);
    sha_count_add_kernel<<<1, 1, 0, s>>>(count(cur), (uint32_t)n);
    VS_HIP(hipGetLastError());
    ub += n;
    groups.push_back({n, 0xffffffffu});
    return 0;
}

// advance every active chain by up to `budget` blocks (0xffffffff: to the end).
// A drain reads the exact count back between throughput-mode
// slices and finishes the last wide_min chains in split (latency) mode, so the
// longest chains' tail runs at the split's per-chain speed.
int ShaEngine::slice(uint32_t budget, hipStream_t s) {
    if (ub == 0) return 0;
    // budgeted slices run beside the next volume's fingerprint pass: split
    // mode leaves that pass room (throughput mode measured slower there)
    if (budget != 0xffffffffu) return launch(budget, kShaSplit, s);
    while (ub >= wide_min) {
        VS_HIP(hipMemcpyAsync(live_h, count(cur), 4, hipMemcpyDeviceToHost, s));
        VS_HIP(hipStreamSynchronize(s));
        const uint32_t live = *live_h;
        if (live == 0) {
            groups.clear();
            ub = 0;
            return 0;
        }
        if (live < wide_min) break;
        VS_TRY(launch(std::max(wide_budget, 1u), kShaWide, s));
    }
    // the final drain: every remaining chain to its end; its longest chains
    // set the finish time, so they run in latency (quad) mode
    return launch(budget, quad_pct ? kShaQuad : kShaSplit, s);
}

int ShaEngine::launch(uint32_t budget, int mode, hipStream_t s) {
    if (ub == 0) return 0;  // every chain finished within the previous budgets
    const int nxt = cur ^ 1;
    uint32_t *cursor = hist.as<uint32_t>() + kShaBuckets;
    uint32_t *partials = cursor + kShaBuckets + 1;
    VS_HIP(hipMemsetAsync(hist.p, 0, kShaBuckets * 4, s));
    const uint32_t sb = (uint32_t)std::min<uint64_t>((ub + 255) / 256, 4096);
    const uint32_t hb = std::min<uint32_t>(sb, (uint32_t)std::max(cus, 1) * 2);
    sha_hist_kernel<<<hb, 256, 0, s>>>(list[cur].as<ShaChain>(), count(cur), budget,
                                       hist.as<uint32_t>());
    VS_HIP(launch_scan_u32(hist.as<uint32_t>(), cursor, kShaBuckets, partials, 0xffffffffu, s));
    sha_scatter_kernel<<<sb, 256, 0, s>>>(list[cur].as<ShaChain>(), count(cur), budget, cursor,
                                          order.as<uint32_t>());
    // quad drain (bucket histogram read back: one synchronisation per drain)
    uint32_t quad_chains = 0, iso_chains = 0;   // latency-mode chains; of those, isolated
    bool shared_tail = false;                    // iso_chains < quad_chains
    if (mode == kShaQuad) {
        VS_HIP(hipMemcpyAsync(hist_h, hist.p, kShaBuckets * 4, hipMemcpyDeviceToHost, s));
        VS_HIP(hipStreamSynchronize(s));
        uint32_t first = 0;
        while (first < kShaBuckets && hist_h[first] == 0) ++first;
        double blocks = 0;
        for (uint32_t k = first; k < kShaBuckets; ++k) blocks += (double)hist_h[k] * bucket_blocks(k);
        // Per-block costs of a chain: split mode beside a busy
        // chip ~2.8 us (the producer crowded on its SIMD); quad mode ~1.6 us
        // beside split tiles, ~1.34 us on a CU of its own (isolated drain:
        // sha_iso_kernel, profiles/r06_quad; 1.45 us with the shared-CU form,
        // profiles/r06_drain); the backlog clears at split-mode throughput,
        // ~1.45 TB/s = 22.7 G blocks/s over the whole chip.
        // (split chains beside a busy chip after a long run, the clock down:
        // up to 3.3 us, profiles/r06_val1/trace_c2; the rule takes 3.0)
        constexpr double kSplitBlockS = 3.0e-6, kBulkBlocksPerS = 22.7e9;
#ifndef VS_SHA_SHARED_TAIL
#define VS_SHA_SHARED_TAIL 1   // isolated drain: chains past the cap in shared-CU latency tiles
#endif
#ifndef VS_SHA_QUAD_CAP2
#define VS_SHA_QUAD_CAP2 16   // isolated: latency-mode chains per two CUs
#endif
        const double quad_s = isolate ? 1.34e-6 : 1.6e-6;
        // isolated, at most 16 chains per two CUs run in latency mode (with
        // two consumer waves per tile, 3 638 chains for a C3 rank on half the
        // CUs took its single pass 225 -> 237-256 ms, profiles/r06_iso32)
        const uint32_t quad_cap = isolate ? (uint32_t)std::max(cus, 2) / 2 * VS_SHA_QUAD_CAP2 : 0xffffffffu;
        const double lmax = first < kShaBuckets ? (double)bucket_blocks(first) : 0.0;
        const double t_bulk = blocks / kBulkBlocksPerS;
        auto count_above = [&](double floor_s) {   // chains whose split-mode time passes floor_s
            uint32_t c = 0;
            for (uint32_t k = first; k < kShaBuckets; ++k) {
                if ((double)bucket_blocks(k) * kSplitBlockS <= floor_s) break;
                c += hist_h[k];
            }
            return c;
        };
        // latency-bound only: the longest chain in split mode would outlast the
        // backlog; otherwise the quad tiles' idle producer lanes only cost
        // throughput
        if (first < kShaBuckets && lmax * kSplitBlockS > t_bulk) {
            if (quad_pct == kQuadAuto) {
                // the drain cannot end before max(longest chain in quad mode,
                // backlog); every chain that would pass that floor in split
                // mode runs in quad mode, started first.  Isolated, each quad
                // tile holds a CU, so the backlog clears on the others: raise
                // the floor until it does
                double floor_s = std::max(lmax * quad_s, t_bulk);
                for (int it = 0; it < 6; ++it) {
                    quad_chains = std::min(count_above(floor_s), quad_cap);
                    if (!isolate) break;
                    const double qtiles = (quad_chains + kIsoChains - 1) / kIsoChains;
                    const double free_cus = std::max((double)cus - qtiles, 1.0);
                    const double tb = t_bulk * cus / free_cus;
                    if (tb <= floor_s) break;
                    floor_s = tb;
                }
                // isolated: the chains above the floor past the cap run in
                // shared-CU latency tiles of the split launch (1.6 us per block
                // beside split tiles, not ~3 in a split tile; a C3 rank's split
                // tail otherwise outlasted its isolated tail, profiles/r06_iso32)
                // Only when the drain is tail-bound (the floor is the longest
                // chain, not the backlog): a fence drain's large backlog lost
                // 3 % to the shared tiles' idle producer lanes
                // (profiles/r06_iso32/ab_shared_distinct2_always.log)
                if (isolate && VS_SHA_SHARED_TAIL && floor_s <= lmax * quad_s) {
                    iso_chains = quad_chains;
                    quad_chains = std::max(quad_chains, count_above(floor_s));
                    shared_tail = true;
                }
            } else {
                for (uint32_t k = first; k < kShaBuckets; ++k) {
                    if ((double)bucket_blocks(k) * 100 < lmax * quad_pct) break;
                    quad_chains += hist_h[k];
                }
            }
        }
        last_quad_chains = quad_chains;
    }
    // zero the next list's count and the tile counter
    VS_HIP(hipMemsetAsync(count(nxt), 0, 4, s));
    VS_HIP(hipMemsetAsync(count(2), 0, 4, s));
    ShaSliceArgs a{};
    a.cur = list[cur].as<ShaChain>();
    a.next = list[nxt].as<ShaChain>();
    a.order = order.as<uint32_t>();
    a.n_cur = count(cur);
    a.n_next = count(nxt);
    a.tile_ctr = count(2);
    a.budget = budget;
    a.quad_chains = quad_chains;
    const uint64_t tiles = (ub + 63) / 64 + (quad_chains + 15) / 16;
    hipEvent_t ka = ev_get ? ev_get() : nullptr, kb = ka ? ev_get() : nullptr;
    if (kb) VS_HIP(hipEventRecord(ka, s));
    if (!shared_tail) iso_chains = quad_chains;
    const uint64_t qi = (iso_chains + kIsoChains - 1) / kIsoChains;   // isolated latency tiles
    last_iso_chains = 0;
    if (mode == kShaQuad && qi && isolate && qi <= (uint64_t)cus / 2 && iso_setup() == 0) {
        last_iso_chains = iso_chains;
        // Isolated drain: each latency tile (sha_iso_kernel, kIsoChains) takes
        // a CU to itself -- it asks for the CU's whole 160 KiB of LDS, so no
        // split workgroup can join it -- and is resident before the split
        // tiles are launched beside it; the split grid covers every CU and
        // takes the latency tiles' CUs as they finish.  (CU-masked streams were
        // tried first: the masks did not hold from one stream pair to the
        // next on this runtime, split tiles ran on "reserved" CUs,
        // profiles/r06_drain/trace_*.log.)
        VS_HIP(hipMemsetAsync(count(3), 0, 4, s));
        VS_HIP(hipEventRecord(iso_ev[0], s));
        VS_HIP(hipStreamWaitEvent(iso_q, iso_ev[0], 0));
        ShaSliceArgs aq = a, ab = a;
        aq.quad_chains = iso_chains;
        aq.resident = iso_res_d;
        ab.quad_lo = iso_chains;   // the split launch: its own latency tiles take the rest
        ab.tile_ctr = count(3);
        __atomic_store_n(iso_res_h, 0u, __ATOMIC_RELAXED);
        sha_iso_kernel<<<(uint32_t)qi, 64 * kIsoWaves, kIsoLdsBytes, iso_q>>>(aq);
        VS_HIP(hipGetLastError());
        VS_HIP(hipEventRecord(iso_ev[1], iso_q));
        // the quad tiles first: the host sees every one of them resident
        // (each bumps a host-visible counter as it starts) before the split
        // grid can take their CUs.  Bounded: after 10 s the split tiles go
        // anyway (results do not depend on the placement).
        const auto t0 = std::chrono::steady_clock::now();
        while (__atomic_load_n(iso_res_h, __ATOMIC_ACQUIRE) < (uint32_t)qi &&
               std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10))
            std::this_thread::yield();
        const uint64_t qt = (iso_chains + 15) / 16;   // tiles' worth of chains the iso launch took
        if (tiles > qt) {
            sha_slice_kernel<<<(uint32_t)std::min<uint64_t>(tiles - qt, (uint64_t)std::max(cus, 1) *
                                                                           (grid_per_cu ? grid_per_cu : 5)),
                               128, 0, s>>>(ab);
            VS_HIP(hipGetLastError());
        }
        VS_HIP(hipStreamWaitEvent(s, iso_ev[1], 0));
    } else if (mode == kShaWide) {
        // persistent grid: 3 waves per SIMD (launch bounds: <= 168 VGPRs)
        const uint64_t slots =
            std::max<uint64_t>((uint64_t)std::max(cus, 1) * 4 * (grid_per_cu ? grid_per_cu : 3) / kWideWaves, 1);
        const uint32_t grid = (uint32_t)std::min<uint64_t>((tiles + kWideWaves - 1) / kWideWaves, slots);
        sha_slice_wide_kernel<<<grid, 64 * kWideWaves, 0, s>>>(a);
    } else {
        // persistent grid: LDS (32 KiB per workgroup) admits 5 workgroups per CU
        const uint32_t grid = (uint32_t)std::min<uint64_t>(
            tiles, (uint64_t)std::max(cus, 1) * (grid_per_cu ? grid_per_cu : 5));
        sha_slice_kernel<<<grid, 128, 0, s>>>(a);
    }
    if (kb) {
        VS_HIP(hipEventRecord(kb, s));
        kernel_pairs.push_back({ka, kb});
    }
    VS_HIP(hipGetLastError());
    cur = nxt;
    // chains of a group finish within ceil(max_blocks / budget) slices
    uint64_t nub = 0;
    std::vector<Group> keep;
    for (Group g : groups) {
        if (budget == 0xffffffffu || g.max_blocks <= budget) continue;
        g.max_blocks -= budget;
        nub += g.n;
        keep.push_back(g);
    }
    groups.swap(keep);
    ub = nub;
    return 0;
}

// the isolated drain's second stream, its events and the host-visible
// residency counter.  0 = ready.
int ShaEngine::iso_setup() {
    if (iso_q) return 0;
    // an isolated latency tile asks for the CU's whole 160 KiB of LDS
    if (hipFuncSetAttribute((const void *)sha_iso_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            kIsoLdsBytes) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    for (auto &e : iso_ev)
        if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            e = nullptr;
            return -1;
        }
    if (!iso_res_h) {
        if (hipHostMalloc((void **)&iso_res_h, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
            hipHostGetDevicePointer((void **)&iso_res_d, iso_res_h, 0) != hipSuccess) {
            (void)hipGetLastError();
            if (iso_res_h) (void)hipHostFree(iso_res_h);
            iso_res_h = iso_res_d = nullptr;
            return -1;
        }
    }
    if (hipStreamCreateWithFlags(&iso_q, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        iso_q = nullptr;
        return -1;
    }
    return 0;
}

#if VS_SHA_TRACE
extern "C" __attribute__((visibility("default"))) int vs_debug_sha_trace(uint64_t *out, uint32_t cap,
                                                                        uint32_t *n, int reset) {
    uint32_t k = 0;
    if (hipMemcpyFromSymbol(&k, HIP_SYMBOL(g_sha_trace_n), 4) != hipSuccess) return -1;
    k = std::min(k, kTraceCap);
    if (n) *n = k;
    if (out && cap && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sha_trace), (size_t)std::min(k, cap) * 32) != hipSuccess)
        return -1;
    const uint32_t z = 0;
    if (reset && hipMemcpyToSymbol(HIP_SYMBOL(g_sha_trace_n), &z, 4) != hipSuccess) return -1;
    return 0;
}
#endif

// ---- synthetic volume bytes -------------------------------------
__device__ __forceinline__ uint64_t splitmix_word(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void synth_kernel(uint64_t seed, uint64_t off, uint64_t n, uint8_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint32_t a = (uint32_t)(off & 7);
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; 8 * t < n; t += stride) {
        const uint64_t w0 = (off >> 3) + t;
        uint64_t v = splitmix_word(seed, w0);
        if (a) v = (v >> (8 * a)) | (splitmix_word(seed, w0 + 1) << (64 - 8 * a));
        const uint64_t o = 8 * t;
        if (o + 8 <= n && (((uintptr_t)(out + o)) & 7) == 0) {
            *(uint64_t *)(out + o) = v;
        } else {
            for (uint32_t k = 0; k < 8 && o + k < n; ++k) out[o + k] = (uint8_t)(v >> (8 * k));
        }
    }
}

hipError_t launch_synth(uint64_t seed, uint64_t off, uint64_t n, uint8_t *out, hipStream_t s) {
    if (!n) return hipSuccess;
    const uint64_t words = (n + 7) / 8;
    uint64_t blocks = (words + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    synth_kernel<<<(uint32_t)blocks, 256, 0, s>>>(seed, off, n, out);
    return hipGetLastError();
}

}  // namespace vsgpu
