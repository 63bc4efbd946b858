// fingerprint.hip -- candidate-cut pass of restic's chunker on gfx950.
//
// Restates the per-byte loop of github.com/restic/chunker@v0.4.0
// chunker.go Next() as a position-independent pass:
// after 64 slides the reference digest equals the canonical fingerprint of
// the 64-byte window, FP(p) = (sum_i B[p-63+i] x^(8(63-i))) mod P, so every
// lane can start anywhere with a 64-byte warm-up and evaluate the cut test
// (FP(p) & splitmask) == 0 at every offset of its strip.
//
// Per byte:
//   D' = (D << 8 | b) ^ MOD[D >> (deg-8)] ^ OUT8[b_old]
// MOD/OUT8 are 256 x u64 tables held in LDS as 32 lane-private copies
// (entry e of copy l at byte e*256 + l*8): the 32 lanes of a ds_read_b64
// lane group always hit 32 distinct bank pairs, whatever the indices.
// 8.5 VALU + 2 ds_read_b64 per byte; the OUT8 lookup is off the digest's
// dependency chain.
//
// The digest chain costs one LDS round trip per byte, so each lane carries
// two strips ("chains") interleaved byte by byte.  The grid is persistent
// (one 12-wave workgroup per CU, tables loaded once); waves take 128 strips
// at a time from a work counter, and the few strips whose reads need bounds
// checks (the first one when it has no 64-byte warm-up before it, the last
// ones) are done by wave 0 of workgroup 0 beside the others.  Each lane
// reads whole 64-byte groups (four back-to-back dwordx4 loads, one cache-line
// pair), three per chain: the group 64 bytes back (the evicted bytes), the
// current group and the next.  The hot loop only notes which groups hold a
// candidate; their exact offsets are found after the strip by re-rolling each
// noted group from a 64-byte warm-up (the window property again).
#include <cstdlib>

#include "internal.hpp"

namespace vsgpu {

constexpr uint32_t kTabEntries = 256 * kFpCopies;  // u64 entries per table
constexpr uint32_t kOut8Byte = kTabEntries * 8;    // byte offset of OUT8 in LDS (0x10000)
static_assert(kOut8Byte == 0x10000, "roll() builds OUT8 addresses with v_perm");
#ifndef VS_FP_CHAINS
#define VS_FP_CHAINS 2
#endif
constexpr int kChains = VS_FP_CHAINS;             // strips per lane
constexpr uint32_t kUnit = 64 * kChains;          // strips per work unit

#ifndef VS_FP_GROUP
#define VS_FP_GROUP 16
#endif
constexpr int kGW = VS_FP_GROUP;      // words per group buffer (16: 64 B, 32: 128 B = one line)
constexpr int kGB = 4 * kGW;          // bytes per group
typedef uint32_t G16[16];  // one 64-byte group as 16 little-endian words (warm-up, process_group)
typedef uint32_t GBuf[kGW];

template <bool GUARD>
__device__ __forceinline__ uint4 load16(const uint8_t *data, int64_t off, uint64_t dlen) {
    if (!GUARD) return *(const uint4 *)(data + off);
    if (off >= 0 && (uint64_t)off + 16 <= dlen) return *(const uint4 *)(data + off);
    uint32_t w[4] = {0, 0, 0, 0};
    for (int i = 0; i < 16; ++i) {
        int64_t p = off + i;
        if (p >= 0 && (uint64_t)p < dlen) w[i >> 2] |= (uint32_t)data[p] << (8 * (i & 3));
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

template <bool GUARD>
__device__ __forceinline__ void load_group(G16 &g, const uint8_t *data, int64_t off,
                                           uint64_t dlen) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint4 v = load16<GUARD>(data, off + 16 * q, dlen);
        g[4 * q + 0] = v.x;
        g[4 * q + 1] = v.y;
        g[4 * q + 2] = v.z;
        g[4 * q + 3] = v.w;
    }
}

__device__ __forceinline__ uint64_t lds_u64(const char *lds, uint32_t byte_addr) {
    return *(const uint64_t *)(lds + byte_addr);
}

// Issue costs on gfx950 (profiles/r05_valu, tools/valu/valu_ops3.hip): v_perm,
// v_alignbit, v_and_or and v_bfe take ~4.2 cycles per wave-instruction, while
// v_bitop3 whose three sources are VGPRs, v_lshrrev with an inline shift and
// the two-operand logic ops take ~2.3.  kFF00 is 0xff00 held in a VGPR (an
// SGPR or literal operand would make the v_bitop3 a 4.2-cycle one).
#ifndef VS_FP_BITOP3
#define VS_FP_BITOP3 1
#endif

// One byte of the rolling window.  oldw/neww hold the evicted / incoming byte
// in byte lane J.  FAST: deg >= 48 (sh >= 8); SH8 >= 0: sh - 8 known at
// compile time (restic's polynomials have degree 53: SH8 = 5).
template <int J, bool FAST = false, int SH8 = -1>
__device__ __forceinline__ void roll(uint32_t &hi, uint32_t &lo, uint32_t oldw, uint32_t neww,
                                     uint32_t lane8, uint32_t sh, const char *lds,
                                     uint32_t kFF00 = 0xff00u) {
    const uint32_t lane8o = lane8 | kOut8Byte;
    // lane8o = lane*8 | 0x10000 (OUT8 base): one v_perm builds
    // [lane*8, b_old, 0x01, 0x00] = 0x10000 + b_old*256 + lane*8; byte 1
    // needs no move: (oldw & 0xff00) | lane8o, one all-VGPR v_bitop3
    const uint32_t oaddr = (VS_FP_BITOP3 && SH8 >= 0 && J == 1)
                               ? __builtin_amdgcn_bitop3_b32(oldw, kFF00, lane8o, 0xEA)
                               : __builtin_amdgcn_perm(lane8o, oldw, 0x0c060004u | (J << 8));
    // MOD address idx*256 + lane*8.  FAST: a two-operand shift and one v_and_or
    // instead of v_bfe + v_lshl_or; with SH8 the shift is an inline constant
    // and the and-or an all-VGPR v_bitop3 ((a & b) | c = 0xEA)
    const uint32_t maddr =
        (VS_FP_BITOP3 && SH8 >= 0) ? __builtin_amdgcn_bitop3_b32(hi >> SH8, kFF00, lane8, 0xEA)
        : FAST                     ? (((hi >> (sh - 8)) & 0xff00u) | lane8)
                                   : ((__builtin_amdgcn_ubfe(hi, sh, 8) << 8) | lane8);
    const uint64_t ov = lds_u64(lds, oaddr);
    const uint64_t mv = lds_u64(lds, maddr);
    const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 24);            // hi<<8 | lo>>24
    const uint32_t nlo = __builtin_amdgcn_perm(lo, neww, 0x06050400u | J);  // lo<<8 | b_new
    hi = __builtin_amdgcn_bitop3_b32(nhi, (uint32_t)(mv >> 32), (uint32_t)(ov >> 32), 0x96);
    lo = __builtin_amdgcn_bitop3_b32(nlo, (uint32_t)mv, (uint32_t)ov, 0x96);
}

// warm-up roll: the window still holds virtual zeros, OUT8[0] == 0
template <int J>
__device__ __forceinline__ void roll_warm(uint32_t &hi, uint32_t &lo, uint32_t neww,
                                          uint32_t lane8, uint32_t sh, const char *lds) {
    const uint32_t idx = __builtin_amdgcn_ubfe(hi, sh, 8);
    const uint64_t mv = lds_u64(lds, (idx << 8) | lane8);
    const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 24);
    const uint32_t nlo = __builtin_amdgcn_perm(lo, neww, 0x06050400u | J);
    hi = nhi ^ (uint32_t)(mv >> 32);
    lo = nlo ^ (uint32_t)mv;
}

// kernel variants: mask within the low digest word / wider than 32 bits /
// FAST = low word and deg >= 48: cheaper MOD address / FAST53 = FAST with
// deg == 53 (every restic repository polynomial): the shift an inline constant
constexpr int kFpNarrow = 0, kFpWide = 1, kFpFast = 2, kFpFast53 = 3;

template <bool WIDE>
__device__ __forceinline__ uint32_t cut_bits(uint32_t hi, uint32_t lo, uint32_t mlo,
                                             uint32_t mhi) {
    if (WIDE) return (lo & mlo) | (hi & mhi);
    return lo & mlo;
}

// 64 bytes for CH chains, interleaved byte by byte for ILP.  m[c] collects the
// minimum masked digest: 0 <=> a candidate in this group.
template <int CH, bool WIDE>
__device__ __forceinline__ void process_group(uint32_t (&hi)[CH], uint32_t (&lo)[CH],
                                              const G16 (&old)[CH], const G16 (&nw)[CH],
                                              uint32_t (&m)[CH], uint32_t lane8, uint32_t sh,
                                              const char *lds, uint32_t mlo, uint32_t mhi) {
#pragma unroll
    for (int c = 0; c < CH; ++c) m[c] = 0xffffffffu;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                switch (j) {
                    case 0: roll<0>(hi[c], lo[c], old[c][w], nw[c][w], lane8, sh, lds); break;
                    case 1: roll<1>(hi[c], lo[c], old[c][w], nw[c][w], lane8, sh, lds); break;
                    case 2: roll<2>(hi[c], lo[c], old[c][w], nw[c][w], lane8, sh, lds); break;
                    default: roll<3>(hi[c], lo[c], old[c][w], nw[c][w], lane8, sh, lds); break;
                }
                m[c] = __builtin_elementwise_min(m[c], cut_bits<WIDE>(hi[c], lo[c], mlo, mhi));
            }
        }
    }
}

// process_group with the next group streamed into `old` as it is consumed:
// once quarter q of the evicted bytes has been rolled past, its four words are
// refilled with quarter q of the group after `nw` (at byte offset nxt[c]).
// Two 64-byte buffers per strip then hold the evicted bytes, the incoming
// bytes and the prefetch.
template <int CH, bool GUARD, int MODE>
__device__ __forceinline__ void process_group_pf(uint32_t (&hi)[CH], uint32_t (&lo)[CH],
                                                 GBuf (&old)[CH], const GBuf (&nw)[CH],
                                                 uint32_t (&m)[CH], uint32_t lane8, uint32_t sh,
                                                 const char *lds, const FpArgs &a,
                                                 const int64_t (&nxt)[CH], uint32_t kFF00,
                                                 uint32_t mlo) {
#pragma unroll
    for (int c = 0; c < CH; ++c) m[c] = 0xffffffffu;
#pragma unroll
    for (int q = 0; q < kGW / 4; ++q) {
#pragma unroll
        for (int w = 4 * q; w < 4 * q + 4; ++w) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
#pragma unroll
                for (int c = 0; c < CH; ++c) {
                    constexpr bool F = MODE == kFpFast || MODE == kFpFast53;
                    constexpr int S8 = MODE == kFpFast53 ? 5 : -1;
                    switch (j) {
                        case 0: roll<0, F, S8>(hi[c], lo[c], old[c][w], nw[c][w], lane8, sh, lds, kFF00); break;
                        case 1: roll<1, F, S8>(hi[c], lo[c], old[c][w], nw[c][w], lane8, sh, lds, kFF00); break;
                        case 2: roll<2, F, S8>(hi[c], lo[c], old[c][w], nw[c][w], lane8, sh, lds, kFF00); break;
                        default: roll<3, F, S8>(hi[c], lo[c], old[c][w], nw[c][w], lane8, sh, lds, kFF00); break;
                    }
                    // (a v_min_u16 prefilter on the low 16 digest bits measured
                    // slower: 27.8 vs 22.8 ms per 64 GiB)
                    m[c] = __builtin_elementwise_min(
                        m[c], cut_bits<MODE == kFpWide>(hi[c], lo[c], mlo, a.mask_hi));
                }
            }
        }
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const uint4 v = load16<GUARD>(a.data, nxt[c] + 16 * q, a.dlen);
            old[c][4 * q + 0] = v.x;
            old[c][4 * q + 1] = v.y;
            old[c][4 * q + 2] = v.z;
            old[c][4 * q + 3] = v.w;
        }
    }
}

template <bool GUARD>
__device__ __forceinline__ void load_buf(GBuf &g, const uint8_t *data, int64_t off,
                                         uint64_t dlen) {
#pragma unroll
    for (int q = 0; q < kGW / 4; ++q) {
        const uint4 v = load16<GUARD>(data, off + 16 * q, dlen);
        g[4 * q + 0] = v.x;
        g[4 * q + 1] = v.y;
        g[4 * q + 2] = v.z;
        g[4 * q + 3] = v.w;
    }
}

// ---- candidate offsets: re-roll the noted groups ---------------------------------
template <bool GUARD>
__device__ __forceinline__ uint32_t byte_at(const uint8_t *data, int64_t p, uint64_t dlen) {
    if (GUARD && (p < 0 || (uint64_t)p >= dlen)) return 0;
    return data[p];
}

struct StripRec {
    uint64_t k;      // strip index
    uint32_t cnt;    // candidates so far
    uint32_t slot;   // dense pool slot
};

__device__ void rec_dense_alloc(const FpArgs &a, StripRec &r) {
    const uint32_t words = a.strip / 32;
    uint32_t slot = atomicAdd(a.pool_next, 1u);
    if (slot >= a.pool_cap) {
        atomicOr(a.flags, kFlagPoolOverflow);
        r.slot = kNoSlot;
        return;
    }
    r.slot = slot;
    uint4 *bm = (uint4 *)(a.pool + (uint64_t)slot * words);
    for (uint32_t i = 0; i < words / 4; ++i) bm[i] = make_uint4(0, 0, 0, 0);
    uint32_t *bw = a.pool + (uint64_t)slot * words;
    for (int i = 0; i < kSlots; ++i) {
        uint32_t o = a.offs[r.k * kSlots + i];
        bw[o >> 5] |= 1u << (o & 31);
    }
}

// Every candidate in [from, to) of strip r (from - strip_base and to - from
// multiples of 64): the digest entering `from` is rebuilt from the 64 bytes
// before it, then the window rolls byte by byte.
template <bool GUARD, bool WIDE>
__device__ void rescan(const FpArgs &a, StripRec &r, int64_t from, int64_t to, uint32_t lane8,
                       const char *lds, uint64_t strip_base) {
    const uint32_t sh = a.idx_shift;
    uint32_t hi = 0, lo = 0;
    for (int64_t p = from - 64; p < from; ++p) {
        const uint32_t idx = __builtin_amdgcn_ubfe(hi, sh, 8);
        const uint64_t mv = lds_u64(lds, (idx << 8) | lane8);
        hi = __builtin_amdgcn_alignbit(hi, lo, 24) ^ (uint32_t)(mv >> 32);
        lo = ((lo << 8) | byte_at<GUARD>(a.data, p, a.dlen)) ^ (uint32_t)mv;
    }
    for (int64_t g = from; g < to; g += 64) {
        uint64_t bits = 0;
        for (int j = 0; j < 64; ++j) {
            const int64_t p = g + j;
            const uint32_t bo = byte_at<GUARD>(a.data, p - 64, a.dlen);
            const uint32_t bn = byte_at<GUARD>(a.data, p, a.dlen);
            const uint32_t idx = __builtin_amdgcn_ubfe(hi, sh, 8);
            const uint64_t mv = lds_u64(lds, (idx << 8) | lane8);
            const uint64_t ov = lds_u64(lds, kOut8Byte + (bo << 8) + lane8);
            const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 24);
            const uint32_t nlo = (lo << 8) | bn;
            hi = nhi ^ (uint32_t)(mv >> 32) ^ (uint32_t)(ov >> 32);
            lo = nlo ^ (uint32_t)mv ^ (uint32_t)ov;
            if (cut_bits<WIDE>(hi, lo, a.mask_lo, a.mask_hi) == 0 && (uint64_t)p < a.scan_end) {
                const uint32_t off = (uint32_t)((uint64_t)p - strip_base);
                if (r.cnt < (uint32_t)kSlots) {
                    a.offs[r.k * kSlots + r.cnt] = off;
                } else {
                    if (r.cnt == (uint32_t)kSlots) rec_dense_alloc(a, r);
                    bits |= 1ull << j;
                }
                r.cnt++;
            }
        }
        if (bits && r.slot != kNoSlot) {
            uint32_t *bw = a.pool + (uint64_t)r.slot * (a.strip / 32);
            const uint32_t w0 = (uint32_t)(((uint64_t)g - strip_base) >> 5);
            bw[w0] |= (uint32_t)bits;
            bw[w0 + 1] |= (uint32_t)(bits >> 32);
        }
    }
}

// noted groups of one chain: up to three 8-bit group indices and a count in
// the top byte; kNoteAll = more than three (the whole strip is re-rolled)
constexpr uint32_t kNoteAll = 0xff000000u;
__device__ __forceinline__ uint32_t note_group(uint32_t notes, uint32_t g) {
    const uint32_t n = notes >> 24;
    if (n >= 3) return kNoteAll;
    return (notes | (g << (8 * n))) + (1u << 24);
}

// CH strips per lane, byte-interleaved.  kk[c]: strip indices; valid[c] false
// for a padding chain (it computes but records nothing).
template <int CH, bool GUARD, int MODE>
__device__ __forceinline__ void run_strips(const FpArgs &a, const char *lds, uint32_t lane8,
                                           const uint64_t (&kk)[CH], const bool (&valid)[CH],
                                           uint32_t kFF00, uint32_t mlo) {
    const uint32_t sh = a.idx_shift;
    const uint32_t G = a.strip / kGB;  // groups per strip, even (and < 256)
    int64_t sb[CH];  // strip base (data offset)
    uint32_t hi[CH], lo[CH], m[CH], notes[CH];
    GBuf A[CH], B[CH];  // evicted / incoming bytes; the evicted buffer refills with the next group
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        sb[c] = (int64_t)(a.base + kk[c] * a.strip);
        load_buf<GUARD>(A[c], a.data, sb[c] - kGB, a.dlen);  // warm-up bytes (last 64 used)
        load_buf<GUARD>(B[c], a.data, sb[c], a.dlen);        // group 0
        hi[c] = 0;
        lo[c] = 0;
        notes[c] = 0;
    }
    // warm-up over the 64 bytes before the strip: the window starts as 64
    // virtual zero bytes, digest 0 (with 128-byte groups the first 64 bytes of
    // A are never used)
#pragma unroll
    for (int w = kGW - 16; w < kGW; ++w) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            roll_warm<0>(hi[c], lo[c], A[c][w], lane8, sh, lds);
            roll_warm<1>(hi[c], lo[c], A[c][w], lane8, sh, lds);
            roll_warm<2>(hi[c], lo[c], A[c][w], lane8, sh, lds);
            roll_warm<3>(hi[c], lo[c], A[c][w], lane8, sh, lds);
        }
    }

    // group GI: evicted bytes in OLD (group GI-1, refilled with GI+1 as it is
    // consumed; the last group reloads itself), incoming in NEW
#define VS_GROUP(OLD, NEW, GI)                                                            \
    {                                                                                     \
        int64_t nx_[CH];                                                                  \
        _Pragma("unroll") for (int c = 0; c < CH; ++c)                                    \
            nx_[c] = sb[c] + kGB * (int64_t)min((GI) + 1, G - 1);                          \
        process_group_pf<CH, GUARD, MODE>(hi, lo, OLD, NEW, m, lane8, sh, lds, a, nx_,      \
                                          kFF00, mlo);                                    \
        _Pragma("unroll") for (int c = 0; c < CH; ++c) {                                  \
            if (m[c] == 0) notes[c] = note_group(notes[c], (GI));                         \
        }                                                                                 \
    }

    for (uint32_t g = 0; g < G; g += 2) {
        VS_GROUP(A, B, g)
        VS_GROUP(B, A, g + 1)
    }
#undef VS_GROUP

#pragma unroll
    for (int c = 0; c < CH; ++c) {
        if (!valid[c]) continue;
        StripRec r{kk[c], 0, kNoSlot};
        const uint32_t n = notes[c] >> 24;
        if (notes[c] == kNoteAll) {
            rescan<GUARD, MODE == kFpWide>(a, r, sb[c], sb[c] + a.strip, lane8, lds, (uint64_t)sb[c]);
        } else {
            for (uint32_t i = 0; i < n; ++i) {
                const int64_t g0 = sb[c] + kGB * (int64_t)((notes[c] >> (8 * i)) & 0xff);
                rescan<GUARD, MODE == kFpWide>(a, r, g0, g0 + kGB, lane8, lds, (uint64_t)sb[c]);
            }
        }
        a.counts[r.k] = r.cnt;
        a.dense_slot[r.k] = r.slot;
    }
}

template <int MODE, int THREADS>
__global__ __launch_bounds__(THREADS) void fp_kernel(FpArgs a) {
    __shared__ __attribute__((aligned(16))) uint64_t tabs[2 * kTabEntries];  // 128 KiB
    for (uint32_t i = threadIdx.x; i < kTabEntries; i += blockDim.x) {
        const uint32_t e = i / kFpCopies;
        tabs[i] = a.mod_tab[e];
        tabs[kTabEntries + i] = a.out8_tab[e];
    }
    __syncthreads();
    const char *lds = (const char *)tabs;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lane8 = (threadIdx.x & 31) * 8;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // 0xff00 and the cut mask as VGPR operands (opaque to the compiler, which
    // would otherwise fold them into SGPR / literal operands: see roll())
    uint32_t kFF00 = 0xff00u, mlo = a.mask_lo;
    if (VS_FP_BITOP3 && MODE == kFpFast53) {
        asm volatile("v_mov_b32 %0, 0xff00" : "=v"(kFF00));
        asm volatile("v_mov_b32 %0, %1" : "=v"(mlo) : "s"(a.mask_lo));
    }
    // bounds-checked strips: one per lane on wave 0 of workgroup 0
    if (blockIdx.x == 0 && wave == 0) {
        for (uint64_t e0 = 0; e0 < a.n_edge; e0 += 64) {
            const uint64_t e = e0 + lane;
            const bool v = e < a.n_edge;
            const uint64_t ee = v ? e : 0;
            const uint64_t kk[1] = {ee < a.k_lo ? ee : a.k_hi + (ee - a.k_lo)};
            const bool vv[1] = {v};
            run_strips<1, true, MODE>(a, lds, lane8, kk, vv, kFF00, mlo);
        }
    }
    // interior strips: units of 64 * kChains strips, kChains per lane
    for (;;) {
        uint32_t u = 0;
        if (lane == 0) u = atomicAdd(a.work, 1u);
        u = __builtin_amdgcn_readfirstlane(__shfl(u, 0, 64));
        const uint64_t k0 = a.k_lo + (uint64_t)u * kUnit;
        if (k0 >= a.k_hi) break;
        uint64_t kk[kChains];
        bool vv[kChains];
#pragma unroll
        for (int c = 0; c < kChains; ++c) {
            const uint64_t k = k0 + 64 * c + lane;
            vv[c] = k < a.k_hi;
            kk[c] = vv[c] ? k : k0;
        }
        run_strips<kChains, false, MODE>(a, lds, lane8, kk, vv, kFF00, mlo);
    }
}

// the register budget the kernel is compiled for: its launch size, unless a
// co-residency A/B build (VS_FP_LB 1024, VS_FP_THREADS 768) launches fewer
// waves than it budgets for, leaving a SHA-256 workgroup room on every CU
#ifndef VS_FP_LB
#define VS_FP_LB VS_FP_THREADS
#endif
constexpr int kFpLaunchBound = VS_FP_LB;

hipError_t launch_fingerprint(const FpArgs &a, bool wide, bool fast, int cus, hipStream_t s) {
    const bool deg53 = fast && a.idx_shift == 13;
    const uint64_t units = (a.k_hi - a.k_lo + kUnit - 1) / kUnit;
    if (units == 0 && a.n_edge == 0) return hipSuccess;
    const uint64_t grid =
        std::max<uint64_t>(1, std::min<uint64_t>(units, (uint64_t)std::max(cus, 1)));
    if (wide)
        fp_kernel<kFpWide, kFpLaunchBound><<<(uint32_t)grid, kFpThreads, 0, s>>>(a);
    else if (deg53)
        fp_kernel<kFpFast53, kFpLaunchBound><<<(uint32_t)grid, kFpThreads, 0, s>>>(a);
    else if (fast)
        fp_kernel<kFpFast, kFpLaunchBound><<<(uint32_t)grid, kFpThreads, 0, s>>>(a);
    else
        fp_kernel<kFpNarrow, kFpLaunchBound><<<(uint32_t)grid, kFpThreads, 0, s>>>(a);
    return hipGetLastError();
}

}  // namespace vsgpu
