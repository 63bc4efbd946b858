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
#include "internal.hpp"

namespace vsgpu {

constexpr uint32_t kTabEntries = 256 * kFpCopies;  // u64 entries per table
constexpr uint32_t kOut8Byte = kTabEntries * 8;    // byte offset of OUT8 in LDS (0x10000)
static_assert(kOut8Byte == 0x10000, "roll() builds OUT8 addresses with v_perm");

typedef uint32_t G16[16];  // one 64-byte group as 16 little-endian words

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
        uint4 v = load16<GUARD>(data, off + 16 * q, dlen);
        g[4 * q + 0] = v.x;
        g[4 * q + 1] = v.y;
        g[4 * q + 2] = v.z;
        g[4 * q + 3] = v.w;
    }
}

__device__ __forceinline__ uint64_t lds_u64(const char *lds, uint32_t byte_addr) {
    return *(const uint64_t *)(lds + byte_addr);
}

// One byte of the rolling window.  oldw/neww hold the evicted / incoming byte
// in byte lane J.  Returns the new low digest word (for the cut test).
template <int J>
__device__ __forceinline__ uint32_t roll(uint32_t &hi, uint32_t &lo, uint32_t oldw,
                                         uint32_t neww, uint32_t lane8, uint32_t sh,
                                         const char *lds) {
    const uint32_t lane8o = lane8 | kOut8Byte;
    // lane8o = lane*8 | 0x10000 (OUT8 base): one v_perm builds
    // [lane*8, b_old, 0x01, 0x00] = 0x10000 + b_old*256 + lane*8
    const uint32_t oaddr = __builtin_amdgcn_perm(lane8o, oldw, 0x0c060004u | (J << 8));
    const uint32_t idx = __builtin_amdgcn_ubfe(hi, sh, 8);
    const uint32_t maddr = (idx << 8) | lane8;
    const uint64_t ov = lds_u64(lds, oaddr);
    const uint64_t mv = lds_u64(lds, maddr);
    const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 24);            // hi<<8 | lo>>24
    const uint32_t nlo = __builtin_amdgcn_perm(lo, neww, 0x06050400u | J);  // lo<<8 | b_new
    hi = __builtin_amdgcn_bitop3_b32(nhi, (uint32_t)(mv >> 32), (uint32_t)(ov >> 32), 0x96);
    lo = __builtin_amdgcn_bitop3_b32(nlo, (uint32_t)mv, (uint32_t)ov, 0x96);
    return lo;
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
#define VS_ROLL2(J0, J1)                                                                 \
    {                                                                                    \
        uint32_t a_[CH], b_[CH];                                                         \
        _Pragma("unroll") for (int c = 0; c < CH; ++c) a_[c] =                           \
            (roll<J0>(hi[c], lo[c], old[c][w], nw[c][w], lane8, sh, lds),                \
             cut_bits<WIDE>(hi[c], lo[c], mlo, mhi));                                    \
        _Pragma("unroll") for (int c = 0; c < CH; ++c) b_[c] =                           \
            (roll<J1>(hi[c], lo[c], old[c][w], nw[c][w], lane8, sh, lds),                \
             cut_bits<WIDE>(hi[c], lo[c], mlo, mhi));                                    \
        _Pragma("unroll") for (int c = 0; c < CH; ++c) m[c] =                            \
            __builtin_elementwise_min(__builtin_elementwise_min(m[c], a_[c]), b_[c]);    \
    }
        VS_ROLL2(0, 1)
        VS_ROLL2(2, 3)
#undef VS_ROLL2
    }
}

// ---- rare path: a group holds at least one candidate -------------------------
template <bool GUARD>
__device__ __forceinline__ uint8_t byte_at(const uint8_t *data, int64_t p, uint64_t dlen) {
    if (GUARD && (p < 0 || (uint64_t)p >= dlen)) return 0;
    return data[p];
}

struct StripRec {
    uint64_t k;      // strip index
    uint32_t cnt;    // candidates so far
    uint32_t slot;   // dense pool slot
    bool valid;      // chain maps to a real strip
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

template <bool GUARD, bool WIDE>
__device__ void rare_group(const FpArgs &a, StripRec &r, int64_t gpos, uint32_t hi,
                           uint32_t lo, uint32_t sh, uint32_t lane8, const char *lds,
                           uint64_t strip_base) {
    // gpos: data offset of the group's first byte; (hi,lo): digest before it
    uint64_t bits = 0;
    for (int j = 0; j < 64; ++j) {
        const int64_t p = gpos + j;
        const uint32_t bo = byte_at<GUARD>(a.data, p - 64, a.dlen);
        const uint32_t bn = byte_at<GUARD>(a.data, p, a.dlen);
        const uint32_t idx = __builtin_amdgcn_ubfe(hi, sh, 8);
        const uint64_t mv = lds_u64(lds, (idx << 8) | lane8);
        const uint64_t ov = lds_u64(lds, kOut8Byte + (bo << 8) + lane8);
        const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 24);
        const uint32_t nlo = (lo << 8) | bn;
        hi = nhi ^ (uint32_t)(mv >> 32) ^ (uint32_t)(ov >> 32);
        lo = nlo ^ (uint32_t)mv ^ (uint32_t)ov;
        if (cut_bits<WIDE>(hi, lo, a.mask_lo, a.mask_hi) == 0 && (uint64_t)p < a.scan_end &&
            r.valid) {
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
        const uint32_t words = a.strip / 32;
        uint32_t *bw = a.pool + (uint64_t)r.slot * words;
        const uint32_t w0 = (uint32_t)(((uint64_t)gpos - strip_base) >> 5);
        bw[w0] |= (uint32_t)bits;
        bw[w0 + 1] |= (uint32_t)(bits >> 32);
    }
}

template <int CH, bool GUARD, bool WIDE>
__global__ __launch_bounds__(kFpThreads) void fp_kernel(FpArgs a) {
    __shared__ __attribute__((aligned(16))) uint64_t tabs[2 * kTabEntries];  // 128 KiB
    for (uint32_t i = threadIdx.x; i < kTabEntries; i += blockDim.x) {
        const uint32_t e = i / kFpCopies;
        tabs[i] = a.mod_tab[e];
        tabs[kTabEntries + i] = a.out8_tab[e];
    }
    __syncthreads();
    const char *lds = (const char *)tabs;
    const uint32_t lane8 = (threadIdx.x & 31) * 8;
    const uint32_t sh = a.idx_shift;
    const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t G = a.strip / 64;  // checked groups per strip (multiple of 3)

    StripRec rec[CH];
    int64_t sb[CH];  // strip base (data offset)
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        uint64_t k = tid + (uint64_t)c * T;
        rec[c].valid = k < a.k_count;
        if (!rec[c].valid) k = a.k_count - 1;
        rec[c].k = a.k_first + k;
        rec[c].cnt = 0;
        rec[c].slot = kNoSlot;
        sb[c] = (int64_t)(a.base + rec[c].k * a.strip);
    }

    uint32_t hi[CH], lo[CH], m[CH];
    G16 X[CH], Y[CH], Z[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        load_group<GUARD>(X[c], a.data, sb[c] - 64, a.dlen);  // warm-up bytes
        load_group<GUARD>(Y[c], a.data, sb[c], a.dlen);       // group 1
    }
    // warm-up: the window starts as 64 virtual zero bytes, digest 0
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        hi[c] = 0;
        lo[c] = 0;
    }
#pragma unroll
    for (int w = 0; w < 16; ++w) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            roll_warm<0>(hi[c], lo[c], X[c][w], lane8, sh, lds);
            roll_warm<1>(hi[c], lo[c], X[c][w], lane8, sh, lds);
            roll_warm<2>(hi[c], lo[c], X[c][w], lane8, sh, lds);
            roll_warm<3>(hi[c], lo[c], X[c][w], lane8, sh, lds);
        }
    }

#define VS_GROUP(OLD, NEW, NEXT, GI)                                                      \
    {                                                                                     \
        if ((GI) + 1 <= G) {                                                              \
            _Pragma("unroll") for (int c = 0; c < CH; ++c)                                \
                load_group<GUARD>(NEXT[c], a.data, sb[c] + 64 * (int64_t)(GI), a.dlen);   \
        }                                                                                 \
        uint32_t h0[CH], l0[CH];                                                          \
        _Pragma("unroll") for (int c = 0; c < CH; ++c) {                                  \
            h0[c] = hi[c];                                                                \
            l0[c] = lo[c];                                                                \
        }                                                                                 \
        process_group<CH, WIDE>(hi, lo, OLD, NEW, m, lane8, sh, lds, a.mask_lo, a.mask_hi); \
        _Pragma("unroll") for (int c = 0; c < CH; ++c) {                                  \
            if (m[c] == 0)                                                                \
                rare_group<GUARD, WIDE>(a, rec[c], sb[c] + 64 * (int64_t)((GI) - 1), h0[c], \
                                        l0[c], sh, lane8, lds, (uint64_t)sb[c]);          \
        }                                                                                 \
    }

    for (uint32_t g = 1; g <= G; g += 3) {
        VS_GROUP(X, Y, Z, g)
        VS_GROUP(Y, Z, X, g + 1)
        VS_GROUP(Z, X, Y, g + 2)
    }
#undef VS_GROUP

#pragma unroll
    for (int c = 0; c < CH; ++c) {
        if (rec[c].valid) {
            a.counts[rec[c].k] = rec[c].cnt;
            a.dense_slot[rec[c].k] = rec[c].slot;
        }
    }
}

#ifndef VS_FP_CHAINS
#define VS_FP_CHAINS 1
#endif

hipError_t launch_fingerprint(const FpArgs &a, bool guard, bool wide, hipStream_t s) {
    if (a.k_count == 0) return hipSuccess;
    constexpr int CH = VS_FP_CHAINS;
    const uint64_t threads = (a.k_count + CH - 1) / CH;
    const uint32_t blocks = (uint32_t)((threads + kFpThreads - 1) / kFpThreads);
    if (guard) {
        if (wide)
            fp_kernel<CH, true, true><<<blocks, kFpThreads, 0, s>>>(a);
        else
            fp_kernel<CH, true, false><<<blocks, kFpThreads, 0, s>>>(a);
    } else {
        if (wide)
            fp_kernel<CH, false, true><<<blocks, kFpThreads, 0, s>>>(a);
        else
            fp_kernel<CH, false, false><<<blocks, kFpThreads, 0, s>>>(a);
    }
    return hipGetLastError();
}

}  // namespace vsgpu
