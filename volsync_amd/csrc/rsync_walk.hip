// rsync_walk.hip -- match.c hash_search as a device-resident greedy walk
//  for the XXH3 strong sums rsync 3.2.3 negotiates by
// default (xxh128; also xxh3), blength > 240.
//
// The host walk (rsync_api.hip) needs every weak-sum candidate of every
// offset first: the exhaustive scan reads each source byte twice, tests all of
// them against a table that no longer fits LDS at C4's block counts, and then
// sorts, copies and walks millions of candidates on one host core.  The walk
// itself visits only a fraction of the offsets: one per block where the
// source matches, every offset only in the literal stretch after an edit.
// Here every wave walks one segment of the source exactly as hash_search
// does, in two modes:
//   RUN   at an offset the walk visits after a match (or at a segment start):
//         the 64 lanes read the whole window once, 16 bytes per lane per
//         1 KiB XXH3 block, and produce its weak sum (get_checksum1) and its
//         XXH3 strong sum together; the chain of blocks with that weak sum is
//         walked in rsync's order (descending index, length check, strong
//         compare, false alarms counted, want_i preference).
//   STEP  after a window that did not match: 1024 offsets per batch, 16 per
//         lane; each lane's window sums come from a wave prefix scan of the
//         rolling deltas, then 16 rolling updates; every offset is tested
//         against the LDS prefilter, the filter and the directory, and the
//         hits are visited in offset order (a RUN-style window hash each).
// Segments are walked speculatively from their own start; a stitch pass
// re-walks a segment from its true entry (the previous segment's exit
// offset and want_i) until it makes a match the speculative walk also made,
// from where the two are identical.  The result is
// bit-identical to hash_search: same matches, same false-alarm count.
#include "internal.hpp"
#include "strong.hpp"

namespace vsgpu {
namespace {

using vsstrong::P32_1;

constexpr uint32_t kWalkThreads = 1024;            // 16 waves; the 128 KiB prefilter admits one WG/CU
constexpr uint32_t kLdsFiltWordsW = 1u << 15;      // 2^20-bit LDS prefilter
constexpr uint64_t kBatch = 1024;                  // STEP offsets per wave batch (16 per lane)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 gl16(const uint8_t *p) {
    typedef __attribute__((address_space(1))) const u32x4 g4;
    const u32x4 v = *(g4 *)(uintptr_t)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

// 16 aligned bytes at d + al, zero past dlen
__device__ __forceinline__ uint4 gl16_guard(const uint8_t *d, uint64_t al, uint64_t dlen) {
    if (al + 16 <= dlen) return gl16(d + al);
    uint32_t v[4] = {0, 0, 0, 0};
    for (uint32_t i = 0; i < 16; ++i)
        if (al + i < dlen) v[i >> 2] |= (uint32_t)d[al + i] << (8 * (i & 3));
    return make_uint4(v[0], v[1], v[2], v[3]);
}

// 16 bytes at d + pos, pos & 15 == sh (wave-uniform), from two aligned loads
// and a funnel shift; bytes at or past dlen read as 0
__device__ __forceinline__ void ld16(const uint8_t *d, uint64_t pos, uint32_t sh, uint64_t dlen,
                                     uint32_t (&w)[4]) {
    const uint64_t al = pos - sh;
    const uint4 c0 = gl16_guard(d, al, dlen);
    if (sh == 0) {
        w[0] = c0.x; w[1] = c0.y; w[2] = c0.z; w[3] = c0.w;
        return;
    }
    const uint4 c1 = gl16_guard(d, al + 16, dlen);
    const uint32_t v0 = c0.x, v1 = c0.y, v2 = c0.z, v3 = c0.w, v4 = c1.x, v5 = c1.y, v6 = c1.z,
                   v7 = c1.w;
    const uint32_t r = sh & 3;
    switch (sh >> 2) {  // uniform
    case 0:
        w[0] = __builtin_amdgcn_alignbyte(v1, v0, r); w[1] = __builtin_amdgcn_alignbyte(v2, v1, r);
        w[2] = __builtin_amdgcn_alignbyte(v3, v2, r); w[3] = __builtin_amdgcn_alignbyte(v4, v3, r);
        break;
    case 1:
        w[0] = __builtin_amdgcn_alignbyte(v2, v1, r); w[1] = __builtin_amdgcn_alignbyte(v3, v2, r);
        w[2] = __builtin_amdgcn_alignbyte(v4, v3, r); w[3] = __builtin_amdgcn_alignbyte(v5, v4, r);
        break;
    case 2:
        w[0] = __builtin_amdgcn_alignbyte(v3, v2, r); w[1] = __builtin_amdgcn_alignbyte(v4, v3, r);
        w[2] = __builtin_amdgcn_alignbyte(v5, v4, r); w[3] = __builtin_amdgcn_alignbyte(v6, v5, r);
        break;
    default:
        w[0] = __builtin_amdgcn_alignbyte(v4, v3, r); w[1] = __builtin_amdgcn_alignbyte(v5, v4, r);
        w[2] = __builtin_amdgcn_alignbyte(v6, v5, r); w[3] = __builtin_amdgcn_alignbyte(v7, v6, r);
        break;
    }
}

__device__ __forceinline__ int dot4(uint32_t word, uint32_t w, int acc) {
    return __builtin_amdgcn_sdot4((int)word, (int)w, acc, false);
}

__device__ __forceinline__ uint64_t shx64(uint64_t v, int m) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}
// sum over the 16 lanes with the same (lane & 3)
__device__ __forceinline__ uint64_t red16(uint64_t v) {
    v += shx64(v, 4);
    v += shx64(v, 8);
    v += shx64(v, 16);
    v += shx64(v, 32);
    return v;
}
__device__ __forceinline__ uint32_t red64(uint32_t v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v += (uint32_t)__shfl_xor((int)v, m, 64);
    return v;
}
// wave-uniform values made explicit (scalar registers, scalar branches): the
// walk's control flow is uniform by construction, and values the compiler
// cannot prove uniform (shuffle results, per-lane loads of one address) would
// otherwise turn its loop exits into divergent ones
__device__ __forceinline__ uint32_t uni(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ int32_t unis(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}
__device__ __forceinline__ uint64_t rdl64(uint64_t v, int lane) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}
// exclusive prefix sum over the wave (lane order)
__device__ __forceinline__ uint32_t excl_scan(uint32_t v, uint32_t lane) {
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    return x - v;
}

// Per-lane XXH3 secret words of the 16-bytes-per-lane layout: lane l holds
// words 2m, 2m+1 of stripe s (l = 4s + m) of every 1 KiB block.
struct LaneSec {
    uint64_t s0, s1;    // stripe secret words s + 2m, s + 2m + 1
    uint64_t sc0, sc1;  // scramble words 16 + 2m, 17 + 2m
    uint64_t l0, l1;    // last stripe: byte offsets 121 + 16m, 129 + 16m
    uint64_t i0, i1;    // initial accumulators 2m, 2m + 1
};
__device__ __forceinline__ LaneSec lane_secrets(uint32_t lane, uint64_t seed) {
    using namespace vsstrong;
    const uint32_t s = lane >> 2, m = lane & 3;
    LaneSec r;
    r.s0 = sec64(s + 2 * m, seed);
    r.s1 = sec64(s + 2 * m + 1, seed);
    r.sc0 = sec64(16 + 2 * m, seed);
    r.sc1 = sec64(17 + 2 * m, seed);
    r.l0 = csec_at(121 + 16 * m, seed);
    r.l1 = csec_at(129 + 16 * m, seed);
    const uint64_t init[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
    r.i0 = init[0];
    r.i1 = init[1];
#pragma unroll
    for (uint32_t j = 1; j < 4; ++j) {
        r.i0 = (m == j) ? init[2 * j] : r.i0;
        r.i1 = (m == j) ? init[2 * j + 1] : r.i1;
    }
    return r;
}

__device__ __forceinline__ uint64_t scramble(uint64_t a, uint64_t sec) {
    a ^= a >> 47;
    a ^= sec;
    return a * P32_1;
}

// weak-sum parts of 16 bytes at window offset q
__device__ __forceinline__ void weak16(const uint32_t (&w)[4], uint32_t q, uint32_t &sx,
                                       uint32_t &sux) {
    int s = 0, t = 0;
    s = dot4(w[0], 0x01010101u, s);
    s = dot4(w[1], 0x01010101u, s);
    s = dot4(w[2], 0x01010101u, s);
    s = dot4(w[3], 0x01010101u, s);
    t = dot4(w[0], 0x03020100u, t);
    t = dot4(w[1], 0x07060504u, t);
    t = dot4(w[2], 0x0b0a0908u, t);
    t = dot4(w[3], 0x0f0e0d0cu, t);
    sx += (uint32_t)s;
    sux += q * (uint32_t)s + (uint32_t)t;
}

#ifdef VS_WALK_DEBUG
#define WPROG(A_, LANE_, PH_, OFF_, EX_)                                                  \
    do {                                                                                  \
        if ((A_).dbg && (LANE_) == 0) {                                                   \
            const uint32_t wv_ = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;       \
            __hip_atomic_store(&(A_).dbg[wv_ * 4 + 0], (uint64_t)(PH_), __ATOMIC_RELAXED, \
                               __HIP_MEMORY_SCOPE_SYSTEM);                                \
            __hip_atomic_store(&(A_).dbg[wv_ * 4 + 1], (uint64_t)(OFF_), __ATOMIC_RELAXED,\
                               __HIP_MEMORY_SCOPE_SYSTEM);                                \
            __hip_atomic_store(&(A_).dbg[wv_ * 4 + 2], (uint64_t)(EX_), __ATOMIC_RELAXED, \
                               __HIP_MEMORY_SCOPE_SYSTEM);                                \
        }                                                                                 \
    } while (0)
#else
#define WPROG(A_, LANE_, PH_, OFF_, EX_) \
    do {                                 \
    } while (0)
#endif

struct Win {
    uint32_t weak;
    uint64_t lo, hi;
};

// Weak sum and XXH3 (64 / 128, seeded) of the window data[o, o + len),
// len > 240, computed by the whole wave (every lane returns them).
// Restates vsstrong::xxh3_long + merge and get_checksum1 (rsync.hip
// weak_sum); tests compare both with the C oracle / libxxhash.
__device__ Win wave_window(const RsWalkArgs &a, const LaneSec &ls, uint32_t lane, uint64_t o,
                           uint64_t len) {
    using namespace vsstrong;
    const uint8_t *d = a.data;
    const uint64_t dlen = a.dlen;
    const uint32_t s = lane >> 2, m = lane & 3;
    uint64_t A0 = ls.i0, A1 = ls.i1;
    uint32_t sx = 0, sux = 0;
    const uint32_t sh = (uint32_t)(o & 15);
    const uint64_t nb = (len - 1) / 1024;
    for (uint64_t b = 0; b < nb; ++b) {
        uint32_t w[4];
        const uint32_t q = (uint32_t)(b * 1024 + 16 * lane);
        ld16(d, o + q, sh, dlen, w);
        const uint64_t d0 = ((uint64_t)w[1] << 32) | w[0], d1 = ((uint64_t)w[3] << 32) | w[2];
        const uint64_t k0 = d0 ^ ls.s0, k1 = d1 ^ ls.s1;
        uint64_t c0 = (uint64_t)(uint32_t)k0 * (k0 >> 32) + d1;
        uint64_t c1 = (uint64_t)(uint32_t)k1 * (k1 >> 32) + d0;
        weak16(w, q, sx, sux);
        c0 = red16(c0);
        c1 = red16(c1);
        A0 = scramble(A0 + c0, ls.sc0);
        A1 = scramble(A1 + c1, ls.sc1);
    }
    const uint32_t ns = (uint32_t)(((len - 1) - nb * 1024) / 64);
    if (ns) {
        uint32_t w[4] = {0, 0, 0, 0};
        const uint32_t q = (uint32_t)(nb * 1024 + 16 * lane);
        if (s < ns) ld16(d, o + q, sh, dlen, w);
        const uint64_t d0 = ((uint64_t)w[1] << 32) | w[0], d1 = ((uint64_t)w[3] << 32) | w[2];
        const uint64_t k0 = d0 ^ ls.s0, k1 = d1 ^ ls.s1;
        uint64_t c0 = (s < ns) ? (uint64_t)(uint32_t)k0 * (k0 >> 32) + d1 : 0;
        uint64_t c1 = (s < ns) ? (uint64_t)(uint32_t)k1 * (k1 >> 32) + d0 : 0;
        if (s < ns) weak16(w, q, sx, sux);
        A0 += red16(c0);
        A1 += red16(c1);
    }
    {
        // last stripe [len - 64, len), secret offset 192 - 64 - 7; every
        // group computes it (no reduction), lanes 0..3 weak-sum the bytes no
        // earlier stripe covered
        uint32_t w[4];
        const uint64_t q = len - 64 + 16 * m;
        ld16(d, o + q, (uint32_t)((o + len) & 15), dlen, w);
        const uint64_t d0 = ((uint64_t)w[1] << 32) | w[0], d1 = ((uint64_t)w[3] << 32) | w[2];
        const uint64_t k0 = d0 ^ ls.l0, k1 = d1 ^ ls.l1;
        A0 += (uint64_t)(uint32_t)k0 * (k0 >> 32) + d1;
        A1 += (uint64_t)(uint32_t)k1 * (k1 >> 32) + d0;
        const uint64_t covered = nb * 1024 + (uint64_t)ns * 64;
        if (lane < 4) {
            // zero the bytes below `covered` (at most 64 - (len - covered) of them)
            uint32_t wm[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t b0 = q + 4 * k;
                uint32_t mask = 0xffffffffu;
                if (b0 + 4 <= covered) mask = 0;
                else if (b0 < covered) mask = 0xffffffffu << (8 * (uint32_t)(covered - b0));
                wm[k] = w[k] & mask;
            }
            weak16(wm, (uint32_t)q, sx, sux);
        }
    }
    sx = red64(sx);
    sux = red64(sux);
    Win r;
    r.weak = uni((sx & 0xffffu) | (((uint32_t)len * sx - sux) << 16));
    Xxh3Long st;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        st.acc[2 * j] = rdl64(A0, j);
        st.acc[2 * j + 1] = rdl64(A1, j);
    }
    r.lo = st.merge(11, len * P64_1, a.seed);
    r.hi = (a.csum_type == kXxh3_128) ? st.merge(192 - 64 - 11, ~(len * P64_2), a.seed) : 0;
    return r;
}

// the first s2length bytes of (lo, hi) equal block i's sum2
__device__ __forceinline__ bool strong_eq(const RsWalkArgs &a, uint32_t i, uint64_t lo,
                                          uint64_t hi) {
    const uint64_t t0 = a.sum2p[2 * (uint64_t)i], t1 = a.sum2p[2 * (uint64_t)i + 1];
    return ((lo ^ t0) & a.s2mask_lo) == 0 && ((hi ^ t1) & a.s2mask_hi) == 0;
}

// hash_search's chain walk at one offset whose window (length klen) has weak
// sum `sum` and strong sum (lo, hi): blocks with sum1 == sum in descending
// index order, a length check, the strong compare (false alarm on mismatch),
// and the want_i preference.  Returns the matched block or -1.  Uniform.
__device__ int32_t chain_match(const RsWalkArgs &a, uint32_t sum, uint64_t lo, uint64_t hi,
                               int32_t want, uint32_t klen, uint64_t &fa) {
    const uint32_t b = sum >> (32 - a.dbits);
    const uint32_t p0 = uni(a.dir[b]), p1 = uni(a.dir[b + 1]);
    for (uint32_t p = p0; p < p1; ++p) {
        const uint64_t key = uni64(a.tkey[p]);
        const uint32_t s1 = (uint32_t)(key >> 32);
        if (s1 < sum) continue;
        if (s1 > sum) break;
        int32_t i = (int32_t)~(uint32_t)key;
        const uint32_t li = ((uint32_t)i == a.count - 1 && a.remainder) ? a.remainder : a.blength;
        if (li != klen) continue;
        if (!uni((uint32_t)strong_eq(a, (uint32_t)i, lo, hi))) {
            ++fa;
            continue;
        }
        if (i != want && want >= 0 && (uint32_t)want < a.count && uni(a.sum1[want]) == sum &&
            uni((uint32_t)strong_eq(a, (uint32_t)want, lo, hi)))
            i = want;
        return i;
    }
    return -1;
}

// does a full-length block with sum1 == sum exist?  LDS prefilter, filter,
// then the directory (uniform per lane, divergent across lanes)
__device__ __forceinline__ bool probe_full(const RsWalkArgs &a, uint32_t sum) {
    const uint32_t f = sum >> (32 - a.fbits);
    if (!((a.filt[f >> 5] >> (f & 31)) & 1u)) return false;
    const uint32_t b = sum >> (32 - a.dbits);
    const uint32_t p0 = a.dir[b], p1 = a.dir[b + 1];
    for (uint32_t p = p0; p < p1; ++p) {
        const uint64_t key = a.tkey[p];
        const uint32_t s1 = (uint32_t)(key >> 32);
        if (s1 > sum) break;
        if (s1 < sum) continue;
        const uint32_t i = ~(uint32_t)key;
        if (!(i == a.count - 1 && a.remainder)) return true;
    }
    return false;
}

__device__ __forceinline__ int32_t sbyte(const uint8_t *d, uint64_t p) {
    return (int32_t)(int8_t)d[p];
}

// The segment's speculative walk, as a merge target of a re-walk
struct SpecView {
    const int64_t *off;
    const int32_t *idx;
    const int64_t *fab;
    uint32_t n;
    uint64_t fa;
    int64_t exit_off;
    int32_t exit_want;
};

struct SegResult {
    uint32_t n;          // matches written to out_*
    uint32_t from;       // merged: spec matches [from, spec n) follow; else 0xffffffff
    uint64_t fa;
    int64_t exit_off;
    int32_t exit_want;
};

// hash_search from (o, want) over [o, stop); full windows only below
// min(stop, full_end).  Matches go to out_off/out_idx/out_fab (lane 0
// writes); with `spec`, the walk ends at its first match the speculative walk
// also made.
__device__ SegResult walk_segment(const RsWalkArgs &a, const LaneSec &ls, const uint32_t *lfilt,
                                  uint32_t lane, int64_t o, int32_t want, int64_t stop,
                                  int64_t *out_off, int32_t *out_idx, int64_t *out_fab,
                                  uint32_t cap, const SpecView *spec) {
    const int64_t fend = min(stop, (int64_t)a.full_end);
    const uint64_t L = a.blength;
    const uint8_t *d = a.data;
    SegResult res{0, 0xffffffffu, 0, 0, want};
    uint64_t fa = 0;
    uint32_t n = 0;
    bool run = true;
    uint32_t S1 = 0, S2 = 0;  // STEP: window sums at o (low 16 bits meaningful)
    // after a match at h with block i: emit, merge check, next offset
    auto on_match = [&](int64_t h, int32_t i, uint64_t fa_visit) -> bool {
        if (lane == 0 && n < cap) {
            out_off[n] = h;
            out_idx[n] = i;
            out_fab[n] = (int64_t)fa_visit;
        }
        ++n;
        want = i + 1;
        if (spec) {
            // binary search the speculative matches for offset h
            uint32_t lo = 0, hi = spec->n;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if ((int64_t)uni64((uint64_t)spec->off[mid]) < h) lo = mid + 1;
                else hi = mid;
            }
            const bool hitm = lo < spec->n &&
                              uni((uint32_t)(spec->off[lo] == h && spec->idx[lo] == i)) != 0;
            if (hitm) {
                res.from = lo + 1;
                fa = fa_visit + spec->fa - uni64((uint64_t)spec->fab[lo]);
                o = spec->exit_off;
                want = spec->exit_want;
                return true;
            }
        }
        const uint32_t li = ((uint32_t)i == a.count - 1 && a.remainder) ? a.remainder : a.blength;
        o = h + li;
        return false;
    };
    bool merged = false;
    uint64_t it = 0;
    while (!merged && o < fend) {
        ++it;
        WPROG(a, lane, 1, o, it);
        if (run) {
            const Win w = wave_window(a, ls, lane, (uint64_t)o, L);
            const uint64_t fa_visit = fa;
            const int32_t i = unis(chain_match(a, w.weak, w.lo, w.hi, want, (uint32_t)L, fa));
            WPROG(a, lane, 3, o, i);
            if (i >= 0) {
                merged = on_match(o, i, fa_visit);
                continue;
            }
            // roll the window one byte: hash_search's s1/s2 update
            const int32_t xo = sbyte(d, (uint64_t)o);
            const int32_t xi = (o + 1 < fend) ? sbyte(d, (uint64_t)o + L) : 0;
            S1 = uni((w.weak & 0xffffu) - (uint32_t)xo + (uint32_t)xi);
            S2 = uni((w.weak >> 16) - (uint32_t)L * (uint32_t)xo + S1);
            ++o;
            run = false;
            continue;
        }
        // ---- STEP: offsets [A, A + 1024) of which [o, fend) count ----
        const uint64_t A = (uint64_t)o & ~15ull;
        // sums at A: roll back from o (at most 15 steps)
        uint32_t T1 = S1, T2 = S2;
        for (uint64_t u = (uint64_t)o; u > A; --u) {
            const uint64_t v = u - 1;
            const int32_t xo = sbyte(d, v), xi = sbyte(d, v + L);
            T2 = T2 - T1 + (uint32_t)L * (uint32_t)xo;
            T1 = T1 - (uint32_t)(xi - xo);
        }
        T1 = uni(T1);
        T2 = uni(T2);
        const uint64_t c = A + 16 * (uint64_t)lane;
        uint32_t wo[4], wi[4];
        {
            const uint4 v = gl16_guard(d, c, a.dlen);
            wo[0] = v.x; wo[1] = v.y; wo[2] = v.z; wo[3] = v.w;
        }
        ld16(d, c + L, (uint32_t)((c + L) & 15), a.dlen, wi);
        int Xo = 0, Xi = 0, Eo = 0, Ei = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            Xo = dot4(wo[k], 0x01010101u, Xo);
            Xi = dot4(wi[k], 0x01010101u, Xi);
            // weights 16 - t for byte t = 4k .. 4k+3
            const uint32_t wt = (uint32_t)((16 - 4 * k) | ((15 - 4 * k) << 8) | ((14 - 4 * k) << 16) |
                                           ((13 - 4 * k) << 24));
            Eo = dot4(wo[k], wt, Eo);
            Ei = dot4(wi[k], wt, Ei);
        }
        const uint32_t D = (uint32_t)(Xi - Xo), E = (uint32_t)(Ei - Eo), X = (uint32_t)Xo;
        const uint32_t P = excl_scan(D, lane);
        const uint32_t Y = excl_scan(E + 16u * P - (uint32_t)L * X, lane);
        uint32_t s1 = T1 + P;
        uint32_t s2 = T2 + 16u * lane * T1 + Y;
        uint32_t sums[16];
        uint32_t valid = 0;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            sums[t] = __builtin_amdgcn_perm(s2, s1, 0x05040100u);  // (s1 & 0xffff) | (s2 << 16)
            const int32_t xo = __builtin_amdgcn_sbfe((int)wo[t >> 2], 8 * (t & 3), 8);
            const int32_t xi = __builtin_amdgcn_sbfe((int)wi[t >> 2], 8 * (t & 3), 8);
            s1 += (uint32_t)(xi - xo);
            s2 = s2 - (uint32_t)L * (uint32_t)xo + s1;
            const int64_t q = (int64_t)c + t;
            valid |= (uint32_t)(q >= o && q < fend) << t;
        }
        // membership: LDS prefilter, then filter + directory for the survivors
        uint32_t hit = 0;
        if (a.lbits) {
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const uint32_t fl = sums[t] >> (32 - a.lbits);
                hit |= ((lfilt[fl >> 5] >> (fl & 31)) & 1u) << t;
            }
            hit &= valid;
        } else {
            hit = valid;
        }
        for (uint32_t m = hit; m;) {
            const int t = __builtin_ctz(m);
            m &= m - 1;
            uint32_t st = sums[0];
#pragma unroll
            for (int k = 1; k < 16; ++k) st = (t == k) ? sums[k] : st;
            if (!probe_full(a, st)) hit &= ~(1u << t);
        }
        // visit the hits in offset order (lane order, then bit order)
        bool matched = false;
        uint64_t lanes = __ballot(hit != 0);
        WPROG(a, lane, 5, o, lanes);
        while (lanes) {
            const uint32_t hl = (uint32_t)__builtin_ctzll(lanes);
            const uint32_t hm = (uint32_t)__builtin_amdgcn_readlane((int)hit, (int)hl);
            const uint32_t t = (uint32_t)__builtin_ctz(hm);
            const int64_t h = (int64_t)A + 16 * (int64_t)hl + t;
            WPROG(a, lane, 6, h, lanes);
            const Win w = wave_window(a, ls, lane, (uint64_t)h, L);
            WPROG(a, lane, 7, h, w.weak);
            const uint64_t fa_visit = fa;
            const int32_t i = unis(chain_match(a, w.weak, w.lo, w.hi, want, (uint32_t)L, fa));
            if (i >= 0) {
                merged = on_match(h, i, fa_visit);
                matched = true;
                run = true;
                break;
            }
            if (lane == hl) hit &= hit - 1;
            lanes = __ballot(hit != 0);
        }
        if (matched) continue;
        // no match in this batch: continue at A + 1024 with lane 63's sums
        const uint64_t nx = A + kBatch;
        if ((int64_t)nx >= fend) {
            o = fend;
            break;
        }
        S1 = (uint32_t)__builtin_amdgcn_readlane((int)s1, 63);
        S2 = (uint32_t)__builtin_amdgcn_readlane((int)s2, 63);
        o = (int64_t)nx;
    }
    WPROG(a, lane, 9, o, n);
    res.n = n;
    res.fa = fa;
    res.exit_off = o;
    res.exit_want = want;
    return res;
}

__device__ __forceinline__ void load_prefilter(const RsWalkArgs &a, uint32_t *lfilt) {
    const uint32_t lw = a.lbits ? (1u << a.lbits) / 32 : 0;
    for (uint32_t i = threadIdx.x; i < lw; i += blockDim.x) lfilt[i] = a.filt_l[i];
    __syncthreads();
}

// segments are dealt to waves statically (grid-stride): wave w walks
// segments w, w + W, w + 2W, ...
__device__ __forceinline__ uint32_t wave_id() {
    return uni(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64);
}
__device__ __forceinline__ uint32_t wave_count() { return gridDim.x * (blockDim.x / 64); }

__device__ __forceinline__ int64_t seg_lo(const RsWalkArgs &a, uint32_t k) {
    return a.lo + (int64_t)k * a.seg_len;
}
__device__ __forceinline__ int64_t seg_hi(const RsWalkArgs &a, uint32_t k) {
    return min(a.lo + (int64_t)(k + 1) * a.seg_len, a.hi);
}

// speculative walk of every segment from its own start (segment 0 from the
// range's speculative entry a.e0 / a.w0; the others with want_i "no
// preference" = count)
__global__ __launch_bounds__(kWalkThreads) void rs_walk_spec_kernel(RsWalkArgs a) {
    __shared__ uint32_t lfilt[kLdsFiltWordsW];
    load_prefilter(a, lfilt);
    const uint32_t lane = threadIdx.x & 63;
    const LaneSec ls = lane_secrets(lane, a.seed);
    for (uint32_t k = wave_id(); k < a.nseg; k += wave_count()) {
        WPROG(a, lane, 11, k, a.nseg);
        const int64_t e = (int64_t)uni64((uint64_t)(k ? seg_lo(a, k) : a.e0));
        const int32_t w = unis(k ? (int32_t)a.count : a.w0);
        const uint64_t base = (uint64_t)k * a.cap;
        const SegResult r = walk_segment(a, ls, lfilt, lane, e, w, seg_hi(a, k), a.spec_off + base,
                                         a.spec_idx + base, a.spec_fab + base, a.cap, nullptr);
        if (lane == 0) {
            a.spec_n[k] = r.n;
            a.spec_fa[k] = r.fa;
            a.spec_exit[k] = r.exit_off;
            a.spec_exitw[k] = r.exit_want;
            a.fin_entry[k] = e;
            a.fin_entryw[k] = w;
            a.fin_from[k] = 0xffffffffu;   // the final walk is the speculative one
            a.fin_n[k] = 0;
            a.fin_fa[k] = r.fa;
            a.exit_new[k] = r.exit_off;
            a.exitw_new[k] = r.exit_want;
            if (r.n > a.cap) atomicOr(a.flags, 2u);
        }
        WPROG(a, lane, 10, k, r.n);
    }
    WPROG(a, lane, 12, 0, 0);
}

// one stitch pass: a segment whose entry (the previous segment's exit from
// the last pass, or a.e0 / a.w0) differs from the entry of its current walk
// re-walks from it, merging into its speculative walk
__global__ __launch_bounds__(kWalkThreads) void rs_walk_stitch_kernel(RsWalkArgs a) {
    __shared__ uint32_t lfilt[kLdsFiltWordsW];
    load_prefilter(a, lfilt);
    const uint32_t lane = threadIdx.x & 63;
    const LaneSec ls = lane_secrets(lane, a.seed);
    for (uint32_t k = wave_id(); k < a.nseg; k += wave_count()) {
        WPROG(a, lane, 21, k, a.nseg);
        const int64_t e = (int64_t)uni64((uint64_t)(k ? a.exit_old[k - 1] : a.e0));
        const int32_t w = unis(k ? a.exitw_old[k - 1] : a.w0);
        const bool same = uni((uint32_t)(e == a.fin_entry[k] && w == a.fin_entryw[k])) != 0;
        if (same) {
            WPROG(a, lane, 23, k, e);
            if (lane == 0) {
                a.exit_new[k] = a.exit_old[k];
                a.exitw_new[k] = a.exitw_old[k];
            }
        } else {
        const uint64_t base = (uint64_t)k * a.cap;
        SpecView sv{a.spec_off + base, a.spec_idx + base, a.spec_fab + base, uni(a.spec_n[k]),
                    uni64(a.spec_fa[k]), (int64_t)uni64((uint64_t)a.spec_exit[k]),
                    unis(a.spec_exitw[k])};
        SegResult r;
        if (e == seg_lo(a, k) && w == (k ? (int32_t)a.count : a.spec_w0)) {
            // back to the speculative entry
            r = SegResult{0, 0, sv.fa, sv.exit_off, sv.exit_want};
        } else {
            r = walk_segment(a, ls, lfilt, lane, e, w, seg_hi(a, k), a.fin_off + base,
                             a.fin_idx + base, a.fin_fab + base, a.cap, &sv);
        }
        if (lane == 0) {
            a.fin_entry[k] = e;
            a.fin_entryw[k] = w;
            a.fin_n[k] = r.n;
            a.fin_from[k] = (r.from == 0xffffffffu) ? sv.n : r.from;
            a.fin_fa[k] = r.fa;
            a.exit_new[k] = r.exit_off;
            a.exitw_new[k] = r.exit_want;
            if (r.exit_off != a.exit_old[k] || r.exit_want != a.exitw_old[k]) atomicOr(a.flags, 1u);
            if (r.n > a.cap) atomicOr(a.flags, 2u);
        }
        WPROG(a, lane, 20, k, r.n);
        }
    }
    WPROG(a, lane, 22, 0, 0);
}

// sum2 (count x s2length bytes) -> 16 zero-padded bytes per block
__global__ void rs_pad_sum2_kernel(const uint8_t *sum2, uint32_t count, uint32_t s2length,
                                   uint64_t *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    uint64_t v[2] = {0, 0};
    for (uint32_t j = 0; j < s2length; ++j)
        v[j >> 3] |= (uint64_t)sum2[(uint64_t)i * s2length + j] << (8 * (j & 7));
    out[2 * (uint64_t)i] = v[0];
    out[2 * (uint64_t)i + 1] = v[1];
}

}  // namespace

hipError_t launch_rs_walk(const RsWalkArgs &a, bool stitch, int cus, hipStream_t s) {
    if (!a.nseg) return hipSuccess;
    if (a.lbits > 20) return hipErrorInvalidValue;
    const uint32_t waves = kWalkThreads / 64;
    const uint64_t grid = std::min<uint64_t>((a.nseg + waves - 1) / waves, (uint64_t)std::max(cus, 1));
    hipError_t e = hipMemsetAsync(a.work, 0, 4, s);
    if (e != hipSuccess) return e;
    if (stitch)
        rs_walk_stitch_kernel<<<(uint32_t)grid, kWalkThreads, 0, s>>>(a);
    else
        rs_walk_spec_kernel<<<(uint32_t)grid, kWalkThreads, 0, s>>>(a);
    return hipGetLastError();
}

hipError_t launch_rs_pad_sum2(const uint8_t *sum2, uint32_t count, uint32_t s2length,
                              uint64_t *out, hipStream_t s) {
    if (!count) return hipSuccess;
    rs_pad_sum2_kernel<<<(count + 255) / 256, 256, 0, s>>>(sum2, count, s2length, out);
    return hipGetLastError();
}

}  // namespace vsgpu
