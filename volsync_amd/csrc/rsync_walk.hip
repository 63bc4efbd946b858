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
#include <utility>

#include "internal.hpp"
#include "strong.hpp"

namespace vsgpu {
namespace {

using vsstrong::P32_1;

#ifndef VS_WALK_T
#define VS_WALK_T 512
#endif
#ifndef VS_WALK_RRING
#define VS_WALK_RRING 4
#endif
#ifndef VS_WALK_FRING
#define VS_WALK_FRING 2
#endif
// STEP probes: every survivor of a batch in one round trip, a lane each
// (stage1 / stage2 in walk_segment); 0 = each lane probes its own in turn
#ifndef VS_WALK_LATEFW
#define VS_WALK_LATEFW 0
#endif
#ifndef VS_WALK_PSCAN
#define VS_WALK_PSCAN 1
#endif
constexpr uint32_t kWalkThreads = VS_WALK_T;             // 8 waves (up to 256 VGPRs each); the 128 KiB prefilter admits one WG/CU
constexpr uint32_t kWalkRing = VS_WALK_RRING;                  // window blocks in flight per lane in the wave walk
#ifndef VS_WALK_LDSF
#define VS_WALK_LDSF (1u << 15)
#endif
constexpr uint32_t kLdsFiltWordsW = VS_WALK_LDSF;  // 2^20-bit LDS prefilter
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
// exclusive prefix sum over the wave (lane order): the GFX9 DPP scan
// (row_shr 1/2/4/8 inside each row, then row_bcast 15 / 31 across rows)
__device__ __forceinline__ uint32_t excl_scan(uint32_t v, uint32_t) {
    uint32_t x = v;
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
    return x - v;
}

// ---- four windows per wave ------------------------------------------------
// A wave hashes up to kRows windows at once, one per 16-lane row: lane
// (row r, q = 4s' + m) reads 16 bytes of each 256-byte quarter of every 1 KiB
// XXH3 block of window r, i.e. words 2m, 2m+1 of stripes s' , s'+4, s'+8,
// s'+12, so a row's load is 256 contiguous bytes and the per-block reduction
// (over s') stays inside the row (two DPP row rotations).  Loads are issued
// kRing blocks ahead of their use; the window bytes are read with unaligned
// dwordx4 loads (gfx950 runs in unaligned-access mode; hipcc emits the same
// for a byte-aligned memcpy).
constexpr uint32_t kRows = 4;
constexpr uint32_t kRing = 2;   // blocks in flight per lane

// DPP move within the wave (row rotations, quad permutations)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
    return ((uint64_t)dpp<CTRL>((uint32_t)(v >> 32)) << 32) | dpp<CTRL>((uint32_t)v);
}
// sum over the 4 lanes of a row with the same q & 3 (row_ror 4, row_ror 8)
__device__ __forceinline__ uint64_t row_sum_sp(uint64_t v) {
    v += dpp64<0x124>(v);
    v += dpp64<0x128>(v);
    return v;
}
// sum over the 16 lanes of a row
__device__ __forceinline__ uint32_t row_sum16(uint32_t v) {
    v += dpp<0x121>(v);
    v += dpp<0x122>(v);
    v += dpp<0x124>(v);
    v += dpp<0x128>(v);
    return v;
}
// sum over a quad (quad_perm [1,0,3,2] then [2,3,0,1])
__device__ __forceinline__ uint64_t quad_sum(uint64_t v) {
    v += dpp64<0xB1>(v);
    v += dpp64<0x4E>(v);
    return v;
}

__device__ __forceinline__ uint4 ldu16(const uint8_t *p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}

// The seeded custom secret (XXH3_initCustomSecret: even words + seed, odd
// words - seed), 24 words, staged in LDS once per workgroup: a lane reads its
// stripe's two words with one ds_read2_b64 instead of holding 20 registers.
// Words 24 .. 69 hold the pairs (w[i], w[i + 1]), i < 23, 16-byte aligned:
// the wide flushes read a stripe's two words with one ds_read_b128 at a
// lane-dependent stripe (wide_windows).
struct RowSec {
    const uint64_t *w;   // LDS, [kSecWords]
};
constexpr uint32_t kSecWords = 24 + 2 * 23;
__device__ __forceinline__ void load_secret(uint64_t *lsec, uint64_t seed) {
    if (threadIdx.x < 24) lsec[threadIdx.x] = vsstrong::sec64(threadIdx.x, seed);
    if (threadIdx.x < 46) {
        const uint32_t i = threadIdx.x >> 1;
        lsec[24 + threadIdx.x] = vsstrong::sec64(i + (threadIdx.x & 1), seed);
    }
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

// one 16-byte piece: XXH3 accumulate of words 2m, 2m+1 with secrets (k0, k1)
__device__ __forceinline__ void acc16(const uint4 v, uint64_t k0s, uint64_t k1s, uint64_t &c0,
                                      uint64_t &c1) {
    const uint64_t d0 = ((uint64_t)v.y << 32) | v.x, d1 = ((uint64_t)v.w << 32) | v.z;
    const uint64_t k0 = d0 ^ k0s, k1 = d1 ^ k1s;
    c0 += (uint64_t)(uint32_t)k0 * (k0 >> 32) + d1;
    c1 += (uint64_t)(uint32_t)k1 * (k1 >> 32) + d0;
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

// Optional per-wave phase timing (a.prof != nullptr, set in profiling builds):
// s_memtime cycles and counts per phase, summed into a.prof[wave * 16 + ...]
enum : int {
    kPrRun = 0, kPrStep = 1, kPrFlush = 2, kPrChain = 3, kPrSeg = 4,
    kPrBandFill = 5, kPrBandPairs = 6, kPrBandChain = 7,
    // the wave walk's STEP batch, split: sums, LDS prefilter, blocked-filter
    // gathers, directory probes, queueing
    kPrStepSums = 8, kPrStepLds = 9, kPrStepGather = 10, kPrStepProbe = 11, kPrStepQueue = 12,
    // wide flushes: iterations per pass, windows per pass (sums, not cycles)
    kPrFlushIters = 13, kPrFlushWin = 14,
    kPrN = 16
};
// The counters live in scalar registers; compiled in only with the build
// flag VS_WALK_PROF (tools/build_variant.sh walkprof -DVS_WALK_PROF=1; that
// library, selected by VSGPU_LIB=..., profiles every walk -- the library reads
// no environment variable): 16 phases x two u64 otherwise spill SGPRs into
// VGPR lanes all over the production kernel.
#ifdef VS_WALK_PROF
struct WProf {
    bool on;
    uint64_t cyc[kPrN], cnt[kPrN];
};
__device__ __forceinline__ uint64_t wclock(const WProf &w) {
    return w.on ? (uint64_t)__builtin_amdgcn_s_memtime() : 0;
}
__device__ __forceinline__ void wadd(WProf &w, int ph, uint64_t t0) {
    if (w.on) {
        w.cyc[ph] += (uint64_t)__builtin_amdgcn_s_memtime() - t0;
        w.cnt[ph] += 1;
    }
}
#define WPROF_INIT(on_) WProf wp{(on_), {}, {}}
#else
struct WProf {
    static constexpr bool on = false;
    uint64_t cyc[kPrN], cnt[kPrN];   // never touched: `on` is a constant false
};
__device__ __forceinline__ uint64_t wclock(const WProf &) { return 0; }
__device__ __forceinline__ void wadd(WProf &, int, uint64_t) {}
#define WPROF_INIT(on_) WProf wp; (void)(on_)
#endif

struct RowWin {
    uint32_t weak;     // get_checksum1 of the row's window (WEAK only)
    uint64_t lo, hi;   // XXH3 low / high 64 bits (valid in lanes q < 4 of the row)
};

// Weak sum (WEAK) and seeded XXH3 (64 / 128) of the window data[o, o + len),
// len > 240, o per row (the lane's row's window; rows may repeat a window).
// Every window is a full one inside the readable data.  Restates
// vsstrong::xxh3_long + merge and get_checksum1 (rsync.hip weak_sum); tests
// compare both with the C oracle / libxxhash.
template <bool WEAK, uint32_t RING = kRing>
__device__ RowWin rows_window(const RsWalkArgs &a, const RowSec &rs, uint32_t lane, uint64_t o,
                              uint64_t len) {
    using namespace vsstrong;
    const uint32_t q = lane & 15, sp = q >> 2, m = q & 3;
    const uint8_t *p = a.data + o + 16 * q;   // this lane's piece of each 256-byte quarter
    uint64_t A0 = (m == 0) ? P32_3 : (m == 1) ? P64_2 : (m == 2) ? P64_4 : P64_5;
    uint64_t A1 = (m == 0) ? P64_1 : (m == 1) ? P64_3 : (m == 2) ? P32_2 : P32_1;
    uint32_t sx = 0, sux = 0;
    const uint32_t nb = (uint32_t)((len - 1) / 1024);
    auto block = [&](const uint4 (&v)[4], uint32_t b) {
        uint64_t c0 = 0, c1 = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            acc16(v[j], rs.w[4 * j + sp + 2 * m], rs.w[4 * j + sp + 2 * m + 1], c0, c1);
            if (WEAK) {
                const uint32_t w[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
                weak16(w, b * 1024 + 256 * j + 16 * q, sx, sux);
            }
        }
        A0 = scramble(A0 + row_sum_sp(c0), rs.w[16 + 2 * m]);
        A1 = scramble(A1 + row_sum_sp(c1), rs.w[17 + 2 * m]);
    };
    auto load = [&](uint4 (&v)[4], uint32_t b) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = ldu16(p + (uint64_t)b * 1024 + 256 * j);
    };
    // full blocks through a ring of RING blocks in flight
    static_assert(RING >= 2, "at least two blocks in flight");
    uint4 ring[RING][4];
#pragma unroll
    for (uint32_t k = 0; k < RING; ++k)
        if (k < nb) load(ring[k], k);
    for (uint32_t b = 0; b < nb; b += RING) {
#pragma unroll
        for (uint32_t k = 0; k < RING; ++k) {
            if (b + k >= nb) break;
            block(ring[k], b + k);
            if (b + k + RING < nb) load(ring[k], b + k + RING);
        }
    }
    // the partial block: ns stripes, no scramble
    const uint32_t ns = (uint32_t)(((len - 1) - (uint64_t)nb * 1024) / 64);
    if (ns) {
        uint64_t c0 = 0, c1 = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (4 * j + sp < ns) {
                const uint4 v = ldu16(p + (uint64_t)nb * 1024 + 256 * j);
                acc16(v, rs.w[4 * j + sp + 2 * m], rs.w[4 * j + sp + 2 * m + 1], c0, c1);
                if (WEAK) {
                    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
                    weak16(w, nb * 1024 + 256 * j + 16 * q, sx, sux);
                }
            }
        }
        A0 += row_sum_sp(c0);
        A1 += row_sum_sp(c1);
    }
    RowWin r;
    // last stripe [len - 64, len), secret offset 192 - 64 - 7 = 121: lanes with
    // s' == 0 (q == m) add it and weak-sum the bytes no earlier stripe covered
    uint64_t tA = 0, tB = 0;
    if (sp == 0) {
        const uint32_t qq = (uint32_t)(len - 64 + 16 * m);
        const uint4 v = ldu16(a.data + o + qq);
        uint64_t c0 = 0, c1 = 0;
        acc16(v, csec_at(121 + 16 * m, a.seed), csec_at(129 + 16 * m, a.seed), c0, c1);
        A0 += c0;
        A1 += c1;
        if (WEAK) {
            const uint64_t covered = (uint64_t)nb * 1024 + (uint64_t)ns * 64;
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
            uint32_t wm[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t b0 = qq + 4 * k;
                uint32_t mask = 0xffffffffu;
                if (b0 + 4 <= covered) mask = 0;
                else if (b0 < covered) mask = 0xffffffffu << (8 * (uint32_t)(covered - b0));
                wm[k] = w[k] & mask;
            }
            weak16(wm, qq, sx, sux);
        }
        // merge terms of accumulators 2m, 2m + 1 (64-bit: offset 11; high half: 117)
        tA = fold64(A0 ^ csec_at(11 + 16 * m, a.seed), A1 ^ csec_at(19 + 16 * m, a.seed));
        if (a.csum_type == kXxh3_128)
            tB = fold64(A0 ^ csec_at(117 + 16 * m, a.seed), A1 ^ csec_at(125 + 16 * m, a.seed));
    }
    tA = quad_sum(tA);
    tB = quad_sum(tB);
    r.lo = xxh3_aval(len * P64_1 + tA);
    r.hi = (a.csum_type == kXxh3_128) ? xxh3_aval(~(len * P64_2) + tB) : 0;
    r.weak = 0;
    if (WEAK) {
        sx = row_sum16(sx);
        sux = row_sum16(sux);
        r.weak = (sx & 0xffffu) | (((uint32_t)len * sx - sux) << 16);
    }
    return r;
}

// ---- wide flushes: up to 16 windows, address-lockstep ----------------------
// At real C4 density a resync after an edit visits ~64 false-alarm windows of
// one block length within ~2 block lengths of source; hashed four at a time
// (rows_window) every flush re-streams the whole span, latency-bound on the
// 8 KiB a wave keeps in flight.  Here window j (lanes 4j .. 4j+3, lane k owning
// accumulators 2k, 2k+1 and reading bytes [16k, 16k + 16) of every stripe --
// the signature pass's layout) hashes its block b = t - tau_j in iteration t,
// tau_j = (h_j - h_0) >> 10, so every window of the wave reads inside the same
// 2 KiB, [h_0 + 1024 t, h_0 + 1024 t + 2048).  The wave loads each KiB of
// that span once, 16 bytes per lane, kWideD iterations ahead (4 registers per
// KiB in flight), and writes it into a per-wave LDS ring of two 1 KiB slots
// plus a mirror of slot 0 (so a window's 2 KiB are always contiguous); the
// windows read their stripes from there (three aligned qwords per 16 bytes,
// in a bank-balanced per-lane stripe order, realigned by the window's byte
// offset; see wide_windows).  Windows
// not yet started or already finished compute on stale bytes and keep their
// accumulators.  Same XXH3 as rows_window; window j's results sit in lanes
// 4j .. 4j+3.
constexpr uint32_t kWideQ = 16;
#ifndef VS_PREDICT
#define VS_PREDICT 3
#endif
constexpr uint32_t kPredict = VS_PREDICT;   // blocks want .. want + 2 flag a likely resync hit
#ifndef VS_WIDE_D
#define VS_WIDE_D 8
#endif
// KiB in flight per wave: 8.  Round 4 measured 2, 4, 6, 8 at 44.6, 45.2, 46.5,
// 46.3 ms of share walk (fewer registers held across the call beat a deeper
// prefetch, profiles/r04_walk_step/ab_wd*); with round 5's 136-VGPR flush (no
// callee saves) 4, 6, 8 measure 41.67-41.76, 41.56-41.58, 41.08-41.13 ms at
// the share and 41.0-41.3, 41.05-41.16, 40.64-40.75 at the 64 GiB shape
// (profiles/r05_walk/prefetch); 12 and 16 no longer unroll (the ring goes to
// scratch)
constexpr uint32_t kWideD = VS_WIDE_D;
constexpr uint32_t kWideRingBytes = 3 * 1024;             // per wave: slots 0, 1, mirror of 0

// f(integral_constant<uint32_t, I>) for I < N, unrolled at compile time (asm
// immediates need constants)
template <class F, uint32_t... I>
__device__ __forceinline__ void sfor_(F &&f, std::integer_sequence<uint32_t, I...>) {
    (f(std::integral_constant<uint32_t, I>{}), ...);
}
template <uint32_t N, class F>
__device__ __forceinline__ void sfor(F &&f) {
    sfor_(f, std::make_integer_sequence<uint32_t, N>{});
}

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
// stripe S of a wide flush: 24 ring bytes (three ds_read_b64 from the
// lane's rotated stripe base rb) and its secret pair (ds_read_b128); the
// registers are written when wide_wait says so
template <uint32_t S>
__device__ __forceinline__ void wide_issue(uint32_t rb, uint32_t sb, uint64_t &r01, uint64_t &r23,
                                           uint64_t &r45, u64x2 &kk) {
    asm volatile(
        "ds_read_b64 %0, %4 offset:%6\n\t"
        "ds_read_b64 %1, %4 offset:%7\n\t"
        "ds_read_b64 %2, %4 offset:%8\n\t"
        "ds_read_b128 %3, %5 offset:%9"
        : "=v"(r01), "=v"(r23), "=v"(r45), "=v"(kk)
        : "v"(rb), "v"(sb), "n"(256 * (S >> 2)), "n"(256 * (S >> 2) + 8), "n"(256 * (S >> 2) + 16),
          "n"(64 * (S >> 2))
        : "memory");
}
// a stripe's four reads have landed once at most N later LDS operations
// are outstanding (the counter holds 15)
#ifndef VS_WIDE_PIPE
#define VS_WIDE_PIPE 3
#endif
constexpr uint32_t kWidePipe = VS_WIDE_PIPE;   // stripes in flight per lane
// wide_issue's loads are invisible to the compiler until wide_wait: a copy or
// spill of r01 / r23 / r45 / kk between the two would read the registers
// before the data lands.  tools/check_lds_asm.py checks the compiled walk for
// that (every read of a pending destination VGPR before its s_waitcnt); the
// shipped depths are the ones it has passed.
#ifndef VS_WIDE_UNCHECKED
static_assert(VS_WIDE_PIPE == 3 && VS_WIDE_D == 8,
              "wide-flush depth not checked by tools/check_lds_asm.py (define VS_WIDE_UNCHECKED for A/B builds)");
#endif
template <uint32_t N>
__device__ __forceinline__ void wide_wait(uint64_t &r01, uint64_t &r23, uint64_t &r45, u64x2 &kk) {
    static_assert(N <= 15, "lgkmcnt");
    asm volatile("s_waitcnt lgkmcnt(%4)"
                 : "+v"(r01), "+v"(r23), "+v"(r45), "+v"(kk)
                 : "n"(N)
                 : "memory");
}

typedef __attribute__((address_space(1))) const uint8_t g_u8;
typedef __attribute__((address_space(3))) const uint64_t l_u64;
typedef __attribute__((address_space(3))) uint8_t l_u8;
typedef __attribute__((address_space(1))) const u64x2 g_u64x2;
// 16 bytes at any byte address (one global_load_dwordx4: gfx950 unaligned mode)
__device__ __forceinline__ u64x2 gld2(g_u8 *p) {
    return *(g_u64x2 *)p;
}
__device__ __forceinline__ void acc2(const u64x2 d, uint64_t k0s, uint64_t k1s, uint64_t &c0,
                                     uint64_t &c1) {
    const uint64_t k0 = d.x ^ k0s, k1 = d.y ^ k1s;
    c0 += (uint64_t)(uint32_t)k0 * (k0 >> 32) + d.y;
    c1 += (uint64_t)(uint32_t)k1 * (k1 >> 32) + d.x;
}

// Not inlined: inlined, its registers and the STEP state live across a flush
// spilled 75 VGPRs of the walk (26 without it; called, 64).  Typed pointers and uniform
// scalars: a call boundary would otherwise turn every load into a flat one
// and the block loop into a divergent one.
__device__ __noinline__ RowWin wide_windows(g_u8 *data, uint64_t dlen, l_u64 *sw0, l_u8 *ring,
                                            uint64_t seed, int csum_type, uint32_t lane, int64_t qh,
                                            uint32_t nq, uint64_t len) {
    using namespace vsstrong;
    nq = uni(nq);
    len = uni64(len);
    seed = uni64(seed);
    dlen = uni64(dlen);
    csum_type = unis(csum_type);
    const uint32_t j = lane >> 2, k = lane & 3;
    const int64_t h0 = (int64_t)rdl64((uint64_t)qh, 0);
    const int64_t hl = (int64_t)rdl64((uint64_t)qh, (int)(nq - 1));
    // windows past nq copy window 0 (lower half) or 8 (upper half, if live)
    // and read its addresses: an LDS broadcast, no bank of their own
    const uint32_t jd = j < nq ? j : (j >= 8 && nq > 8 ? 8u : 0u);
    const int64_t hj = (int64_t)(((uint64_t)(uint32_t)__shfl((int)(uint32_t)((uint64_t)qh >> 32),
                                                             (int)jd, 64) << 32) |
                                 (uint32_t)__shfl((int)(uint32_t)qh, (int)jd, 64));
    const uint32_t tau = (uint32_t)((hj - h0) >> 10);
    const uint32_t rj = (uint32_t)(hj - h0) - 1024 * tau;   // window j's offset in iteration t's 2 KiB
    const uint32_t sh = rj & 3;                              // its bytes' offset in LDS dwords
    const uint32_t nb = (uint32_t)((len - 1) / 1024);
    const uint32_t T = uni((uint32_t)((hl - h0) >> 10)) + nb;
    uint64_t a0 = (k == 0) ? P32_3 : (k == 1) ? P64_2 : (k == 2) ? P64_4 : P64_5;
    uint64_t a1 = (k == 0) ? P64_1 : (k == 1) ? P64_3 : (k == 2) ? P32_2 : P32_1;
    const uint64_t scr0 = sw0[16 + 2 * k], scr1 = sw0[17 + 2 * k];
    // Bank-balanced stripe order.  A lane reads its 16 bytes of a stripe as
    // three aligned ds_read_b64 (24 bytes from (rj & ~7) + 16 k + 64 sigma,
    // realigned below), whose bank pair -- (address / 8) mod 32 within a
    // 256-byte bank row -- is b + 8 sigma, b = (rj >> 3) + 2 k, plus the
    // wave's ring base, common to all its lanes.  A half-wave (8 windows x 4 lanes)
    // meets the 32 pairs in 8 classes (b mod 8), four pairs each (sigma
    // mod 4 picks one); each lane walks its stripes in the order
    // sigma = 4 g + ((u + q) & 3) for s = 4 g + u, q chosen so that the
    // lanes of one class take distinct pairs at every s (their rank in the
    // class, mod 4).  Random window offsets otherwise put several lanes of a
    // half on one bank (the dword reads: 54 % of LDS cycles conflicted,
    // profiles/r04_end).  XXH3 sums the stripes' contributions, so the order
    // is free; the secret pair follows sigma.
    uint32_t q;
    {
        const uint32_t b = (rj >> 3) + 2 * k;
        const uint32_t cls = b & 7;
        const bool part = j < nq || j == 8;
        const uint64_t below = ((1ull << lane) - 1) & (lane < 32 ? 0xffffffffull : 0xffffffff00000000ull);
        uint64_t mine = 0;
#pragma unroll
        for (uint32_t c = 0; c < 8; ++c) {
            const uint64_t m = __ballot(part && cls == c);
            mine = cls == c ? m : mine;
        }
        const uint32_t rank = (uint32_t)__builtin_popcountll(mine & below);
        const uint32_t qs = (uint32_t)(rank - (b >> 3)) & 3;
        const uint32_t src = j < nq ? lane : (j >= 8 ? 32 + k : k);
        q = (uint32_t)__shfl((int)qs, (int)src, 64);
    }
    const uint32_t e4 = (rj >> 2) & 1;   // the 16 bytes start in the qword's upper dword
    const uint32_t upm = e4 ? 0xffffffffu : 0u;   // select mask (a VGPR: v_bitop3 stays 2.3 cycles)
    // LDS byte addresses: the ring, and the secret pairs (2 k + sigma)
    const uint32_t ringa = (uint32_t)(uintptr_t)ring;
    const uint32_t seca = (uint32_t)(uintptr_t)(sw0 + 24) + 32 * k;
    uint32_t roff[4], sb[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
        roff[u] = (rj & ~7u) + 16 * k + 64 * ((u + q) & 3);
        sb[u] = seca + 16 * ((u + q) & 3);
    }
    // KiB n of the span: [h0 + 1024 n, + 1024), lane l's 16 bytes (clamped at
    // the data end: no active window reads past it).  The loads are issued in
    // asm and waited for by hand (vmcnt counts in issue order): the compiler's
    // own accounting of a register ring carried across the loop's back edge
    // waits for every load at the loop head, which exposes a full memory
    // latency per group of kWideD iterations.
    const uint64_t src = (uint64_t)(uintptr_t)(data + h0 + 16 * lane);
    const uint64_t room = dlen - 16 - ((uint64_t)h0 + 16 * lane);
    auto fetch = [&](uint32_t n) -> u32x4 {
        const uint64_t o = 1024ull * n;
        const uint64_t at = src + (o < room ? o : room);
        u32x4 v;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(at) : "memory");
        return v;
    };
    // KiB n into slot n & 1 (and slot 0's mirror); the ring is this wave's
    auto put = [&](uint32_t n, const u32x4 v) {
        *(__attribute__((address_space(3))) u32x4 *)(ring + 1024 * (n & 1) + 16 * lane) = v;
        if ((n & 1) == 0) *(__attribute__((address_space(3))) u32x4 *)(ring + 2048 + 16 * lane) = v;
    };
    u32x4 inflight[kWideD];   // KiB t + 1 + i for i < kWideD, at the top of iteration t
    {
        u32x4 v0 = fetch(0);
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(v0) :: "memory");
        put(0, v0);
    }
#pragma unroll
    for (uint32_t i = 0; i < kWideD; ++i) inflight[i] = fetch(1 + i);
    static_assert(kWideD % 2 == 0, "t & 1 == u & 1 below");
    for (uint32_t t0 = 0; t0 < T; t0 += kWideD) {
#pragma unroll
        for (uint32_t u = 0; u < kWideD; ++u) {
            const uint32_t t = t0 + u;
            if (t >= T) break;
            // KiB t + 1 (the oldest of the kWideD loads in flight) joins the
            // ring (slot t + 1 & 1; KiB t stays in the other slot); the
            // register goes on to KiB t + 1 + kWideD
            asm volatile("s_waitcnt vmcnt(%1)" : "+v"(inflight[u]) : "n"(kWideD - 1) : "memory");
            put(t + 1, inflight[u]);
            inflight[u] = fetch(t + 1 + kWideD);
            uint64_t c0 = 0, c1 = 0;
            // the reads are issued in asm and waited for by hand: plain
            // loads the compiler merges into ds_read2_b64 (8 LDS cycles
            // against 2 for a ds_read_b64), volatile ones it waits for one
            // stripe at a time
            const uint32_t tb = (t & 1) << 10;
            uint32_t rb[4];
#pragma unroll
            for (uint32_t w = 0; w < 4; ++w) rb[w] = ringa + roff[w] + tb;
            // three stripes in flight: stripe v + 3 is issued once v is hashed
            uint64_t r01[16], r23[16], r45[16];
            u64x2 kk[16];
            sfor<kWidePipe>([&](auto V) {
                constexpr uint32_t v = decltype(V)::value;
                wide_issue<v>(rb[v & 3], sb[v & 3], r01[v], r23[v], r45[v], kk[v]);
            });
            sfor<16>([&](auto V) {
                constexpr uint32_t v = decltype(V)::value;
                constexpr uint32_t later = 15 - v < kWidePipe - 1 ? 15 - v : kWidePipe - 1;
                wide_wait<4 * later>(r01[v], r23[v], r45[v], kk[v]);
                const uint32_t r0 = (uint32_t)r01[v], r1 = (uint32_t)(r01[v] >> 32),
                               r2 = (uint32_t)r23[v], r3 = (uint32_t)(r23[v] >> 32),
                               r4 = (uint32_t)r45[v], r5 = (uint32_t)(r45[v] >> 32);
                // all-VGPR v_bitop3 selects (2.3 cycles; a v_cndmask on an
                // SGPR mask issues at 4.25)
                const uint32_t z0 = __builtin_amdgcn_bitop3_b32(upm, r1, r0, 0xCA),
                               z1 = __builtin_amdgcn_bitop3_b32(upm, r2, r1, 0xCA),
                               z2 = __builtin_amdgcn_bitop3_b32(upm, r3, r2, 0xCA),
                               z3 = __builtin_amdgcn_bitop3_b32(upm, r4, r3, 0xCA),
                               z4 = __builtin_amdgcn_bitop3_b32(upm, r5, r4, 0xCA);
                const uint32_t y0 = __builtin_amdgcn_alignbyte(z1, z0, sh);
                const uint32_t y1 = __builtin_amdgcn_alignbyte(z2, z1, sh);
                const uint32_t y2 = __builtin_amdgcn_alignbyte(z3, z2, sh);
                const uint32_t y3 = __builtin_amdgcn_alignbyte(z4, z3, sh);
                acc2(u64x2{((uint64_t)y1 << 32) | y0, ((uint64_t)y3 << 32) | y2}, kk[v].x,
                     kk[v].y, c0, c1);
                // the sums here, in stripe order: left to itself the compiler
                // defers all 32 multiplies to the end and holds every
                // stripe's words live (248 VGPRs, 46 of them saved per call)
                asm volatile("" : "+v"(c0), "+v"(c1));
                if constexpr (v + kWidePipe < 16)
                    wide_issue<v + kWidePipe>(rb[(v + kWidePipe) & 3], sb[(v + kWidePipe) & 3],
                                              r01[v + kWidePipe], r23[v + kWidePipe],
                                              r45[v + kWidePipe], kk[v + kWidePipe]);
                __builtin_amdgcn_sched_barrier(0);
            });
            const bool on = t >= tau && t - tau < nb;
            const uint64_t n0 = scramble(a0 + c0, scr0), n1 = scramble(a1 + c1, scr1);
            a0 = on ? n0 : a0;
            a1 = on ? n1 : a1;
        }
    }
    // the loads still in flight write registers the caller will reuse
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    g_u8 *p = data + hj + 16 * k;
    // the partial block (ns stripes, no scramble) and the last stripe
    const uint32_t ns = (uint32_t)(((len - 1) - (uint64_t)nb * 1024) / 64);
    {
        uint64_t c0 = 0, c1 = 0;
        g_u8 *q = p + (uint64_t)nb * 1024;
#pragma unroll
        for (uint32_t s = 0; s < 16; ++s)
            if (s < ns) acc2(gld2(q + 64 * s), sw0[s + 2 * k], sw0[s + 2 * k + 1], c0, c1);
        acc2(gld2(data + hj + len - 64 + 16 * k), csec_at(121 + 16 * k, seed),
             csec_at(129 + 16 * k, seed), c0, c1);
        a0 += c0;
        a1 += c1;
    }
    uint64_t tA = fold64(a0 ^ csec_at(11 + 16 * k, seed), a1 ^ csec_at(19 + 16 * k, seed));
    uint64_t tB = (csum_type == kXxh3_128)
                      ? fold64(a0 ^ csec_at(117 + 16 * k, seed), a1 ^ csec_at(125 + 16 * k, seed))
                      : 0;
    tA = quad_sum(tA);
    tB = quad_sum(tB);
    RowWin r;
    r.weak = 0;
    r.lo = xxh3_aval(len * P64_1 + tA);
    r.hi = (csum_type == kXxh3_128) ? xxh3_aval(~(len * P64_2) + tB) : 0;
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

// chain_match without the want_i preference, one window per lane (lanes diverge): the queued windows of
// a flush resolve their chains in parallel -- one set of directory / key /
// strong-sum round trips per flush instead of one per window, visited in
// order afterwards (chain_prefer applies want_i where a window matched)
__device__ int32_t chain_scan_lane(const RsWalkArgs &a, uint32_t sum, uint64_t lo, uint64_t hi,
                                   uint32_t klen, uint32_t &fa) {
    const uint32_t b = sum >> (32 - a.dbits);
    const uint32_t p0 = a.dir[b], p1 = a.dir[b + 1];
    for (uint32_t p = p0; p < p1; ++p) {
        const uint64_t key = a.tkey[p];
        const uint32_t s1 = (uint32_t)(key >> 32);
        if (s1 < sum) continue;
        if (s1 > sum) break;
        const int32_t i = (int32_t)~(uint32_t)key;
        const uint32_t li = ((uint32_t)i == a.count - 1 && a.remainder) ? a.remainder : a.blength;
        if (li != klen) continue;
        if (!strong_eq(a, (uint32_t)i, lo, hi)) {
            ++fa;
            continue;
        }
        return i;
    }
    return -1;
}

__device__ __forceinline__ int32_t chain_prefer(const RsWalkArgs &a, int32_t i, uint32_t sum,
                                                uint64_t lo, uint64_t hi, int32_t want) {
    if (i >= 0 && i != want && want >= 0 && (uint32_t)want < a.count && uni(a.sum1[want]) == sum &&
        uni((uint32_t)strong_eq(a, (uint32_t)want, lo, hi)))
        return want;
    return i;
}

// does a full-length block with sum1 == sum exist?  (the directory; the
// filters were tested by the caller; uniform per lane, divergent across lanes)
__device__ __forceinline__ bool probe_full(const RsWalkArgs &a, uint32_t sum) {
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

// membership-bucket words of sum (one 32-byte load: two 16-byte pieces)
__device__ __forceinline__ void bucket_load(const RsWalkArgs &a, uint32_t sum, uint4 &b0, uint4 &b1) {
    const uint4 *b = (const uint4 *)(a.bkt + (uint64_t)rs_bucket(sum, a.bbits) * kBucketWords);
    b0 = b[0];
    b1 = b[1];
}
// is sum in the loaded bucket?  (the directory walk for an overflowed one)
__device__ __forceinline__ bool bucket_has(const RsWalkArgs &a, uint32_t sum, const uint4 &b0,
                                           const uint4 &b1) {
    const uint32_t w[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    if (w[0] > kBucketSlots) return probe_full(a, sum);
    bool hit = false;
#pragma unroll
    for (uint32_t i = 0; i < kBucketSlots; ++i) hit |= (i < w[0]) & (w[1 + i] == sum);
    return hit;
}
// probe_full through the membership buckets
__device__ __forceinline__ bool probe_bucket(const RsWalkArgs &a, uint32_t sum) {
    uint4 b0, b1;
    bucket_load(a, sum, b0, b1);
    return bucket_has(a, sum, b0, b1);
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

// The speculative walk's false-alarm windows, recorded for the stitch: the
// offset of each visited window with false alarms and the walk's running
// total after it (lane 0 writes; n counts past cap on overflow)
struct FaRec {
    int64_t *off;
    uint32_t *cum;
    uint32_t cap;
    uint32_t n;
    __device__ __forceinline__ void add(uint32_t lane, int64_t h, uint64_t fa) {
        if (lane == 0 && n < cap) {
            off[n] = h;
            cum[n] = (uint32_t)fa;
        }
        ++n;
    }
};

// STEP batch [A, A + 1024): lane l's leaving bytes [A + 16 l, +16) and the
// entering bytes one block later (A is 16-aligned); bytes past dlen read 0
__device__ __forceinline__ void batch_load(const RsWalkArgs &a, uint64_t A, uint32_t lane,
                                           uint4 &wo, uint4 &wi) {
    const uint64_t c = A + 16 * (uint64_t)lane, L = a.blength;
    if (A + kBatch + L + 16 <= a.dlen) {
        wo = gl16(a.data + c);
        wi = ldu16(a.data + c + L);
        return;
    }
    wo = gl16_guard(a.data, c, a.dlen);
    uint32_t w[4];
    ld16(a.data, c + L, (uint32_t)((c + L) & 15), a.dlen, w);
    wi = make_uint4(w[0], w[1], w[2], w[3]);
}

// lane j's value, j < kRows, selected per lane by its row (rows >= nv take row 0)
__device__ __forceinline__ int64_t by_row(int64_t v, uint32_t lane, uint32_t nv) {
    const uint32_t r = lane >> 4;
    const uint32_t src = r < nv ? r : 0;
    int64_t out = (int64_t)rdl64((uint64_t)v, 0);
#pragma unroll
    for (uint32_t j = 1; j < kRows; ++j) {
        const int64_t x = (int64_t)rdl64((uint64_t)v, (int)j);
        out = (src == j) ? x : out;
    }
    return out;
}

// hash_search from (o, want) over [o, stop); full windows only below
// min(stop, full_end).  Matches go to out_off/out_idx/out_fab (lane 0
// writes); with `spec`, the walk ends at its first match the speculative walk
// also made.
//   RUN   windows o, o + L, o + 2L, o + 3L are hashed together (one per row;
//         the later ones speculatively, after a match) and visited in order.
//   STEP  batches of 1024 offsets (16 per lane) from a wave scan of the
//         rolling deltas; weak hits are queued in offset order and hashed
//         kRows at a time (rows), then visited in order.
// Only visited windows count: a speculative window the walk does not reach
// is dropped, so matches and false alarms are hash_search's.
template <uint32_t RING>
__device__ SegResult walk_segment(const RsWalkArgs &a, const RowSec &rs, const uint32_t *lfilt,
                                  uint8_t *wring, uint32_t *pscr,
                                  uint32_t lane, int64_t o, int32_t want, int64_t stop,
                                  int64_t *out_off, int32_t *out_idx, int64_t *out_fab,
                                  uint32_t cap, const SpecView *spec, WProf &wp,
                                  FaRec *rec = nullptr) {
    const int64_t fend = min(stop, (int64_t)a.full_end);
    const uint64_t L = a.blength;
    // STEP hits per flush: kWideQ (wide passes) needs windows of whole blocks
    const uint32_t fq = (a.flushq > kRows && L > 1024) ? kWideQ : kRows;
    const uint8_t *d = a.data;
    const uint32_t row = lane >> 4;
    SegResult res{0, 0xffffffffu, 0, 0, want};
    uint64_t fa = 0;
    uint32_t n = 0;
    bool run = true;
    bool ahead = false;       // RUN: speculate past the first window (after a match)
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
    while (!merged && o < fend) {
        WPROG(a, lane, 1, o, n);
        if (run) {
            // windows o + j L below fend, j < k
            const int64_t room = (fend - o + (int64_t)L - 1) / (int64_t)L;
            const uint32_t k = ahead ? (uint32_t)min<int64_t>(kRows, room) : 1u;
            const int64_t orow = o + (int64_t)L * (int64_t)(row < k ? row : 0);
            uint64_t t0 = wclock(wp);
            const RowWin w = rows_window<true, RING>(a, rs, lane, (uint64_t)orow, L);
            wadd(wp, kPrRun, t0);
            for (uint32_t j = 0; j < k; ++j) {
                const int64_t oj = o;
                const uint32_t wk = (uint32_t)__builtin_amdgcn_readlane((int)w.weak, (int)(16 * j));
                const uint64_t lo = rdl64(w.lo, (int)(16 * j)), hi = rdl64(w.hi, (int)(16 * j));
                const uint64_t fa_visit = fa;
                t0 = wclock(wp);
                const int32_t i = unis(chain_match(a, wk, lo, hi, want, (uint32_t)L, fa));
                if (rec && fa != fa_visit) rec->add(lane, oj, fa);
                wadd(wp, kPrChain, t0);
                WPROG(a, lane, 3, oj, i);
                if (i >= 0) {
                    merged = on_match(oj, i, fa_visit);
                    ahead = true;
                    if (merged || o != oj + (int64_t)L) break;   // short last block: re-plan
                    continue;
                }
                // roll the window one byte: hash_search's s1/s2 update
                const int32_t xo = sbyte(d, (uint64_t)oj);
                const int32_t xi = (oj + 1 < fend) ? sbyte(d, (uint64_t)oj + L) : 0;
                S1 = uni((wk & 0xffffu) - (uint32_t)xo + (uint32_t)xi);
                S2 = uni((wk >> 16) - (uint32_t)L * (uint32_t)xo + S1);
                o = oj + 1;
                run = false;
                break;
            }
            continue;
        }
        // ---- STEP: batches [A, A + 1024) from o; offsets below `from` are done ----
        uint64_t A = (uint64_t)o & ~15ull;
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
        uint32_t nq = 0;        // queued hits: lane j < nq holds hit j (offset, weak sum)
        int64_t qh = 0;
        uint32_t qsum = 0;
        bool matched = false;
        // The likely resync: after an edit inside block want, the walk usually
        // matches block want + 1 (or a few later), so a hit whose weak sum is
        // one of theirs is flushed at once instead of after more hits past it
        // (a.flushpredict; only when a flush runs, never what it finds)
        uint32_t pw[kPredict];
#pragma unroll
        for (uint32_t m = 0; m < kPredict; ++m) {
            const uint32_t b = (uint32_t)want + m;
            pw[m] = (a.flushpredict && want >= 0 && b < a.count) ? uni(a.sum1[b]) : 0xffffffffu;
        }
        uint4 cwo, cwi;         // the batch's leaving / entering bytes (16 per lane)
        batch_load(a, A, lane, cwo, cwi);
        // Stage 1 of a batch: its window sums, the LDS prefilter and the
        // blocked filter, and the membership-bucket load of each lane's first
        // surviving offset.  Stage 2 (probe results, queueing, flushes) of
        // batch A runs after stage 1 of batch A + 1024, so the bucket loads of
        // A are in flight behind A + 1024's sums and filter reads instead of
        // stalling the wave; a match in A drops A + 1024's stage 1.  Stage 1
        // also issues the loads of the batch after the one it tests.
        struct Stage {
            uint32_t hit;        // offsets passing both filters
            uint32_t sums[16];   // (s1 & 0xffff) | (s2 << 16) per offset
            uint32_t t1, t2;     // the sums at the next batch's first offset (uniform)
            uint32_t pt;         // the probed offset of the lane (16: none)
#if VS_WALK_PSCAN
            uint32_t base;       // spread: the lane's first survivor's rank in the batch
            uint32_t ns;         // spread: survivors in the batch (uniform; 0: each lane its own)
#endif
            uint4 b0, b1;        // its membership bucket
        };
        uint4 nwo = cwo, nwi = cwi;
        uint64_t fw[16];
        auto stage1a = [&](uint64_t Ab, const uint4 &bo, const uint4 &bi, uint32_t t1, uint32_t t2,
                          int64_t fromb, Stage &st) {
            uint64_t tb = wclock(wp);
            const uint64_t c = Ab + 16 * (uint64_t)lane;
            const uint32_t wo[4] = {bo.x, bo.y, bo.z, bo.w};
            const uint32_t wi[4] = {bi.x, bi.y, bi.z, bi.w};
            // the next batch's bytes, in flight while this one is tested
            nwo = bo;
            nwi = bi;
            if ((int64_t)(Ab + kBatch) < fend) batch_load(a, Ab + kBatch, lane, nwo, nwi);
            int Xo = 0, Xi = 0, Eo = 0, Ei = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                Xo = dot4(wo[k], 0x01010101u, Xo);
                Xi = dot4(wi[k], 0x01010101u, Xi);
                // weights 16 - t for byte t = 4k .. 4k+3
                const uint32_t wt = (uint32_t)((16 - 4 * k) | ((15 - 4 * k) << 8) |
                                               ((14 - 4 * k) << 16) | ((13 - 4 * k) << 24));
                Eo = dot4(wo[k], wt, Eo);
                Ei = dot4(wi[k], wt, Ei);
            }
            const uint32_t D = (uint32_t)(Xi - Xo), E = (uint32_t)(Ei - Eo), X = (uint32_t)Xo;
            const uint32_t P = excl_scan(D, lane);
            const uint32_t Y = excl_scan(E + 16u * P - (uint32_t)L * X, lane);
            uint32_t s1 = t1 + P;
            uint32_t s2 = t2 + 16u * lane * t1 + Y;
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                st.sums[t] = __builtin_amdgcn_perm(s2, s1, 0x05040100u);  // (s1 & 0xffff) | (s2 << 16)
                const int32_t xo = __builtin_amdgcn_sbfe((int)wo[t >> 2], 8 * (t & 3), 8);
                const int32_t xi = __builtin_amdgcn_sbfe((int)wi[t >> 2], 8 * (t & 3), 8);
                s1 += (uint32_t)(xi - xo);
                s2 = s2 - (uint32_t)L * (uint32_t)xo + s1;
            }
            // offsets c + t in [fromb, fend): bits [lo, hi) (one range per
            // lane, not a 64-bit compare pair per offset: share walk
            // 41.4 -> 40.7 ms, profiles/r05_walk/steprange)
            const int64_t lo = min<int64_t>(max<int64_t>(fromb - (int64_t)c, 0), 16);
            const int64_t hi = min<int64_t>(max<int64_t>(fend - (int64_t)c, 0), 16);
            const uint32_t valid = ((1u << (uint32_t)hi) - 1u) & ~((1u << (uint32_t)lo) - 1u);
            st.t1 = (uint32_t)__builtin_amdgcn_readlane((int)s1, 63);
            st.t2 = (uint32_t)__builtin_amdgcn_readlane((int)s2, 63);
            wadd(wp, kPrStepSums, tb);
            // membership: the LDS prefilter (top lbits of the sum), then the
            // L2-resident blocked filter for all 16 offsets at once -- offsets
            // the prefilter rejected read word 0, so their loads coalesce;
            // all 16 reads of each stage are issued before any is consumed
            uint64_t tsub = wclock(wp);
            uint32_t hit = valid;
            if (a.lbits) {
                uint32_t lw[16];
#pragma unroll
                for (int t = 0; t < 16; ++t) lw[t] = lfilt[(st.sums[t] >> (32 - a.lbits)) >> 5];
                uint32_t lh = 0;
#pragma unroll
                for (int t = 0; t < 16; ++t)
                    lh |= ((lw[t] >> ((st.sums[t] >> (32 - a.lbits)) & 31)) & 1u) << t;
                hit &= lh;
            }
            wadd(wp, kPrStepLds, tsub);
            tsub = wclock(wp);
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const bool on = (hit >> t) & 1u;
                fw[t] = a.filt_b[on ? rs_bloom_word(st.sums[t], a.fbits) : 0u];
            }
            st.hit = hit;
            wadd(wp, kPrStepGather, tsub);
        };
        // the blocked filter's words (issued by stage1a, tested by stage1b)
        auto stage1b = [&](Stage &st) {
            uint64_t tsub = wclock(wp);
            uint32_t hit = st.hit;
            {
                uint32_t pass = 0;
#pragma unroll
                for (int t = 0; t < 16; ++t) {
                    const uint64_t m = rs_bloom_mask(st.sums[t]);
                    pass |= (uint32_t)((fw[t] & m) == m) << t;
                }
                hit &= pass;
            }
            st.hit = hit;
            st.pt = hit ? (uint32_t)__builtin_ctz(hit) : 16u;
#if VS_WALK_PSCAN
            // A lane with several survivors used to probe them one dependent
            // load at a time, and the wave waited for its most crowded lane
            // (≈ 2.5 loads per batch at the real C4 density, 7.3 K cycles:
            // profiles/r05_walk/flushspan).  When some lane has more than one,
            // the batch's survivors are spread a lane each instead: survivor
            // r (offset order) goes to pscr[r], lane r loads its bucket, and
            // every probe is one round trip in flight behind the next batch's
            // stage 1.  pt then carries lane j's survivor sum.
            st.ns = 0;
            if (__ballot(hit & (hit - 1u))) {
                const uint32_t pc = (uint32_t)__builtin_popcount(hit);
                st.base = excl_scan(pc, lane);
                st.ns = uni((uint32_t)__builtin_amdgcn_readlane((int)(st.base + pc), 63));
                uint32_t r = st.base;
#pragma unroll
                for (int t = 0; t < 16; ++t) {
                    if (((hit >> t) & 1u) && r < 64) pscr[r] = st.sums[t];
                    r += (hit >> t) & 1u;
                }
                // (a wave's LDS accesses complete in issue order)
                st.pt = lane < st.ns ? pscr[lane] : 0u;
                if (lane < st.ns) bucket_load(a, st.pt, st.b0, st.b1);
            } else
#endif
            if (hit) {
                uint32_t sv = st.sums[0];
#pragma unroll
                for (uint32_t k = 1; k < 16; ++k) sv = (st.pt == k) ? st.sums[k] : sv;
                bucket_load(a, sv, st.b0, st.b1);
            }
            wadd(wp, kPrStepGather, tsub);
        };
        Stage cur, nxt;
        stage1a(A, cwo, cwi, T1, T2, o, cur);
        stage1b(cur);
        for (;;) {
            uint64_t tb = wclock(wp);
            const uint64_t nx = A + kBatch;
            const bool last = (int64_t)nx >= fend;
            if (!last) {
                cwo = nwo;
                cwi = nwi;
                stage1a(nx, cwo, cwi, cur.t1, cur.t2, (int64_t)nx, nxt);
#if !VS_WALK_LATEFW
                stage1b(nxt);
#endif
            }
            // stage 2 of batch A: the probe results (the preloaded bucket for
            // the lane's first offset, the rest probed now -- rare)
            uint64_t tsub = wclock(wp);
            uint32_t hit = cur.hit;
#if VS_WALK_PSCAN
            if (cur.ns) {
                const bool in = lane < cur.ns && bucket_has(a, cur.pt, cur.b0, cur.b1);
                const uint64_t res = __ballot(in);   // bit r: survivor r's sum is in the table
                uint32_t keep = 0, r = cur.base;
                for (uint32_t mm = cur.hit; mm; ++r) {
                    const int t = __builtin_ctz(mm);
                    mm &= mm - 1;
                    bool ok;
                    if (r < 64) {
                        ok = (res >> r) & 1u;
                    } else {   // past the wave's 64 survivors (rare): probed here
                        uint32_t st = cur.sums[0];
#pragma unroll
                        for (int k = 1; k < 16; ++k) st = (t == k) ? cur.sums[k] : st;
                        ok = probe_bucket(a, st);
                    }
                    keep |= (uint32_t)ok << t;
                }
                hit = keep;
            } else
#endif
            if (hit) {
                uint32_t sv = cur.sums[0];
#pragma unroll
                for (uint32_t k = 1; k < 16; ++k) sv = (cur.pt == k) ? cur.sums[k] : sv;
                if (!bucket_has(a, sv, cur.b0, cur.b1)) hit &= ~(1u << cur.pt);
                for (uint32_t mm = cur.hit & ~(1u << cur.pt); mm;) {
                    const int t = __builtin_ctz(mm);
                    mm &= mm - 1;
                    uint32_t st = cur.sums[0];
#pragma unroll
                    for (int k = 1; k < 16; ++k) st = (t == k) ? cur.sums[k] : st;
                    if (!probe_bucket(a, st)) hit &= ~(1u << t);
                }
            }
            wadd(wp, kPrStepProbe, tsub);
#if VS_WALK_LATEFW
            // batch A + 1024's filter words land behind batch A's probe results
            if (!last) stage1b(nxt);
#endif
            // queue the hits in offset order (lane order, then bit order);
            // a full queue is flushed and queueing goes on with the batch's
            // remaining hits (all past the last visited one)
            bool predicted = false;
            for (;;) {
                tsub = wclock(wp);
                uint64_t lanes = __ballot(hit != 0);
                WPROG(a, lane, 5, (int64_t)A, lanes);
                while (lanes && nq < fq) {
                    const uint32_t hl = (uint32_t)__builtin_ctzll(lanes);
                    const uint32_t hm = (uint32_t)__builtin_amdgcn_readlane((int)hit, (int)hl);
                    const uint32_t t = (uint32_t)__builtin_ctz(hm);
                    uint32_t st = cur.sums[0];
#pragma unroll
                    for (uint32_t k = 1; k < 16; ++k) st = (t == k) ? cur.sums[k] : st;
                    const uint32_t sv = (uint32_t)__builtin_amdgcn_readlane((int)st, (int)hl);
                    const int64_t h = (int64_t)A + 16 * (int64_t)hl + t;
                    if (lane == nq) {
                        qh = h;
                        qsum = sv;
                    }
                    ++nq;
                    if (lane == hl) hit &= hit - 1;
                    lanes = __ballot(hit != 0);
                    bool likely = false;
#pragma unroll
                    for (uint32_t m = 0; m < kPredict; ++m) likely |= sv == pw[m];
                    if (likely) {
                        predicted = true;
                        break;
                    }
                }
                wadd(wp, kPrStepQueue, tsub);
                const bool more = lanes != 0;              // hits of this batch not yet queued
                // flush: a full queue, the scan's end, or (a.flushspan) the
                // scan ran that far past the first queued hit
                const bool span = a.flushspan && nq &&
                                  (int64_t)(A + kBatch) - (int64_t)rdl64((uint64_t)qh, 0) >=
                                      (int64_t)a.flushspan;
                if (!(nq == fq || (!more && last && nq) || span || predicted)) break;
                predicted = false;
                // hash the queued windows together, visit them in order: more
                // than kRows in one address-lockstep pass, else one per row
                const bool wide = fq == kWideQ && nq > kRows;   // (wide for every flush: no faster)
                uint64_t tf = wclock(wp);
#ifdef VS_WALK_PROF
                if (wp.on && wide) {   // the pass's iterations (KiB of span + blocks) and windows
                    const int64_t s0 = (int64_t)rdl64((uint64_t)qh, 0), s1 = (int64_t)rdl64((uint64_t)qh, (int)(nq - 1));
                    wp.cyc[kPrFlushIters] += (uint64_t)((s1 - s0) >> 10) + (L - 1) / 1024;
                    wp.cnt[kPrFlushIters] += 1;
                    wp.cyc[kPrFlushWin] += nq;
                    wp.cnt[kPrFlushWin] += 1;
                }
#endif
                RowWin w;
                if (wide) {
                    w = wide_windows((g_u8 *)(uintptr_t)a.data, a.dlen, (l_u64 *)rs.w,
                                     (l_u8 *)wring + (threadIdx.x >> 6) * kWideRingBytes,
                                     a.seed, a.csum_type, lane, qh, nq, L);
                } else {
                    const int64_t orow = by_row(qh, lane, nq);
                    // (two blocks in flight here: the next batch's stage 1 is live)
                    w = rows_window<false, VS_WALK_FRING>(a, rs, lane, (uint64_t)orow, L);
                }
                wadd(wp, kPrFlush, tf);
                // lane j < nq scans window j's chain (its strong sum moved
                // from lane 16 j, or 4 j after a wide pass); the visits then
                // only read the results
                tf = wclock(wp);
                const uint32_t wstride = wide ? 4u : 16u;
                const int src = (int)(wstride * (lane < nq ? lane : 0));
                const uint64_t wl = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(w.lo >> 32), src, 64) << 32) |
                                    (uint32_t)__shfl((int)(uint32_t)w.lo, src, 64);
                const uint64_t wh = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(w.hi >> 32), src, 64) << 32) |
                                    (uint32_t)__shfl((int)(uint32_t)w.hi, src, 64);
                uint32_t cfa = 0;
                const int32_t cidx = lane < nq ? chain_scan_lane(a, qsum, wl, wh, (uint32_t)L, cfa) : -1;
                wadd(wp, kPrChain, tf);
                for (uint32_t j = 0; j < nq; ++j) {
                    const int64_t h = (int64_t)rdl64((uint64_t)qh, (int)j);
                    const uint32_t sv = (uint32_t)__builtin_amdgcn_readlane((int)qsum, (int)j);
                    const uint64_t lo = rdl64(w.lo, (int)(wstride * j)), hi = rdl64(w.hi, (int)(wstride * j));
                    const uint64_t fa_visit = fa;
                    WPROG(a, lane, 6, h, j);
                    fa += (uint32_t)__builtin_amdgcn_readlane((int)cfa, (int)j);
                    if (rec && fa != fa_visit) rec->add(lane, h, fa);
                    const int32_t ci = __builtin_amdgcn_readlane(cidx, (int)j);
                    const int32_t i = ci >= 0 ? unis(chain_prefer(a, ci, sv, lo, hi, want)) : -1;
                    if (i >= 0) {
                        merged = on_match(h, i, fa_visit);
                        matched = true;
                        break;
                    }
                }
                nq = 0;
                if (matched || !more) break;
            }
            wadd(wp, kPrStep, tb);
            if (matched) break;
            if (last) {
                o = fend;
                break;
            }
            A = nx;
            cur = nxt;
        }
        if (matched) {
            run = true;
            ahead = true;
        }
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

// segments are taken from a work counter (a.work, zeroed before each launch):
// their cost varies with the edits they hold, so dealing them statically
// leaves the grid waiting on its most loaded waves
__device__ __forceinline__ uint32_t next_segment(const RsWalkArgs &a, uint32_t lane) {
    uint32_t k = 0;
    if (lane == 0) k = atomicAdd(a.work, 1u);
    return uni(k);
}

// segments [1, nseg1) are seg_len long from segb (segment 0 runs from lo to
// segment 1), the tail's seg_len2 (handed out last)
__device__ __forceinline__ int64_t seg_lo(const RsWalkArgs &a, uint32_t k) {
    return k == 0        ? a.lo
           : k <= a.nseg1 ? a.segb + (int64_t)k * a.seg_len
                          : a.segb + (int64_t)a.nseg1 * a.seg_len + (int64_t)(k - a.nseg1) * a.seg_len2;
}
__device__ __forceinline__ int64_t seg_hi(const RsWalkArgs &a, uint32_t k) {
    return min(seg_lo(a, k + 1), a.hi);
}

// speculative walk of every segment from its own start (segment 0 from the
// range's speculative entry a.e0 / a.w0; the others with want_i "no
// preference" = count)
template <uint32_t T, uint32_t RING>
__global__ __launch_bounds__(T) void rs_walk_spec_kernel(RsWalkArgs a) {
    __shared__ uint32_t lfilt[kLdsFiltWordsW];
    __shared__ __attribute__((aligned(16))) uint64_t lsec[kSecWords];
    __shared__ __attribute__((aligned(16))) uint8_t wring[kWideRingBytes * (kWalkThreads / 64) + 16];
    __shared__ uint32_t pscr[kWalkThreads / 64][64];   // per wave: a STEP batch's survivors' sums
    load_secret(lsec, a.seed);
    load_prefilter(a, lfilt);
    const uint32_t lane = threadIdx.x & 63;
    const RowSec rs{lsec};
    WPROF_INIT(a.prof != nullptr);
    for (uint32_t k = next_segment(a, lane); k < a.nseg; k = next_segment(a, lane)) {
        WPROG(a, lane, 11, k, a.nseg);
        const uint64_t ts = wclock(wp);
        const int64_t e = (int64_t)uni64((uint64_t)(k ? seg_lo(a, k) : a.e0));
        const int32_t w = unis(k ? (int32_t)a.count : a.w0);
        const uint64_t base = (uint64_t)k * a.cap;
        FaRec rec{a.spec_fao + (uint64_t)k * a.facap, a.spec_fac + (uint64_t)k * a.facap,
                  a.facap, 0};
        const SegResult r = walk_segment<RING>(a, rs, lfilt, wring, pscr[threadIdx.x >> 6], lane, e, w, seg_hi(a, k),
                                               a.spec_off + base, a.spec_idx + base,
                                               a.spec_fab + base, a.cap, nullptr, wp, &rec);
        wadd(wp, kPrSeg, ts);
        if (lane == 0) {
            a.spec_nfa[k] = rec.n;
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
    if (wp.on && lane == 0) {
        uint64_t *pr = a.prof + (uint64_t)(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) * 2 * kPrN;
        for (int i = 0; i < kPrN; ++i) {
            pr[i] = wp.cyc[i];
            pr[kPrN + i] = wp.cnt[i];
        }
    }
    WPROG(a, lane, 12, 0, 0);
}

// the speculative walk of segment k's false alarms in windows below offset x
// (its recorded running totals; the caller checked they did not overflow)
__device__ __forceinline__ uint64_t fa_before(const RsWalkArgs &a, uint32_t k, int64_t x) {
    const int64_t *off = a.spec_fao + (uint64_t)k * a.facap;
    const uint32_t *cum = a.spec_fac + (uint64_t)k * a.facap;
    uint32_t lo = 0, hi = uni(a.spec_nfa[k]);
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((int64_t)uni64((uint64_t)off[mid]) < x) lo = mid + 1;
        else hi = mid;
    }
    return lo ? (uint64_t)uni(cum[lo - 1]) : 0ull;
}

// A re-walk from (e, w) that the speculative walk of segment k already
// visited: hash_search's state is (offset, want_i), and the speculative walk
// visits every offset of [its entry, its exit) outside its matches' blocks.
// Same state at e: the walks agree from e on, so the final walk is the
// speculative one from its first match at or after e, with the false alarms
// of its windows from e on -- no re-walk.  Another want_i: they visit the
// same offsets until that match (false alarms do not depend on want_i; only
// the choice among equal blocks does), so r.from = 0xfffffffe asks the caller
// to re-walk from it (r.n = its index).  False: no shortcut applies.
__device__ __forceinline__ bool stitch_visited(const RsWalkArgs &a, uint32_t k, const SpecView &sv,
                                               int64_t e, int32_t w, SegResult &r) {
    const uint32_t nfa = uni(a.spec_nfa[k]);
    const int64_t fend = min(seg_hi(a, k), (int64_t)a.full_end);
    if (nfa > a.facap || e < seg_lo(a, k) || e >= fend || e >= sv.exit_off) return false;
    uint32_t lo = 0, hi = sv.n;   // first speculative match at or after e
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((int64_t)uni64((uint64_t)sv.off[mid]) < e) lo = mid + 1;
        else hi = mid;
    }
    int32_t wsp = k ? (int32_t)a.count : a.spec_w0;
    if (lo) {
        const int32_t pi = unis(sv.idx[lo - 1]);
        const int64_t pend = (int64_t)uni64((uint64_t)sv.off[lo - 1]) +
                             (((uint32_t)pi == a.count - 1 && a.remainder) ? a.remainder : a.blength);
        if (e < pend) return false;   // inside a speculative match's block
        wsp = pi + 1;
    }
    if (w == wsp || lo == sv.n) {
        r = SegResult{0, lo, sv.fa - fa_before(a, k, e), sv.exit_off, lo == sv.n ? w : sv.exit_want};
    } else {
        r = SegResult{lo, 0xfffffffeu, 0, 0, w};
    }
    return true;
}

// one stitch pass: a segment whose entry (the previous segment's exit from
// the last pass, or a.e0 / a.w0) differs from the entry of its current walk
// re-walks from it, merging into its speculative walk
__global__ __launch_bounds__(kWalkThreads) void rs_walk_stitch_kernel(RsWalkArgs a) {
    __shared__ uint32_t lfilt[kLdsFiltWordsW];
    __shared__ __attribute__((aligned(16))) uint64_t lsec[kSecWords];
    __shared__ __attribute__((aligned(16))) uint8_t wring[kWideRingBytes * (kWalkThreads / 64) + 16];
    __shared__ uint32_t pscr[kWalkThreads / 64][64];   // per wave: a STEP batch's survivors' sums
    load_secret(lsec, a.seed);
    load_prefilter(a, lfilt);
    const uint32_t lane = threadIdx.x & 63;
    const RowSec rs{lsec};
    WPROF_INIT(false);
    for (uint32_t k = next_segment(a, lane); k < a.nseg; k = next_segment(a, lane)) {
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
        int64_t ws = e;     // where the re-walk starts
        uint64_t fadj = 0;  // false alarms of [e, ws)
        bool walk = true;
        if (stitch_visited(a, k, sv, e, w, r)) {
            walk = r.from == 0xfffffffeu;
            if (walk) {
                // the speculative walk visited e with another want_i: both
                // visit the same offsets up to its next match, where want_i
                // may choose another of equal blocks -- re-walk from there
                ws = (int64_t)uni64((uint64_t)sv.off[r.n]);
                fadj = fa_before(a, k, ws) - fa_before(a, k, e);
            }
        }
        if (walk) {
            r = walk_segment<kWalkRing>(a, rs, lfilt, wring, pscr[threadIdx.x >> 6], lane, ws, w, seg_hi(a, k), a.fin_off + base,
                                    a.fin_idx + base, a.fin_fab + base, a.cap, &sv, wp);
            r.fa += fadj;
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

// sum2 (count x s2length bytes) -> 16 zero-padded bytes per block; with
// sum1_in, also the handle's copy of sum1 (a kernel, not a runtime copy: in a
// PyTorch process hipMemcpyAsync is a blit kernel, and that one measured 12 ms
// for 2 MiB beside the whole-file checksum's SDMA read-back)
__global__ void rs_pad_sum2_kernel(const uint8_t *sum2, uint32_t count, uint32_t s2length,
                                   uint64_t *out, const uint32_t *sum1_in, uint32_t *sum1_out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    if (sum1_in) sum1_out[i] = sum1_in[i];
    uint64_t v[2] = {0, 0};
    for (uint32_t j = 0; j < s2length; ++j)
        v[j >> 3] |= (uint64_t)sum2[(uint64_t)i * s2length + j] << (8 * (j & 7));
    out[2 * (uint64_t)i] = v[0];
    out[2 * (uint64_t)i + 1] = v[1];
}

}  // namespace

int rs_walk_waves_per_cu() { return (int)(kWalkThreads / 64); }

hipError_t launch_rs_walk(const RsWalkArgs &a, bool stitch, int cus, hipStream_t s) {
    if (!a.nseg) return hipSuccess;
    if (a.lbits > 20) return hipErrorInvalidValue;
    // both passes: 8 waves per CU, four window blocks in flight per lane,
    // STEP batches in two stages (one rank of the real C4: 772-778 -> 840
    // GB/s with the membership buckets and without profiling state,
    // profiles/r03_walk_ring)
    const uint32_t waves = kWalkThreads / 64;
    const uint64_t grid = std::min<uint64_t>((a.nseg + waves - 1) / waves, (uint64_t)std::max(cus, 1));
    hipError_t e = hipMemsetAsync(a.work, 0, 4, s);
    if (e != hipSuccess) return e;
    // a build whose LDS prefilter array is smaller than the table's runs
    // without it (the prefilter only rejects; results are the same)
    RsWalkArgs b = a;
    if (b.lbits && ((1u << b.lbits) / 32) > kLdsFiltWordsW) b.lbits = 0;
    if (stitch)
        rs_walk_stitch_kernel<<<(uint32_t)grid, kWalkThreads, 0, s>>>(b);
    else
        rs_walk_spec_kernel<kWalkThreads, kWalkRing><<<(uint32_t)grid, kWalkThreads, 0, s>>>(b);
    return hipGetLastError();
}

// ---- the walk's match list, compacted on the device ------------------------------
// Segment k's final walk is fin[0, fin_n) then spec[fin_from, spec_n) when it
// was re-walked (fin_from != ~0), else spec[0, spec_n): its match count, then
// (after an exclusive scan) its matches at their list positions as 16-byte
// vs_match records (offset, block index, 0), and the false-alarm total.
__device__ __forceinline__ uint32_t seg_from(const RsWalkArgs &a, uint32_t k, uint32_t &nf) {
    const uint32_t ff = a.fin_from[k];
    nf = ff != 0xffffffffu ? a.fin_n[k] : 0u;
    return ff != 0xffffffffu ? ff : 0u;
}

__global__ void rs_collect_count_kernel(RsWalkArgs a, uint32_t *cnt) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.nseg) return;
    uint32_t nf;
    const uint32_t from = seg_from(a, k, nf);
    const uint32_t sn = a.spec_n[k];
    cnt[k] = nf + (sn > from ? sn - from : 0u);
}

__global__ void rs_collect_kernel(RsWalkArgs a, const uint32_t *pos, uint4 *out,
                                  unsigned long long *fa_total) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long fa = 0;
    if (k < a.nseg) {
        uint32_t nf;
        const uint32_t from = seg_from(a, k, nf);
        const uint64_t b = (uint64_t)k * a.cap;
        uint4 *o = out + pos[k];
        for (uint32_t j = 0; j < nf; ++j) {
            const uint64_t off = (uint64_t)a.fin_off[b + j];
            *o++ = make_uint4((uint32_t)off, (uint32_t)(off >> 32), (uint32_t)a.fin_idx[b + j], 0u);
        }
        for (uint32_t j = from; j < a.spec_n[k]; ++j) {
            const uint64_t off = (uint64_t)a.spec_off[b + j];
            *o++ = make_uint4((uint32_t)off, (uint32_t)(off >> 32), (uint32_t)a.spec_idx[b + j], 0u);
        }
        fa = a.fin_fa[k];
    }
    // one 64-bit atomic per wave
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) fa += __shfl_xor(fa, d, 64);
    if ((threadIdx.x & 63) == 0 && fa) atomicAdd(fa_total, fa);
}

hipError_t launch_rs_collect(const RsWalkArgs &a, uint32_t *cnt, uint32_t *pos, uint32_t *partials,
                             uint4 *out, unsigned long long *fa_total, hipStream_t s) {
    hipError_t e = hipMemsetAsync(fa_total, 0, 8, s);
    if (e != hipSuccess || !a.nseg) return e;
    const uint32_t blocks = (a.nseg + 255) / 256;
    rs_collect_count_kernel<<<blocks, 256, 0, s>>>(a, cnt);
    // pos[0, nseg] exclusive; pos[nseg] = the list length
    e = launch_scan_u32(cnt, pos, a.nseg, partials, 0xffffffffu, s);
    if (e != hipSuccess) return e;
    rs_collect_kernel<<<blocks, 256, 0, s>>>(a, pos, out, fa_total);
    return hipGetLastError();
}

hipError_t launch_rs_pad_sum2(const uint8_t *sum2, uint32_t count, uint32_t s2length,
                              uint64_t *out, hipStream_t s, const uint32_t *sum1_in,
                              uint32_t *sum1_out) {
    if (!count) return hipSuccess;
    rs_pad_sum2_kernel<<<(count + 255) / 256, 256, 0, s>>>(sum2, count, s2length, out, sum1_in,
                                                            sum1_out);
    return hipGetLastError();
}

}  // namespace vsgpu
