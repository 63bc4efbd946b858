// select.hip -- bit-exact cut selection of restic's chunker on gfx950.
//
// Restates the min/max rule of github.com/restic/chunker@v0.4.0 chunker.go
// Next(): a chunk that starts at s ends at the first
// candidate p with p - s + 1 >= MinSize, else at s + MaxSize - 1 (forced), else
// at EOF.  The rule is sequential; it is made parallel by:
//   1. speculative walks: one lane per byte-range segment walks the rule from
//      the segment start as if a chunk started there;
//   2. boundary stitch: each segment re-walks from the true exit of its
//      predecessor until it reaches a chunk start of its own speculative path
//      (the two paths then coincide).  Passes repeat until no exit changes;
//      random data converges in one pass.
#include "internal.hpp"

namespace vsgpu {

// ---- generic exclusive scan of min(in[i], clamp) ---------------------------
constexpr int kScanThreads = 1024;
constexpr int kScanPer = 4;
constexpr int kScanTile = kScanThreads * kScanPer;

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(x, d, 64);
        if (lane >= d) x += t;
    }
    return x;
}

// exclusive block scan of one value per thread; returns the block total in *tot
__device__ uint32_t block_excl_scan(uint32_t v, uint32_t *tot) {
    __shared__ uint32_t wsum[kScanThreads / 64 + 1];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int nw = (blockDim.x + 63) >> 6;
    uint32_t inc = wave_incl_scan(v);
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    if (wid == 0) {
        uint32_t x = (lane < nw) ? wsum[lane] : 0;
        uint32_t xi = wave_incl_scan(x);
        if (lane < nw) wsum[lane] = xi - x;
        if (lane == nw - 1) wsum[kScanThreads / 64] = xi;
    }
    __syncthreads();
    uint32_t r = wsum[wid] + inc - v;
    *tot = wsum[kScanThreads / 64];
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(kScanThreads) void scan_reduce_kernel(const uint32_t *in, uint64_t n,
                                                                   uint32_t clamp,
                                                                   uint32_t *partials) {
    const uint64_t b0 = (uint64_t)blockIdx.x * kScanTile;
    uint32_t s = 0;
    for (int i = 0; i < kScanPer; ++i) {
        uint64_t k = b0 + (uint64_t)i * kScanThreads + threadIdx.x;
        if (k < n) s += min(in[k], clamp);
    }
    uint32_t tot;
    block_excl_scan(s, &tot);
    if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kScanThreads) void scan_partials_kernel(uint32_t *partials,
                                                                     uint32_t np) {
    uint32_t carry = 0;
    for (uint32_t b = 0; b < np; b += kScanThreads) {
        uint32_t i = b + threadIdx.x;
        uint32_t v = (i < np) ? partials[i] : 0;
        uint32_t tot;
        uint32_t e = block_excl_scan(v, &tot);
        if (i < np) partials[i] = carry + e;
        carry += tot;
    }
    if (threadIdx.x == 0) partials[np] = carry;
}

__global__ __launch_bounds__(kScanThreads) void scan_apply_kernel(const uint32_t *in, uint64_t n,
                                                                  uint32_t clamp,
                                                                  const uint32_t *partials,
                                                                  uint32_t np, uint32_t *out) {
    // thread t owns elements [b0 + t*kScanPer, +kScanPer) (contiguous per thread)
    const uint64_t b0 = (uint64_t)blockIdx.x * kScanTile;
    uint32_t v[kScanPer];
    uint32_t s = 0;
    for (int i = 0; i < kScanPer; ++i) {
        uint64_t k = b0 + (uint64_t)threadIdx.x * kScanPer + i;
        v[i] = (k < n) ? min(in[k], clamp) : 0;
        s += v[i];
    }
    uint32_t tot;
    uint32_t e = block_excl_scan(s, &tot) + partials[blockIdx.x];
    for (int i = 0; i < kScanPer; ++i) {
        uint64_t k = b0 + (uint64_t)threadIdx.x * kScanPer + i;
        if (k < n) out[k] = e;
        e += v[i];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = partials[np];
}

// out[0..n] = exclusive scan of min(in, clamp); out[n] = total.  partials:
// >= ceil(n / 4096) + 1 entries.
hipError_t launch_scan_u32(const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *partials,
                           uint32_t clamp, hipStream_t s) {
    const uint32_t np = (uint32_t)((n + kScanTile - 1) / kScanTile);
    if (np == 0) {
        return hipMemsetAsync(out, 0, sizeof(uint32_t), s);
    }
    scan_reduce_kernel<<<np, kScanThreads, 0, s>>>(in, n, clamp, partials);
    scan_partials_kernel<<<1, kScanThreads, 0, s>>>(partials, np);
    scan_apply_kernel<<<np, kScanThreads, 0, s>>>(in, n, clamp, partials, np, out);
    return hipGetLastError();
}

// ---- candidate compaction ----------------------------------------------------
__global__ void compact_kernel(SelArgs a, uint64_t *compact) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.nstrips) return;
    const uint32_t n = min(a.counts[k], (uint32_t)kSlots);
    const uint32_t o = a.cstart[k];
    const uint64_t sb = a.base + k * a.strip;
    for (uint32_t i = 0; i < n; ++i) compact[o + i] = sb + a.offs[k * kSlots + i];
}

hipError_t launch_compact(const SelArgs &a, uint32_t *partials, uint64_t *compact,
                          uint32_t *cstart, hipStream_t s) {
    hipError_t e = launch_scan_u32(a.counts, cstart, a.nstrips, partials, kSlots, s);
    if (e != hipSuccess) return e;
    SelArgs b = a;
    b.cstart = cstart;
    const uint32_t blocks = (uint32_t)((a.nstrips + 255) / 256);
    if (blocks) compact_kernel<<<blocks, 256, 0, s>>>(b, compact);
    return hipGetLastError();
}

// ---- the chunk rule ------------------------------------------------------------
// first candidate position >= q (data offsets), ~0 when none was recorded
__device__ uint64_t first_cand(const SelArgs &a, uint64_t q) {
    if (q >= a.scan_end) return ~0ull;
    if (q < a.base) q = a.base;
    const uint64_t k = (q - a.base) / a.strip;
    const uint64_t sb = a.base + k * a.strip;
    const uint32_t cnt = a.counts[k];
    if (cnt > (uint32_t)kSlots) {
        const uint32_t slot = a.dense_slot[k];
        if (slot == kNoSlot) {
            atomicOr(a.flags, kFlagDenseMissing);
            return ~0ull;
        }
        const uint32_t words = a.strip / 32;
        const uint32_t *bw = a.pool + (uint64_t)slot * words;
        const uint32_t r = (uint32_t)(q - sb);
        uint32_t w = r >> 5;
        uint32_t bits = bw[w] & (0xffffffffu << (r & 31));
        for (;;) {
            if (bits) return sb + 32ull * w + (uint32_t)__builtin_ctz(bits);
            if (++w >= words) break;
            bits = bw[w];
        }
    } else {
        for (uint32_t i = 0; i < cnt; ++i) {
            const uint64_t p = sb + a.offs[k * kSlots + i];
            if (p >= q) return p;
        }
    }
    if (k + 1 >= a.nstrips) return ~0ull;
    const uint32_t j = a.cstart[k + 1];
    return (j < a.cstart[a.nstrips]) ? a.compact[j] : ~0ull;
}

// 0 normal cut, 1 forced (MaxSize), 2 EOF, 3 incomplete (needs more bytes)
__device__ int next_cut(const SelArgs &a, uint64_t s, uint64_t &c) {
    const uint64_t q = s + a.min_size - 1;
    const uint64_t lim = s + a.max_size - 1;
    const uint64_t p = first_cand(a, q);
    if (p <= lim && p < a.scan_end) {
        c = p;
        return 0;
    }
    if (lim < a.scan_end) {
        c = lim;
        return 1;
    }
    if (a.final_eof) {
        c = a.dlen - 1;
        return 2;
    }
    return 3;
}

__device__ __forceinline__ void seg_bounds(const SelArgs &a, uint32_t g, uint64_t &lo,
                                           uint64_t &hi) {
    lo = a.own_lo + (uint64_t)g * a.seg_len;
    hi = min(lo + a.seg_len, a.own_hi);
}

__global__ void spec_walk_kernel(SelArgs a) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.nseg) return;
    uint64_t lo, hi;
    seg_bounds(a, g, lo, hi);
    uint64_t s = lo;
    uint32_t n = 0;
    uint64_t ex;
    for (;;) {
        if (s >= hi || s >= a.dlen) {
            ex = s;
            break;
        }
        uint64_t c;
        const int t = next_cut(a, s, c);
        if (t == 3) {
            ex = kIncomplete;
            break;
        }
        if (n < a.maxc) a.spec_cut[(uint64_t)g * a.maxc + n] = c | ((uint64_t)t << 62);
        n++;
        s = c + 1;
    }
    a.spec_n[g] = n;
    a.spec_exit[g] = ex;
}

hipError_t launch_spec_walk(const SelArgs &a, hipStream_t s) {
    if (!a.nseg) return hipSuccess;
    spec_walk_kernel<<<(a.nseg + 63) / 64, 64, 0, s>>>(a);
    return hipGetLastError();
}

__global__ void stitch_kernel(SelArgs a) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.nseg) return;
    uint64_t lo, hi;
    seg_bounds(a, g, lo, hi);
    const uint64_t entry = (g == 0) ? a.entry : a.exit_old[g - 1];
    const uint32_t ns = a.spec_n[g];
    const uint64_t *sc = a.spec_cut + (uint64_t)g * a.maxc;
    uint32_t j = 0, m = 0;
    bool merged = false, incomplete = false;
    uint64_t s = entry;
    if (entry == kIncomplete) {
        incomplete = true;
    } else {
        for (;;) {
            if (s >= hi || s >= a.dlen) break;
            // spec start m: lo, then previous spec cut + 1 (increasing)
            while (m <= ns && (m == 0 ? lo : (sc[m - 1] & kPosMask) + 1) < s) m++;
            if (m <= ns && (m == 0 ? lo : (sc[m - 1] & kPosMask) + 1) == s) {
                merged = true;
                break;
            }
            uint64_t c;
            const int t = next_cut(a, s, c);
            if (t == 3) {
                incomplete = true;
                break;
            }
            if (j < a.maxc) a.st_cut[(uint64_t)g * a.maxc + j] = c | ((uint64_t)t << 62);
            j++;
            s = c + 1;
        }
    }
    const uint64_t ex = merged ? a.spec_exit[g] : (incomplete ? kIncomplete : s);
    a.st_n[g] = j;
    a.st_merge[g] = merged ? m : ns;
    a.st_total[g] = j + (merged ? ns - m : 0);
    a.exit_new[g] = ex;
    if (ex != a.exit_old[g]) atomicOr(a.flags + 2, kFlagChanged);  // flags[2]: per-pass
}

hipError_t launch_stitch(const SelArgs &a, hipStream_t s) {
    if (!a.nseg) return hipSuccess;
    stitch_kernel<<<(a.nseg + 63) / 64, 64, 0, s>>>(a);
    return hipGetLastError();
}

__global__ void emit_kernel(SelArgs a, const uint32_t *seg_off, uint64_t *ch_start,
                            uint64_t *ch_end, uint64_t *n_out) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.nseg) return;
    const uint32_t tot = a.st_total[g];
    const uint32_t jn = a.st_n[g], mi = a.st_merge[g];
    const uint64_t *sc = a.spec_cut + (uint64_t)g * a.maxc;
    const uint64_t *tc = a.st_cut + (uint64_t)g * a.maxc;
    uint64_t prev = (g == 0) ? a.entry : a.exit_old[g - 1];
    const uint32_t o = seg_off[g];
    for (uint32_t i = 0; i < tot; ++i) {
        const uint64_t c = (i < jn) ? tc[i] : sc[mi + (i - jn)];
        ch_start[o + i] = prev;
        ch_end[o + i] = c;
        prev = (c & kPosMask) + 1;
    }
    if (g == a.nseg - 1) *n_out = (uint64_t)o + tot;
}

hipError_t launch_emit(const SelArgs &a, uint32_t *seg_off, uint64_t *ch_start,
                       uint64_t *ch_end, uint64_t *n_out, hipStream_t s) {
    if (!a.nseg) return hipMemsetAsync(n_out, 0, sizeof(uint64_t), s);
    // seg_off needs nseg+1 entries; partial scratch lives after them
    hipError_t e = launch_scan_u32(a.st_total, seg_off, a.nseg, seg_off + a.nseg + 1,
                                   0xffffffffu, s);
    if (e != hipSuccess) return e;
    emit_kernel<<<(a.nseg + 63) / 64, 64, 0, s>>>(a, seg_off, ch_start, ch_end, n_out);
    return hipGetLastError();
}

// ---- Chunk.Cut values ------------------------------------------------------------
__device__ __forceinline__ uint64_t append_byte(uint64_t d, uint32_t b, const uint64_t *mod_tab,
                                                uint32_t shift) {
    const uint32_t idx = (uint32_t)(d >> shift) & 0xff;
    return ((d << 8) | b) ^ mod_tab[idx];
}

__global__ void cut_fp_kernel(const uint8_t *data, uint64_t n, const uint64_t *ch_start,
                              const uint64_t *ch_end, uint64_t min_size,
                              const uint64_t *mod_tab, uint32_t shift, uint64_t *cut_out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t e = ch_end[i];
    const uint64_t c = e & kPosMask;
    const uint64_t s = ch_start[i];
    uint64_t h = 64;
    uint64_t d = 0;
    if ((e >> 62) == 2) {  // EOF chunk: the live digest of a chunk cut short
        const uint64_t len = c - s + 1;
        h = (len > min_size - 64) ? len - (min_size - 64) : 0;
        if (h < 64) d = 1;  // reset() slid a 1 into the window
    }
    if (h > 64) h = 64;
    for (uint64_t j = c + 1 - h; j <= c && h; ++j) d = append_byte(d, data[j], mod_tab, shift);
    cut_out[i] = d;
}

hipError_t launch_cut_fp(const uint8_t *data, uint64_t n, const uint64_t *ch_start,
                         const uint64_t *ch_end, uint64_t min_size, const uint64_t *mod_tab,
                         const uint64_t *, uint32_t idx_shift, uint64_t *cut_out,
                         hipStream_t s) {
    if (!n) return hipSuccess;
    cut_fp_kernel<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(
        data, n, ch_start, ch_end, min_size, mod_tab, idx_shift + 32, cut_out);
    return hipGetLastError();
}

}  // namespace vsgpu
