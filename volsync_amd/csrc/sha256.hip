// sha256.hip -- batched SHA-256 blob IDs on gfx950.
//
// restic's blob ID is sha256.Sum256 of the chunk plaintext
// (restic v0.13.1 internal/restic/id.go Hash, Go crypto/sha256 after
// /root/reference/mover-restic/patch-sources.sh:16-27), computed for every
// chunk in Repository.SaveBlob.
//
// One lane per blob: the Merkle-Damgard chain of a blob is sequential, so
// parallelism is across blobs.  Lanes are fed longest-first (64 KiB buckets)
// so a wave's lanes finish together.  Integer-VALU bound:
// per 64-byte block 64 rounds x 14 ops + 48 schedule words x 10 ops with
// v_bitop3_b32 for Ch / Maj / the three-way XORs, v_alignbit_b32 for
// rotates and v_perm_b32 for the big-endian, byte-misaligned message words.
#include <algorithm>

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

__device__ __forceinline__ void compress(uint32_t st[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wt = w[t & 15] = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
        }
        const uint32_t t1 = h + xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)) + ch(e, f, g) +
                            kK256[t] + wt;
        const uint32_t t2 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)) + maj(a, b, c);
        h = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + t2;
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

// Work-queue SHA-256.  A fixed grid of lanes pulls blobs
// longest-first from a global counter; every loop iteration each busy lane
// compresses exactly one 64-byte block -- a data block, or one of the one or
// two padding blocks it builds from the blob's tail -- so a wave stays full
// until the queue drains and only the fetch / padding build diverge.  Waves
// whose blobs have the most blocks left raise their issue priority, so the
// longest blobs (the latency tail) run at the single-wave issue rate while
// co-resident waves fill the SIMD's remaining issue slots.
__device__ __forceinline__ uint64_t blob_len(const ShaArgs &a, uint64_t i, uint64_t start) {
    return a.ends ? ((a.ends[i] & kPosMask) - start + 1) : a.lens[i];
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}

// The next block's words are loaded while the current block is compressed
// (one wave per SIMD in a latency tail has nothing else to hide the load).
__device__ __forceinline__ void load_words(uint32_t (&d)[17], const uint32_t *wp, uint32_t lim) {
    if (lim >= 64) {
        // data block: one unconditional 64-byte load (merged into 4 x dwordx4)
#pragma unroll
        for (int k = 0; k < 16; ++k) d[k] = wp[k];
        d[16] = (lim > 64) ? wp[16] : 0u;
    } else {
        // padding block (once per blob): only the words that hold tail bytes
#pragma unroll
        for (int k = 0; k < 17; ++k) d[k] = (4u * k < lim) ? wp[k] : 0u;
    }
}

// words of block j: data blocks read 64 B (+4 when misaligned); the first
// padding block reads only the words holding tail bytes (never past the blob)
__device__ __forceinline__ uint32_t block_lim(uint32_t j, uint32_t nfull, uint32_t r,
                                              uint32_t rem) {
    return (j < nfull) ? (r ? 68u : 64u) : (j == nfull ? r + rem : 0u);
}

__global__ __launch_bounds__(256, 4) void sha256_kernel(ShaArgs a) {
    bool has = false, done = false;
    uint32_t ci = 0;               // blob index
    const uint32_t *wp = nullptr;  // 4-aligned words of block b+1 (the prefetch target)
    uint32_t sel = 0;              // v_perm selector: byte misalignment r in its top byte
    uint32_t nfull = 0, b = 0, rem = 0;  // full data blocks, current block, tail bytes
    uint32_t st[8];
    uint32_t d[17];                // raw words of block b
    for (;;) {
        if (!has && !done) {
            const uint32_t t = atomicAdd(a.counter, 1u);
            if (t < a.n) {
                ci = a.order ? a.order[t] : t;
                const uint64_t start = a.starts[ci];
                const uint64_t len = blob_len(a, ci, start);
                const uint32_t r = (uint32_t)(start & 3);
                sel = (r << 24) | ((r + 1) << 16) | ((r + 2) << 8) | (r + 3);
                wp = (const uint32_t *)(a.data + (start - r));
                nfull = (uint32_t)(len >> 6);
                rem = (uint32_t)(len & 63);
                b = 0;
                load_words(d, wp, block_lim(0, nfull, r, rem));
                wp += 16;
                st[0] = 0x6a09e667; st[1] = 0xbb67ae85; st[2] = 0x3c6ef372; st[3] = 0xa54ff53a;
                st[4] = 0x510e527f; st[5] = 0x9b05688c; st[6] = 0x1f83d9ab; st[7] = 0x5be0cd19;
                has = true;
                // raise the issue priority of waves that hold the longest blobs
                const uint32_t left = wave_max_u32(min(nfull >> 13, 3u));
                const uint32_t pr = __builtin_amdgcn_readfirstlane(left);
                if (pr >= 3) __builtin_amdgcn_s_setprio(3);
                else if (pr == 2) __builtin_amdgcn_s_setprio(2);
                else if (pr == 1) __builtin_amdgcn_s_setprio(1);
                else __builtin_amdgcn_s_setprio(0);
            } else {
                done = true;
            }
        }
        if (__all(done)) break;
        if (has) {
            const uint32_t r = sel >> 24;
            uint32_t w[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) w[k] = __builtin_amdgcn_perm(d[k + 1], d[k], sel);
            if (b >= nfull) {
                // padding: [tail bytes, 0x80, zeros] (+ big-endian bit length)
                const uint32_t tl = (b == nfull) ? rem : 0u;
                const bool mark = b == nfull;
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const int v = min(max((int)tl - 4 * k, 0), 4);  // tail bytes in word k
                    const uint32_t keep = (v == 4) ? 0xffffffffu : ~(0xffffffffu >> (8 * v));
                    const uint32_t m80 =
                        (mark && v < 4 && (int)tl >= 4 * k) ? (0x80u << (24 - 8 * v)) : 0u;
                    w[k] = (w[k] & keep) | m80;
                }
                if (b > nfull || rem < 56) {
                    const uint64_t bits = ((uint64_t)nfull * 64 + rem) << 3;
                    w[14] = (uint32_t)(bits >> 32);
                    w[15] = (uint32_t)bits;
                }
            }
            load_words(d, wp, block_lim(b + 1, nfull, r, rem));  // prefetch block b+1
            wp += 16;
            compress(st, w);
            ++b;
            if (b == nfull + (rem < 56 ? 1u : 2u)) {
                uint4 *out = (uint4 *)(a.ids + 32ull * ci);
                out[0] = make_uint4(__builtin_bswap32(st[0]), __builtin_bswap32(st[1]),
                                    __builtin_bswap32(st[2]), __builtin_bswap32(st[3]));
                out[1] = make_uint4(__builtin_bswap32(st[4]), __builtin_bswap32(st[5]),
                                    __builtin_bswap32(st[6]), __builtin_bswap32(st[7]));
                has = false;
            }
        }
    }
}

// grid: one lane per blob up to two waves per SIMD (256 CUs x 4 SIMDs x 2);
// counter: a device word, zeroed here on the stream before the launch
hipError_t launch_sha256(const ShaArgs &a, hipStream_t s) {
    if (!a.n) return hipSuccess;
    hipError_t e = hipMemsetAsync(a.counter, 0, sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    const uint64_t lanes = std::min<uint64_t>(a.n, 2048ull * 64);
    sha256_kernel<<<(uint32_t)((lanes + 255) / 256), 256, 0, s>>>(a);
    return hipGetLastError();
}

// ---- longest-first ordering ---------------------------------------------------
constexpr uint32_t kLenBuckets = 4096;

__device__ __forceinline__ uint32_t len_key(uint64_t i, const uint64_t *starts,
                                            const uint64_t *ends, const uint32_t *lens) {
    const uint64_t len = ends ? ((ends[i] & kPosMask) - starts[i] + 1) : lens[i];
    const uint64_t b = len >> 16;
    return kLenBuckets - 1 - (uint32_t)(b < kLenBuckets ? b : kLenBuckets - 1);
}

__global__ void len_hist_kernel(uint64_t n, const uint64_t *starts, const uint64_t *ends,
                                const uint32_t *lens, uint32_t *hist) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&hist[len_key(i, starts, ends, lens)], 1u);
}

__global__ void len_scatter_kernel(uint64_t n, const uint64_t *starts, const uint64_t *ends,
                                   const uint32_t *lens, uint32_t *cursor, uint32_t *order) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) order[atomicAdd(&cursor[len_key(i, starts, ends, lens)], 1u)] = (uint32_t)i;
}

// hist: scratch of >= 2*kLenBuckets + 8 u32
hipError_t launch_length_order(uint64_t n, const uint64_t *starts, const uint64_t *ends,
                               const uint32_t *lens, uint32_t *hist, uint32_t *order,
                               hipStream_t s) {
    if (!n) return hipSuccess;
    uint32_t *cursor = hist + kLenBuckets;
    uint32_t *partials = cursor + kLenBuckets + 1;
    hipError_t e = hipMemsetAsync(hist, 0, kLenBuckets * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    const uint32_t blocks = (uint32_t)((n + 255) / 256);
    len_hist_kernel<<<blocks, 256, 0, s>>>(n, starts, ends, lens, hist);
    e = launch_scan_u32(hist, cursor, kLenBuckets, partials, 0xffffffffu, s);
    if (e != hipSuccess) return e;
    len_scatter_kernel<<<blocks, 256, 0, s>>>(n, starts, ends, lens, cursor, order);
    return hipGetLastError();
}

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
