// filesum.hip -- rsync's whole-file checksum on the device (SURVEY.md 8(a)
// row R7; rsync 3.2.3 checksum.c sum_init / sum_update / sum_end, which
// match.c matched() feeds with every source byte).  sum_init takes the
// negotiated xfersum with no seed for the xxhash and MD5 types (the seed only
// enters MD4's), so the digest is XXH3_128bits / XXH3_64bits / XXH64(seed 0)
// / MD5 of the whole file, written as sum_end does (LE words).
//
// XXH3 of a long input is 8 64-bit accumulators; each 1 KiB block adds the
// contributions of its 16 stripes and is then scrambled.  The contributions
// of all blocks are independent (fs_contrib_kernel: HBM-bound, 64 B out per
// KiB); the scrambles are one serial chain over the blocks per accumulator
// -- add, xor-shift, multiply, no algebra to split it -- which a host core
// runs ~20x faster than any GPU wave (a dependent op every cycle or so
// against one every 4+ cycles), so it runs there (filesum_host.cpp, fed by
// the contributions read back in pieces).  MD5, XXH64 and
// XXH3 of <= 240 bytes are serial chains with no parallel form: the host
// thread hashes the file's bytes as they are read back (filesum_host.cpp).
#include <algorithm>

#include "internal.hpp"
#include "strong.hpp"

namespace vsgpu {
namespace {

using namespace vsstrong;

__device__ __forceinline__ uint4 ldu16(const uint8_t *p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}

// C[b][8]: block b's 16 stripes accumulated (accumulator i gets word i^1 plus
// lo32 * hi32 of word i ^ secret word s + i), block-major so the host chain
// reads one 64-byte row per block.  Lane (g, m) of a wave owns block
// 16 w + g, accumulators 2m and 2m + 1: the four lanes of a block read its
// 64-byte stripes as one contiguous 64-byte access and write its row as one.
#ifndef VS_FS_LANES
#define VS_FS_LANES 16   // 4 .. 64 (A/B builds: profiles/r05_r7/contrib*)
#endif
static_assert(VS_FS_LANES >= 4 && VS_FS_LANES <= 64 && (VS_FS_LANES & (VS_FS_LANES - 1)) == 0,
              "lanes per block");
// Eight lanes per block: lane (g, m8) of a wave owns block 8 w + g and reads
// 16 bytes at 16 m8 of every 128-byte pair of stripes, so one load
// instruction covers eight blocks' whole 128-byte lines (four lanes per
// block touched 64-byte halves: the other half came in the next
// instruction); lanes m8 and m8 + 4 then add their two stripes' sums.
// 64 GiB: 13.8 -> 12.4 ms, and the walk after it 52.2 -> 50.3 ms (the clock
// the pass costs it; profiles/r05_r7/contrib8).  Sixteen lanes (shipped):
// four blocks' 256-byte runs per instruction, two rounds of sums; 12.3 ms,
// and the walk after it 45.0-45.2 ms (profiles/r05_r7/contrib16).
__global__ __launch_bounds__(256) void fs_contrib_kernel(const uint8_t *p, uint64_t nb,
                                                         uint64_t *C) {
    constexpr uint32_t LN = VS_FS_LANES, SP = LN / 4;   // lanes per block, stripes per load
    const uint32_t lane = threadIdx.x & 63, g = lane / LN, ml = lane & (LN - 1), m = ml & 3,
                   h = ml >> 2;
    // a grid-stride loop over the waves' block groups (a 128 GiB file is
    // 2^27 blocks: one wave per group would overrun the grid's size limit)
    const uint64_t nw = (nb + 64 / LN - 1) / (64 / LN);
    const uint64_t stride = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nw; w += stride) {
    const uint64_t b0 = w * (64 / LN) + g;
    const bool live = b0 < nb;
    const uint64_t b = live ? b0 : nb - 1;   // (dead lanes still take part in the sums)
    const uint8_t *q = p + b * 1024 + 16 * ml;
    uint64_t c0 = 0, c1 = 0;
#pragma unroll
    for (uint32_t i = 0; i < 16 / SP; ++i) {
        const uint32_t s = SP * i + h;
        const uint4 v = ldu16(q + 64 * SP * i);
        const uint64_t d0 = ((uint64_t)v.y << 32) | v.x, d1 = ((uint64_t)v.w << 32) | v.z;
        const uint64_t k0 = d0 ^ kSecret64[s + 2 * m], k1 = d1 ^ kSecret64[s + 2 * m + 1];
        c0 += (uint64_t)(uint32_t)k0 * (k0 >> 32) + d1;
        c1 += (uint64_t)(uint32_t)k1 * (k1 >> 32) + d0;
    }
    // + the other lanes' stripes of the block (lane ^ 4, ^ 8, ...)
#pragma unroll
    for (uint32_t o = 4; o < LN; o <<= 1) {
        c0 += ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(c0 >> 32), (int)o, 64) << 32) |
              (uint32_t)__shfl_xor((int)(uint32_t)c0, (int)o, 64);
        c1 += ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(c1 >> 32), (int)o, 64) << 32) |
              (uint32_t)__shfl_xor((int)(uint32_t)c1, (int)o, 64);
    }
    if (live && !h) {
        uint4 o;
        o.x = (uint32_t)c0;
        o.y = (uint32_t)(c0 >> 32);
        o.z = (uint32_t)c1;
        o.w = (uint32_t)(c1 >> 32);
        *(uint4 *)(C + b * 8 + 2 * m) = o;
    }
    }
}

}  // namespace

hipError_t launch_fs_contrib(const uint8_t *p, uint64_t nb, uint64_t *C, hipStream_t s) {
    if (!nb) return hipSuccess;
    const uint64_t waves = (nb + 64 / VS_FS_LANES - 1) / (64 / VS_FS_LANES);
    // one wave per block group up to 2^24 - 1 workgroups (a grid's global
    // size must stay below 2^32 threads; at 16 lanes a 128 GiB file needs
    // 2^23); the kernel strides over any rest.  (Capped at 2^20 workgroups, every wave striding, the 64 GiB
    // pass took 12.7-12.9 ms against 12.3: profiles/r05_r7/contrib_lanes.)
    const uint64_t wgs = std::min<uint64_t>((waves + 3) / 4, (1ull << 24) - 1);
    fs_contrib_kernel<<<(uint32_t)wgs, 256, 0, s>>>(p, nb, C);
    return hipGetLastError();
}

}  // namespace vsgpu
