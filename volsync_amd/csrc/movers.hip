// movers.hip -- the kernels of SURVEY.md 8(f)'s adjacent rows that reuse the
// hot path's engines:
//  * fixed-size block descriptors for the batched SHA-256 engine: syncthing's
//    scanner hashes every file in blocks (lib/scanner, 128 KiB .. 16 MiB,
//    mover-syncthing/entry.sh:130-135), row (f)4;
//  * blob-ID verification on restore: restic's Repository.LoadBlob rejects a
//    blob whose SHA-256 differs from its ID (mover-restic/entry.sh:215-228),
//    row (f)4;
//  * rsync's receiver reconstruction (receiver.c receive_data): the new file
//    is literal runs and copies of basis blocks, in token order, row (f)2.
#include <algorithm>

#include "internal.hpp"

namespace vsgpu {
namespace {

__global__ void blk_desc_kernel(uint64_t len, uint32_t bs, uint64_t n, uint64_t *off,
                                uint32_t *lens) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t o = i * bs;
    off[i] = o;
    lens[i] = (uint32_t)((len - o < bs) ? len - o : bs);
}

// bad[i] = 1 when blob i's SHA-256 differs from its expected ID; count sums them
__global__ void verify_kernel(const uint8_t *got, const uint8_t *want, uint64_t n, uint32_t *bad,
                              unsigned long long *count) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool b = false;
    if (i < n) {
        const uint4 *g = (const uint4 *)(got + 32 * i), *w = (const uint4 *)(want + 32 * i);
        const uint4 g0 = g[0], g1 = g[1], w0 = w[0], w1 = w[1];
        b = (g0.x ^ w0.x) | (g0.y ^ w0.y) | (g0.z ^ w0.z) | (g0.w ^ w0.w) | (g1.x ^ w1.x) |
            (g1.y ^ w1.y) | (g1.z ^ w1.z) | (g1.w ^ w1.w);
        if (bad) bad[i] = b ? 1u : 0u;
    }
    const uint64_t m = __ballot(b);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(count, (unsigned long long)__popcll(m));
}

// one output piece per workgroup slot (grid-stride): dst[off, off + len) =
// src[soff, soff + len) from the basis (kind 0) or the literal buffer (kind 1)
__global__ __launch_bounds__(256) void recon_kernel(uint8_t *dst, const uint8_t *basis,
                                                    const uint8_t *lit, const ReconPiece *pc,
                                                    uint64_t n) {
    for (uint64_t k = blockIdx.x; k < n; k += gridDim.x) {
        const ReconPiece p = pc[k];
        const uint8_t *src = (p.kind ? lit : basis) + p.src;
        uint8_t *d = dst + p.dst;
        // bytes up to the destination's 16-byte boundary, then 16-byte pieces:
        // aligned stores, loads at whatever alignment the source has (gfx950
        // global loads need none), then the tail bytes
        const uint64_t head = std::min<uint64_t>((16 - ((uintptr_t)d & 15)) & 15, p.len);
        if (threadIdx.x < head) d[threadIdx.x] = src[threadIdx.x];
        const uint64_t n16 = (p.len - head) / 16;
        uint4 *d16 = (uint4 *)(d + head);
        const uint8_t *s16 = src + head;
        for (uint64_t i = threadIdx.x; i < n16; i += blockDim.x) {
            uint4 v;
            __builtin_memcpy(&v, s16 + 16 * i, 16);
            d16[i] = v;
        }
        for (uint64_t i = head + n16 * 16 + threadIdx.x; i < p.len; i += blockDim.x) d[i] = src[i];
    }
}

}  // namespace

hipError_t launch_blk_desc(uint64_t len, uint32_t bs, uint64_t n, uint64_t *off, uint32_t *lens,
                           hipStream_t s) {
    if (!n) return hipSuccess;
    blk_desc_kernel<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(len, bs, n, off, lens);
    return hipGetLastError();
}

hipError_t launch_verify(const uint8_t *got, const uint8_t *want, uint64_t n, uint32_t *bad,
                         unsigned long long *count, hipStream_t s) {
    hipError_t e = hipMemsetAsync(count, 0, 8, s);
    if (e != hipSuccess || !n) return e;
    verify_kernel<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(got, want, n, bad, count);
    return hipGetLastError();
}

hipError_t launch_recon(uint8_t *dst, const uint8_t *basis, const uint8_t *lit,
                        const ReconPiece *pieces, uint64_t n, int cus, hipStream_t s) {
    if (!n) return hipSuccess;
    const uint64_t grid = std::min<uint64_t>(n, (uint64_t)std::max(cus, 1) * 8);
    recon_kernel<<<(uint32_t)grid, 256, 0, s>>>(dst, basis, lit, pieces, n);
    return hipGetLastError();
}

}  // namespace vsgpu
