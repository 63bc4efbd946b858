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
// KiB), the scrambles are a serial chain over the blocks per accumulator
// (fs_chain_kernel: eight independent scalar-unit chains, one wave each),
// run piece by piece with the accumulators
// carried in device memory.  Other types and short files run the one-lane
// restatement (strong.hpp checksum2), which is serial by construction.
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
// lo32 * hi32 of word i ^ secret word s + i).  Lane (g, m) of a wave owns
// block 16 w + g, accumulators 2m and 2m + 1.
__global__ __launch_bounds__(256) void fs_contrib_kernel(const uint8_t *p, uint64_t b0,
                                                         uint64_t nb, uint64_t *C,
                                                         uint64_t stride) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, g = lane >> 2, m = lane & 3;
    const uint64_t b = (gid >> 6) * 16 + g;
    if (b >= nb) return;
    const uint8_t *q = p + (b0 + b) * 1024 + 16 * m;
    uint64_t c0 = 0, c1 = 0;
#pragma unroll
    for (uint32_t s = 0; s < 16; ++s) {
        const uint4 v = ldu16(q + 64 * s);
        const uint64_t d0 = ((uint64_t)v.y << 32) | v.x, d1 = ((uint64_t)v.w << 32) | v.z;
        const uint64_t k0 = d0 ^ kSecret64[s + 2 * m], k1 = d1 ^ kSecret64[s + 2 * m + 1];
        c0 += (uint64_t)(uint32_t)k0 * (k0 >> 32) + d1;
        c1 += (uint64_t)(uint32_t)k1 * (k1 >> 32) + d0;
    }
    // transposed: accumulator i's contributions are contiguous (Ct[i][b])
    C[(2 * m) * stride + b] = c0;
    C[(2 * m + 1) * stride + b] = c1;
}

// acc_j <- scramble(acc_j + C[j][b]) for b in [0, nb): the 8 accumulators
// are independent chains, one wave each, and the whole chain is wave-uniform,
// so it runs on the scalar unit (s_mul_i32 / s_mul_hi_u32 / s_xor / s_add,
// whose dependent issue is far shorter than a VALU round trip), with the
// contributions read through scalar loads 16 blocks ahead.
// state[0..7] = accumulators (in/out).
__global__ __launch_bounds__(64) void fs_chain_kernel(const uint64_t *__restrict__ C,
                                                      uint64_t nb, uint64_t stride,
                                                      uint64_t *state) {
    const uint32_t j = blockIdx.x;
    const uint64_t *__restrict__ cj = C + j * stride;
    const uint64_t sec = kSecret64[16 + j];
    const uint32_t slo = (uint32_t)sec, shi = (uint32_t)(sec >> 32);
    uint64_t acc = state[j];
    uint64_t b = 0;
    // scalar loads run 16 blocks ahead of the chain (double-buffered)
    uint64_t nx[16];
    if (nb >= 16) {
#pragma unroll
        for (int q = 0; q < 16; ++q) nx[q] = cj[q];
    }
    for (; b + 16 <= nb; b += 16) {
        uint64_t c[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) c[q] = nx[q];
        if (b + 32 <= nb) {
#pragma unroll
            for (int q = 0; q < 16; ++q) nx[q] = cj[b + 16 + q];
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const uint64_t u = acc + c[q];
            const uint32_t lo = (uint32_t)u ^ (uint32_t)(u >> 47) ^ slo;
            const uint32_t hi = (uint32_t)(u >> 32) ^ shi;
            acc = (uint64_t)lo * P32_1 + ((uint64_t)(hi * P32_1) << 32);
        }
    }
    for (; b < nb; ++b) {
        const uint64_t u = acc + cj[b];
        const uint32_t lo = (uint32_t)u ^ (uint32_t)(u >> 47) ^ slo;
        const uint32_t hi = (uint32_t)(u >> 32) ^ shi;
        acc = (uint64_t)lo * P32_1 + ((uint64_t)(hi * P32_1) << 32);
    }
    if (threadIdx.x == 0) state[j] = acc;
}

// the partial block, the last stripe, the merge; lanes 0..7
__global__ void fs_tail_kernel(const uint8_t *p, uint64_t len, int csum_type,
                               const uint64_t *state, uint8_t *out) {
    const uint32_t j = threadIdx.x;
    if (j >= 8) return;
    uint64_t acc = state[j];
    const uint64_t nb = (len - 1) / 1024;
    const uint32_t ns = (uint32_t)(((len - 1) - nb * 1024) / 64);
    for (uint32_t s = 0; s < ns; ++s) {
        const uint8_t *q = p + nb * 1024 + 64 * s;
        const uint64_t di = rd64(q + 8 * j), dn = rd64(q + 8 * (j ^ 1));
        const uint64_t k = di ^ kSecret64[s + j];
        acc += dn + (uint64_t)(uint32_t)k * (k >> 32);
    }
    {
        const uint8_t *q = p + len - 64;
        const uint64_t di = rd64(q + 8 * j), dn = rd64(q + 8 * (j ^ 1));
        const uint64_t k = di ^ csec_at(121 + 8 * j, 0);
        acc += dn + (uint64_t)(uint32_t)k * (k >> 32);
    }
    Xxh3Long st;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        st.acc[i] = ((uint64_t)__shfl((int)(acc >> 32), i, 8) << 32) |
                    (uint32_t)__shfl((int)(uint32_t)acc, i, 8);
    if (j == 0) {
        const uint64_t lo = st.merge(11, len * P64_1, 0);
        const uint64_t hi = (csum_type == kXxh3_128) ? st.merge(192 - 64 - 11, ~(len * P64_2), 0) : 0;
        for (int i = 0; i < 8; ++i) {
            out[i] = (uint8_t)(lo >> (8 * i));
            out[8 + i] = (uint8_t)(hi >> (8 * i));
        }
    }
}

__global__ void fs_init_kernel(uint64_t *state) {
    const uint64_t init[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
    if (threadIdx.x < 8) state[threadIdx.x] = init[threadIdx.x];
}

// the one-lane restatement (short XXH3, XXH64, MD5): serial by construction
__global__ void fs_serial_kernel(const uint8_t *p, uint64_t len, int csum_type, uint8_t *out) {
    if (threadIdx.x || blockIdx.x) return;
    uint8_t o[16];
    checksum2(p, len, csum_type, 0, o);
    for (int i = 0; i < 16; ++i) out[i] = o[i];
}

}  // namespace

size_t filesum_scratch_bytes(uint64_t len, uint64_t piece_blocks) {
    const uint64_t nb = len ? (len - 1) / 1024 : 0;
    return 256 + 64 * std::min<uint64_t>(std::max<uint64_t>(nb, 1), piece_blocks);
}

hipError_t launch_filesum(const uint8_t *p, uint64_t len, int csum_type, void *scratch,
                          uint64_t piece_blocks, uint8_t *out, hipStream_t s) {
    uint64_t *state = (uint64_t *)scratch;
    uint64_t *C = state + 32;
    const bool xxh3 = csum_type == kXxh3_128 || csum_type == kXxh3_64;
    if (!xxh3 || len <= 240) {
        fs_serial_kernel<<<1, 64, 0, s>>>(p, len, csum_type, out);
        return hipGetLastError();
    }
    fs_init_kernel<<<1, 64, 0, s>>>(state);
    const uint64_t nb = (len - 1) / 1024;
    const uint64_t stride = std::min(piece_blocks, std::max<uint64_t>(nb, 1));
    for (uint64_t b0 = 0; b0 < nb; b0 += piece_blocks) {
        const uint64_t n = std::min(piece_blocks, nb - b0);
        const uint64_t waves = (n + 15) / 16;
        fs_contrib_kernel<<<(uint32_t)((waves + 3) / 4), 256, 0, s>>>(p, b0, n, C, stride);
        fs_chain_kernel<<<8, 64, 0, s>>>(C, n, stride, state);
    }
    fs_tail_kernel<<<1, 64, 0, s>>>(p, len, csum_type, state, out);
    return hipGetLastError();
}

}  // namespace vsgpu
