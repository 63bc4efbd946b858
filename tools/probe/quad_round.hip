// Cycles per latency-mode (quad) SHA-256 round on one gfx950 SIMD for the
// round forms tried in round 6 (profiles/r06_quad): 0 the select form
// (sha256.hip compress_quad, shared-CU tiles), 1 one DPP add with an asm
// tail, 2 the eight-round asm groups (compress_quad_iso, isolated tiles), 3
// and 4 reorderings of 2.  The consumer loop alone, K + W from LDS as in the
// kernel, no producer.
// s_memtime (shader clock) and s_memrealtime (100 MHz) bracket the loop, so
// the output gives cycles per round and the clock it ran at.  Waves per SIMD
// 1 or 2 tells latency-bound (2 waves take no longer) from issue-bound.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/qr tools/probe/quad_round.hip && /tmp/qr
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return a ^ b ^ c; }
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) { return (e & f) ^ (~e & g); }
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
struct QL { uint32_t s1, s2, s3, m; bool l1; };

#define R0(cur, p1, p2, p3, z, kwn)                                                          \
    {                                                                                        \
        const uint32_t s_ = xor3(__builtin_amdgcn_alignbit(cur, cur, ql.s1),                \
                                 __builtin_amdgcn_alignbit(cur, cur, ql.s2),                 \
                                 __builtin_amdgcn_alignbit(cur, cur, ql.s3));                \
        const uint32_t x_ = __builtin_amdgcn_bitop3_b32(cur, p1, ql.m, 0xD2);               \
        const uint32_t c_ = ch(x_, p1, p2);                                                  \
        const uint32_t t_ = s_ + c_ + z;                                                     \
        const uint32_t a_ = ql.l1 ? p3 : t_;                                                 \
        z = dpp_u32<0xA8>(p2) + (kwn);                                                       \
        p3 = dpp_u32<0xB1>(a_) + t_;                                                         \
    }
#define R1(cur, p1, p2, p3, z, kwn)                                                          \
    {                                                                                        \
        const uint32_t s_ = xor3(__builtin_amdgcn_alignbit(cur, cur, ql.s1),                \
                                 __builtin_amdgcn_alignbit(cur, cur, ql.s2),                 \
                                 __builtin_amdgcn_alignbit(cur, cur, ql.s3));                \
        const uint32_t x_ = __builtin_amdgcn_bitop3_b32(cur, p1, ql.m, 0xD2);               \
        const uint32_t c_ = ch(x_, p1, p2);                                                  \
        const uint32_t t_ = s_ + c_ + z;                                                     \
        uint32_t y_;                                                                         \
        asm("v_xad_u32 %[y], %[p], %[m], %[k]\n\t"                                            \
            "v_add_u32_dpp %[z], %[p], %[y] quad_perm:[1,2,2,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t" \
            "v_add_u32_dpp %[n], %[t], %[t] quad_perm:[2,0,2,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" \
            : [z] "=&v"(z), [n] "=&v"(p3), [y] "=&v"(y_)                                     \
            : [p] "v"(p2), [m] "v"(ql.m), [k] "v"(kwn), [t] "v"(t_));                       \
    }
#define QA(cur, p1, p2, p3, k)                                                              \
    "v_alignbit_b32 %[r1], %[" #cur "], %[" #cur "], %[s1]\n\t"                              \
    "v_alignbit_b32 %[r2], %[" #cur "], %[" #cur "], %[s2]\n\t"                              \
    "v_alignbit_b32 %[r3], %[" #cur "], %[" #cur "], %[s3]\n\t"                              \
    "v_bitop3_b32 %[xx], %[" #cur "], %[" #p1 "], %[m] bitop3:0xd2\n\t"                      \
    "v_bitop3_b32 %[r1], %[r1], %[r2], %[r3] bitop3:0x96\n\t"                                \
    "v_bitop3_b32 %[xx], %[xx], %[" #p1 "], %[" #p2 "] bitop3:0xca\n\t"                      \
    "v_add3_u32 %[tt], %[r1], %[xx], %[z]\n\t"                                               \
    "v_xad_u32 %[yy], %[" #p2 "], %[m], %[" #k "]\n\t"                                        \
    "v_add_u32_dpp %[z], %[" #p2 "], %[yy] quad_perm:[1,2,2,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t" \
    "v_add_u32_dpp %[" #p3 "], %[tt], %[tt] quad_perm:[2,0,2,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
#define Q8(pre, A, B)                                                                        \
    {                                                                                        \
        uint32_t r1, r2, r3, xx, tt, yy;                                                     \
        asm(pre QA(x0, x1, x2, x3, k0) QA(x3, x0, x1, x2, k1) QA(x2, x3, x0, x1, k2)           \
                QA(x1, x2, x3, x0, k3) QA(x0, x1, x2, x3, k4) QA(x3, x0, x1, x2, k5)           \
                    QA(x2, x3, x0, x1, k6) QA(x1, x2, x3, x0, k7)                             \
            : [x0] "+v"(x0), [x1] "+v"(x1), [x2] "+v"(x2), [x3] "+v"(x3), [z] "+v"(z),       \
              [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3), [xx] "=&v"(xx), [tt] "=&v"(tt), \
              [yy] "=&v"(yy)                                                                 \
            : [k0] "v"(A.x), [k1] "v"(A.y), [k2] "v"(A.z), [k3] "v"(A.w), [k4] "v"(B.x),      \
              [k5] "v"(B.y), [k6] "v"(B.z), [k7] "v"(B.w), [m] "v"(ql.m), [s1] "v"(ql.s1),   \
              [s2] "v"(ql.s2), [s3] "v"(ql.s3));                                             \
    }


// F3: v_xad first (r1 no longer adjacent to the previous round's DPP add)
#define QB(cur, p1, p2, p3, k, zr, zw)                                                      \
    "v_xad_u32 %[yy], %[" #p2 "], %[m], %[" #k "]\n\t"                                      \
    "v_alignbit_b32 %[r1], %[" #cur "], %[" #cur "], %[s1]\n\t"                            \
    "v_alignbit_b32 %[r2], %[" #cur "], %[" #cur "], %[s2]\n\t"                            \
    "v_alignbit_b32 %[r3], %[" #cur "], %[" #cur "], %[s3]\n\t"                            \
    "v_bitop3_b32 %[xx], %[" #cur "], %[" #p1 "], %[m] bitop3:0xd2\n\t"                    \
    "v_bitop3_b32 %[r1], %[r1], %[r2], %[r3] bitop3:0x96\n\t"                              \
    "v_bitop3_b32 %[xx], %[xx], %[" #p1 "], %[" #p2 "] bitop3:0xca\n\t"                    \
    "v_add3_u32 %[tt], %[r1], %[xx], %[" #zr "]\n\t"                                        \
    "v_add_u32_dpp %[" #zw "], %[" #p2 "], %[yy] quad_perm:[1,2,2,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t" \
    "s_nop 0\n\t"                                                                            \
    "v_add_u32_dpp %[" #p3 "], %[tt], %[tt] quad_perm:[2,0,2,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
// F4: two z registers, no dependent pair adjacent
#define QC(cur, p1, p2, p3, k, zr, zw)                                                      \
    "v_xad_u32 %[yy], %[" #p2 "], %[m], %[" #k "]\n\t"                                      \
    "v_alignbit_b32 %[r1], %[" #cur "], %[" #cur "], %[s1]\n\t"                            \
    "v_alignbit_b32 %[r2], %[" #cur "], %[" #cur "], %[s2]\n\t"                            \
    "v_bitop3_b32 %[xx], %[" #cur "], %[" #p1 "], %[m] bitop3:0xd2\n\t"                    \
    "v_alignbit_b32 %[r3], %[" #cur "], %[" #cur "], %[s3]\n\t"                            \
    "v_bitop3_b32 %[xx], %[xx], %[" #p1 "], %[" #p2 "] bitop3:0xca\n\t"                    \
    "v_bitop3_b32 %[r1], %[r1], %[r2], %[r3] bitop3:0x96\n\t"                              \
    "v_add_u32_dpp %[" #zw "], %[" #p2 "], %[yy] quad_perm:[1,2,2,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t" \
    "v_add3_u32 %[tt], %[r1], %[xx], %[" #zr "]\n\t"                                        \
    "s_nop 1\n\t"                                                                            \
    "v_add_u32_dpp %[" #p3 "], %[tt], %[tt] quad_perm:[2,0,2,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
#define QB1(cur, p1, p2, p3, k, zr, zw) QB(cur, p1, p2, p3, k, z, z)
#define Q8X(R, pre, A, B)                                                                    \
    {                                                                                        \
        uint32_t r1, r2, r3, xx, tt, yy;                                                     \
        asm(pre R(x0, x1, x2, x3, k0, z, z2) R(x3, x0, x1, x2, k1, z2, z) R(x2, x3, x0, x1, k2, z, z2) \
                R(x1, x2, x3, x0, k3, z2, z) R(x0, x1, x2, x3, k4, z, z2) R(x3, x0, x1, x2, k5, z2, z) \
                    R(x2, x3, x0, x1, k6, z, z2) R(x1, x2, x3, x0, k7, z2, z)                 \
            : [x0] "+v"(x0), [x1] "+v"(x1), [x2] "+v"(x2), [x3] "+v"(x3), [z] "+v"(z),       \
              [z2] "+v"(z2), [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3), [xx] "=&v"(xx),  \
              [tt] "=&v"(tt), [yy] "=&v"(yy)                                                 \
            : [k0] "v"(A.x), [k1] "v"(A.y), [k2] "v"(A.z), [k3] "v"(A.w), [k4] "v"(B.x),      \
              [k5] "v"(B.y), [k6] "v"(B.z), [k7] "v"(B.w), [m] "v"(ql.m), [s1] "v"(ql.s1),   \
              [s2] "v"(ql.s2), [s3] "v"(ql.s3));                                             \
    }

template <int FORM>
__device__ __forceinline__ void block(uint32_t (&x)[4], const uint4 *kw, const QL &ql) {
    uint32_t x0 = x[0], x1 = x[1], x2 = x[2], x3 = x[3];
    if constexpr (FORM >= 3) {
        // F3 single z (QB writes back the z it read: zr == zw), F4 two z registers
        uint32_t z = dpp_u32<0xA9>(x3) + ((x3 ^ ql.m) + kw[15 * 16].w), z2 = 0;
        uint4 a = kw[0], b = kw[16];
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            uint4 na = a, nb = b;
            if (g < 7) {
                na = kw[(2 * g + 2) * 16];
                nb = kw[(2 * g + 3) * 16];
            }
            if constexpr (FORM == 3) {
                if (g == 0) Q8X(QB1, "s_nop 1\n\t", a, b) else Q8X(QB1, "", a, b)
            } else {
                if (g == 0) Q8X(QC, "s_nop 1\n\t", a, b) else Q8X(QC, "", a, b)
            }
            a = na;
            b = nb;
        }
        x[0] += x0 + (z2 & 0);
    } else if constexpr (FORM == 2) {
        uint32_t z = dpp_u32<0xA9>(x3) + ((x3 ^ ql.m) + kw[15 * 16].w);
        uint4 a = kw[0], b = kw[16];
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            uint4 na = a, nb = b;
            if (g < 7) {
                na = kw[(2 * g + 2) * 16];
                nb = kw[(2 * g + 3) * 16];
            }
            if (g == 0)
                Q8("s_nop 1\n\t", a, b)
            else
                Q8("", a, b)
            a = na;
            b = nb;
        }
    } else {
        uint4 v = kw[0];
        uint32_t z = FORM == 1 ? dpp_u32<0xA9>(x3) + ((x3 ^ ql.m) + v.x) : dpp_u32<0xA8>(x3) + v.x;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const uint4 u = q < 15 ? kw[(q + 1) * 16] : make_uint4(0, 0, 0, 0);
            if constexpr (FORM == 1) {
                R1(x0, x1, x2, x3, z, v.y) R1(x3, x0, x1, x2, z, v.z) R1(x2, x3, x0, x1, z, v.w)
                R1(x1, x2, x3, x0, z, u.x)
            } else {
                R0(x0, x1, x2, x3, z, v.y) R0(x3, x0, x1, x2, z, v.z) R0(x2, x3, x0, x1, z, v.w)
                R0(x1, x2, x3, x0, z, u.x)
            }
            v = u;
        }
    }
    if constexpr (FORM < 3) x[0] += x0;
    x[1] += x1;
    x[2] += x2;
    x[3] += x3;
}

template <int FORM>
__global__ __launch_bounds__(512) void qprobe(uint32_t nblk, uint64_t *out, uint32_t *sink) {
    __shared__ uint4 lds[3 * 256];
    for (uint32_t i = threadIdx.x; i < 3 * 256; i += blockDim.x)
        lds[i] = i < 256 ? make_uint4(i * 3 + 1, i * 5 + 2, i * 7 + 3, i * 11 + 4)
                         : i < 512 ? make_uint4(0, 0, 0, 0) : make_uint4(1, 1, 1, 1);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, role = lane & 3, c = lane >> 2;
    QL ql;
    ql.s1 = role == 0 ? 6 : role == 1 ? 2 : 0;
    ql.s2 = role == 0 ? 11 : role == 1 ? 13 : 0;
    ql.s3 = role == 0 ? 25 : role == 1 ? 22 : 0;
    ql.m = role == 1 ? 0xffffffffu : 0u;
    ql.l1 = role == 1;
    const uint4 *kw = role == 0 ? &lds[c] : FORM && role == 1 ? &lds[512 + c] : &lds[256 + c];
    uint32_t x[4];
    for (int i = 0; i < 4; ++i) x[i] = role < 2 ? lane * 4 + i + 1 : 0u;
    __builtin_amdgcn_s_setprio(3);
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t j = 0; j < nblk; ++j) block<FORM>(x, kw, ql);
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    sink[blockIdx.x * blockDim.x + threadIdx.x] = x[0] ^ x[1] ^ x[2] ^ x[3];
    if (lane == 0) {
        const uint32_t w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        out[2 * w] = t1 - t0;
        out[2 * w + 1] = r1 - r0;
    }
}

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);            \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

template <int FORM>
int run(uint32_t waves, uint64_t *out, uint32_t *sink) {
    const uint32_t nblk = 4096;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(qprobe<FORM>, dim3(1), dim3(64 * waves), 0, 0, nblk, out, sink);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
    }
    uint64_t h[32];
    CK(hipMemcpy(h, out, 16 * waves, hipMemcpyDeviceToHost));
    double cyc = 0, rt = 0;
    for (uint32_t w = 0; w < waves; ++w) {
        cyc += (double)h[2 * w] / waves;
        rt += (double)h[2 * w + 1] / waves;
    }
    const double rounds = 64.0 * nblk;
    printf("{\"form\": %d, \"waves_per_wg\": %u, \"cycles_per_round\": %.2f, \"ns_per_block\": %.1f, "
           "\"clock_GHz\": %.3f}\n",
           FORM, waves, cyc / rounds, rt * 10.0 / nblk, cyc / (rt * 10.0));
    return 0;
}

int main() {
    uint64_t *out;
    uint32_t *sink;
    CK(hipMalloc(&out, 64 * 8));
    CK(hipMalloc(&sink, 8 * 64 * 4));
    // 1 wave; 4 waves (one per SIMD); 8 waves (two per SIMD)
    for (uint32_t w : {1u, 8u}) {
        if (run<0>(w, out, sink) || run<1>(w, out, sink) || run<2>(w, out, sink) || run<3>(w, out, sink) ||
            run<4>(w, out, sink))
            return 1;
    }
    return 0;
}
