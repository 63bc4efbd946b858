// valu_ops2.hip -- (second set) issue cost of the candidate instructions for a cheaper
// SHA-256 round and fingerprint step: 64-bit shifts as
// rotations of a duplicated word, 16-bit min3, bit reverse, the 3-operand
// integer forms the kernels use today, and the two-operand controls.  Same
// method as valu_peak.hip: 8 independent chains per lane, s_memtime /
// s_memrealtime stamps so the figure is shader cycles per wave-instruction
// per SIMD at the clock the SIMDs actually ran.
//   hipcc -O3 --offload-arch=gfx950 valu_ops.hip -o valu_ops && ./valu_ops
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int kIters = 2048;
constexpr int kCh = 8;

#define OPS(X) \
    X(0, "v_and_b32", asm volatile("v_and_b32 %0, %0, %1" : "+v"(x[i]) : "v"(y))) \
    X(1, "v_or_b32", asm volatile("v_or_b32 %0, %0, %1" : "+v"(x[i]) : "v"(y))) \
    X(2, "v_lshlrev_b32", asm volatile("v_lshlrev_b32 %0, 5, %0" : "+v"(x[i]))) \
    X(3, "v_add_u32 literal", asm volatile("v_add_u32 %0, 0x428a2f98, %0" : "+v"(x[i]))) \
    X(4, "v_sub_u32", asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y))) \
    X(5, "v_bitop3 (2 vgpr + sgpr)", asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[i]) : "v"(y), "s"(k))) \
    X(6, "v_bitop3 (2 vgpr + inline const)", asm volatile("v_bitop3_b32 %0, %0, %1, 7 bitop3:0x96" : "+v"(x[i]) : "v"(y))) \
    X(7, "v_bitop3 (2 vgpr, x,x,y)", asm volatile("v_bitop3_b32 %0, %0, %0, %1 bitop3:0xca" : "+v"(x[i]) : "v"(y))) \
    X(8, "v_alignbit (vgpr shift)", asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(x[(i + 2) & 7]))) \
    X(9, "v_lshl_add_u32", asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x[i]) : "v"(y))) \
    X(10, "v_add_lshl_u32", asm volatile("v_add_lshl_u32 %0, %0, %1, 3" : "+v"(x[i]) : "v"(y))) \
    X(11, "v_or3_b32", asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(x[(i + 2) & 7]))) \
    X(12, "v_xad_u32", asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(x[(i + 2) & 7]))) \
    X(13, "v_bfi_b32", asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(x[(i + 2) & 7]))) \
    X(14, "v_bfe_u32", asm volatile("v_bfe_u32 %0, %0, 5, 8" : "+v"(x[i]))) \
    X(15, "v_cndmask_b32", asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(y))) \
    X(16, "v_mul_lo_u32", asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y))) \
    X(17, "v_mul_hi_u32", asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y))) \
    X(18, "v_dot4_u32_u8", asm volatile("v_dot4_u32_u8 %0, %1, %2, %0" : "+v"(x[i]) : "v"(y), "v"(x[(i + 2) & 7]))) \
    X(19, "v_alignbyte_b32", asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(x[i]) : "v"(y))) \
    X(20, "mix alignbit+bitop3", asm volatile("v_alignbit_b32 %0, %0, %1, 7\n v_bitop3_b32 %1, %1, %0, %2 bitop3:0x96" : "+v"(x[i]), "+v"(z[i]) : "v"(x[(i + 2) & 7]))) \
    X(21, "mix alignbit+xor", asm volatile("v_alignbit_b32 %0, %0, %1, 7\n v_xor_b32 %1, %1, %2" : "+v"(x[i]), "+v"(z[i]) : "v"(x[(i + 2) & 7]))) \
    X(22, "mix perm+add", asm volatile("v_perm_b32 %0, %0, %1, %2\n v_add_u32 %1, %1, %2" : "+v"(x[i]), "+v"(z[i]) : "v"(x[(i + 2) & 7]))) \
    X(23, "mix xor+add", asm volatile("v_xor_b32 %0, %0, %2\n v_add_u32 %1, %1, %2" : "+v"(x[i]), "+v"(z[i]) : "v"(x[(i + 2) & 7]))) \
    X(24, "v_lshlrev_b32 vgpr amount", asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(x[i]) : "v"(y))) \
    X(25, "v_xor literal", asm volatile("v_xor_b32 %0, 0x5bd1e995, %0" : "+v"(x[i])))

constexpr int kOps = 26;

template <int OP>
__global__ __launch_bounds__(256) void spin(uint32_t *out, uint64_t *stamps, uint32_t seed) {
    uint32_t x[kCh], z[kCh];
    uint64_t q[kCh];
#pragma unroll
    for (int i = 0; i < kCh; ++i) {
        x[i] = seed * (threadIdx.x + 17 * i + 1);
        z[i] = x[i] ^ 0x5bd1e995u;
        q[i] = ((uint64_t)z[i] << 32) | x[i];
    }
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
            for (int i = 0; i < kCh; ++i) {
                const uint32_t y = x[(i + 1) & 7];
                const uint32_t k = seed | 1;
                (void)k;
#define X(N, NAME, STMT) \
    if (OP == N) STMT;
                OPS(X)
#undef X
                (void)y;
            }
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < kCh; ++i) acc ^= x[i] ^ z[i] ^ (uint32_t)q[i] ^ (uint32_t)(q[i] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) {
        uint64_t *s = stamps + 4 * ((uint64_t)blockIdx.x * 4 + threadIdx.x / 64);
        s[0] = c1 - c0;
        s[1] = r1 - r0;
    }
}

template <int OP>
double run(int cus, int wps, uint32_t *out, uint64_t *stamps, double *ghz) {
    const int grid = cus * wps;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    spin<OP><<<grid, 256>>>(out, stamps, 3);
    hipEventRecord(a);
    spin<OP><<<grid, 256>>>(out, stamps, 5);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const int waves = grid * 4;
    std::vector<uint64_t> st((size_t)waves * 4);
    hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> clk;
    for (int w = 0; w < waves; ++w)
        if (st[4 * w + 1]) clk.push_back((double)st[4 * w] / (double)st[4 * w + 1] * 0.1);
    std::sort(clk.begin(), clk.end());
    *ghz = clk.empty() ? 0 : clk[clk.size() / 2];
    // instructions per chain step (the 64-bit add pair is two)
    const double per = (OP >= 20 && OP <= 23) ? 2.0 : 1.0;
    const double wave_instr = (double)waves * kIters * 4 * kCh * per;
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ms * 1e-3 * (*ghz) * 1e9 * cus * 4 / wave_instr;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *out;
    uint64_t *stamps;
    hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
    hipMalloc(&stamps, (size_t)cus * 8 * 4 * 4 * 8);
    const char *names[kOps];
#define X(N, NAME, STMT) names[N] = NAME;
    OPS(X)
#undef X
    printf("{\"cus\": %d, \"unit\": \"shader cycles per wave-instruction per SIMD\", \"ops\": {", cus);
    for (int op = 0; op < kOps; ++op) {
        printf("%s\n \"%s\": {", op ? "," : "", names[op]);
        int first = 1;
        for (int w = 2; w <= 8; w *= 2) {
            double ghz = 0, c = 0;
            switch (op) {
#define X(N, NAME, STMT) \
    case N: c = run<N>(cus, w, out, stamps, &ghz); break;
                OPS(X)
#undef X
            }
            printf("%s\"%d\": [%.2f, %.3f]", first ? "" : ", ", w, c, ghz);
            first = 0;
        }
        printf("}");
        fflush(stdout);
    }
    printf("}}\n");
    hipFree(out);
    hipFree(stamps);
    return 0;
}
