// valu_ops3.hip -- (third set, round 5) issue cost of the operand forms the
// hot loops compile to (tools/isa_mix.py): SGPR operands on two-operand ops,
// v_cndmask with an SGPR pair or a freshly written VCC, v_cmp, v_pk_mov,
// v_min3 / v_and_or, and the controls of the earlier sets.  Same
// method as valu_peak.hip: 8 independent chains per lane, s_memtime /
// s_memrealtime stamps so the figure is shader cycles per wave-instruction
// per SIMD at the clock the SIMDs actually ran.
//   hipcc -O3 --offload-arch=gfx950 valu_ops3.hip -o valu_ops3 && ./valu_ops3
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int kIters = 2048;
constexpr int kCh = 8;

#define OPS(X) \
    X(0, "v_and_b32 (vgpr, sgpr)", asm volatile("v_and_b32 %0, %1, %0" : "+v"(x[i]) : "s"(k))) \
    X(1, "v_lshrrev_b32 (sgpr shift)", asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(x[i]) : "s"(k))) \
    X(2, "v_lshrrev_b32 (inline 5)", asm volatile("v_lshrrev_b32 %0, 5, %0" : "+v"(x[i]))) \
    X(3, "v_min3_u32 (3 vgpr)", asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(x[(i + 2) & 7]))) \
    X(4, "v_cndmask_b32_e64 (sgpr pair)", asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "s"(m))) \
    X(5, "v_cmp_lt_u32 + v_cndmask vcc", asm volatile("v_cmp_lt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(y) : "vcc")) \
    X(6, "v_pk_mov_b32", asm volatile("v_pk_mov_b32 %0, %1, %1 op_sel:[0,1]" : "=v"(q[i]) : "v"(q[(i + 1) & 7]))) \
    X(7, "v_not_b32", asm volatile("v_not_b32 %0, %0" : "+v"(x[i]))) \
    X(8, "v_cmp_lt_u32_e64 (sgpr dst)", asm volatile("v_cmp_lt_u32_e64 %0, %1, %2" : "=s"(mm[i & 1]) : "v"(x[i]), "v"(y))) \
    X(9, "v_bitop3 (3 vgpr, control)", asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xea" : "+v"(x[i]) : "v"(y), "v"(x[(i + 2) & 7]))) \
    X(10, "v_sub_u32_e64", asm volatile("v_sub_u32_e64 %0, %0, %1" : "+v"(x[i]) : "v"(y))) \
    X(11, "v_perm_b32 (sgpr sel)", asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "s"(k))) \
    X(12, "v_add_u32 (vgpr, sgpr)", asm volatile("v_add_u32 %0, %1, %0" : "+v"(x[i]) : "s"(k))) \
    X(13, "v_xor_b32 (vgpr, sgpr)", asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x[i]) : "s"(k))) \
    X(14, "v_alignbit (inline shift, control)", asm volatile("v_alignbit_b32 %0, %0, %1, 24" : "+v"(x[i]) : "v"(y))) \
    X(15, "v_lshlrev_b32 (inline 8, control)", asm volatile("v_lshlrev_b32 %0, 8, %0" : "+v"(x[i]))) \
    X(16, "v_min_u32 (2 vgpr)", asm volatile("v_min_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y))) \
    X(17, "v_max3_u32", asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(x[(i + 2) & 7]))) \
    X(18, "v_add3_u32 (2 vgpr + inline)", asm volatile("v_add3_u32 %0, %0, %1, 7" : "+v"(x[i]) : "v"(y))) \
    X(19, "v_perm_b32 (3 vgpr)", asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(x[(i + 2) & 7]))) \
    X(20, "v_cndmask_b32 vcc (no write)", asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(y))) \
    X(21, "v_lshl_add_u64", asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(q[i]) : "v"(q[(i + 1) & 7]))) \
    X(22, "v_cmp_lt_u64 (vcc)", asm volatile("v_cmp_lt_u64 vcc, %0, %1" :: "v"(q[i]), "v"(q[(i + 1) & 7]) : "vcc")) \
    X(23, "v_min_u32 (vgpr, sgpr)", asm volatile("v_min_u32 %0, %1, %0" : "+v"(x[i]) : "s"(k))) \
    X(24, "v_bitop3 (vgpr, vgpr, inline 7)", asm volatile("v_bitop3_b32 %0, %0, %1, 7 bitop3:0xea" : "+v"(x[i]) : "v"(y))) \
    X(25, "v_and_or_b32 (3 vgpr)", asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(x[(i + 2) & 7])))

constexpr int kOps = 26;

template <int OP>
__global__ __launch_bounds__(256) void spin(uint32_t *out, uint64_t *stamps, uint32_t seed) {
    uint32_t x[kCh], z[kCh];
    uint64_t q[kCh];
    uint64_t mm[2] = {0, 0};
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
                const uint64_t m = 0x5555555555555555ull * (seed & 1);
                (void)k;
                (void)m;
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
    acc ^= (uint32_t)(mm[0] ^ mm[1]);
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
    const double per = (OP == 5) ? 2.0 : 1.0;
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
