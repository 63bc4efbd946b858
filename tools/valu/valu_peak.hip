// valu_peak.hip -- measured VALU issue rate of the integer instructions the
// SHA-256 and fingerprint kernels are made of, per SIMD, at
// 1..8 waves per SIMD.  Each lane runs 8 independent dependency chains of one
// instruction kind, so the rate is issue-bound, not latency-bound.
//   hipcc -O3 --offload-arch=gfx950 valu_peak.hip -o valu_peak && ./valu_peak
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 4096;
constexpr int kChainsPerLane = 8;

template <int OP>
__global__ __launch_bounds__(256) void spin(uint32_t *out, uint32_t seed) {
    uint32_t x[kChainsPerLane];
    float f[kChainsPerLane];
#pragma unroll
    for (int i = 0; i < kChainsPerLane; ++i) {
        x[i] = seed * (threadIdx.x + 17 * i + 1);
        f[i] = (float)x[i];
    }
    const uint32_t k = seed | 1;
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
            for (int i = 0; i < kChainsPerLane; ++i) {
                const uint32_t y = x[(i + 1) & 7];
                if (OP == 0) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "s"(k));
                if (OP == 1) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x[i]) : "v"(y));
                if (OP == 2) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[i]) : "v"(y), "s"(k));
                if (OP == 3) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[i]) : "v"(y));
                if (OP == 4) asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(f[i]) : "v"(f[(i + 1) & 7]));
                if (OP == 5) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "s"(k));
                if (OP == 6) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(x[i]) : "v"(y));
            }
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < kChainsPerLane; ++i) acc ^= x[i] ^ __float_as_uint(f[i]);
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int OP>
double run(int cus, int waves_per_simd, uint32_t *out) {
    // 256-thread blocks = one wave per SIMD per block
    const int grid = cus * waves_per_simd;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    spin<OP><<<grid, 256>>>(out, 3);
    hipEventRecord(a);
    spin<OP><<<grid, 256>>>(out, 5);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double wave_instr = (double)grid * 4 * kIters * 4 * kChainsPerLane;
    const double simd_cycles = ms * 1e-3 * 2.4e9 * cus * 4;
    return simd_cycles / wave_instr;  // cycles per wave-instruction per SIMD
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *out;
    hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
    const char *names[] = {"v_add3_u32", "v_alignbit_b32", "v_bitop3_b32", "v_xor_b32", "v_fma_f32", "v_perm_b32", "v_lshl_or_b32"};
    printf("{\"cus\": %d, \"clock_ghz_assumed\": 2.4, \"cycles_per_wave_instr_per_simd\": {", cus);
    for (int op = 0; op < 7; ++op) {
        printf("%s\"%s\": {", op ? ", " : "", names[op]);
        for (int w = 1; w <= 8; w *= 2) {
            double c = 0;
            switch (op) {
                case 0: c = run<0>(cus, w, out); break;
                case 1: c = run<1>(cus, w, out); break;
                case 2: c = run<2>(cus, w, out); break;
                case 3: c = run<3>(cus, w, out); break;
                case 4: c = run<4>(cus, w, out); break;
                case 5: c = run<5>(cus, w, out); break;
                default: c = run<6>(cus, w, out); break;
            }
            printf("%s\"%d\": %.2f", w > 1 ? ", " : "", w, c);
        }
        printf("}");
    }
    printf("}}\n");
    hipFree(out);
    return 0;
}
