// valu_peak.hip -- measured VALU issue rate of the integer instructions the
// SHA-256 and fingerprint kernels are made of, per SIMD, at
// 1..8 waves per SIMD.  Each lane runs 8 independent dependency chains of one
// instruction kind, so the rate is issue-bound, not latency-bound.
//
// Every wave stamps its spin loop with s_memtime (shader-clock cycles) and
// s_memrealtime (the constant 100 MHz counter): the effective clock =
// d(memtime) / d(realtime) x 100 MHz (median wave).  Cycles per
// wave-instruction per SIMD = the kernel's event time x that clock x SIMDs /
// wave-instructions, so DVFS is separated from issue rate.  The same figure
// at an assumed 2.4 GHz is printed beside it.
//   hipcc -O3 --offload-arch=gfx950 valu_peak.hip -o valu_peak && ./valu_peak
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int kIters = 4096;
constexpr int kChainsPerLane = 8;
constexpr int kOps = 9;

template <int OP>
__global__ __launch_bounds__(256) void spin(uint32_t *out, uint64_t *stamps, uint32_t seed) {
    uint32_t x[kChainsPerLane];
    float f[kChainsPerLane];
#pragma unroll
    for (int i = 0; i < kChainsPerLane; ++i) {
        x[i] = seed * (threadIdx.x + 17 * i + 1);
        f[i] = (float)x[i];
    }
    const uint32_t k = seed | 1;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
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
                if (OP == 7) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(x[i]) : "v"(y));
                if (OP == 8) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(x[i]) : "v"(y));
            }
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < kChainsPerLane; ++i) acc ^= x[i] ^ __float_as_uint(f[i]);
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) {
        uint64_t *s = stamps + 4 * ((uint64_t)blockIdx.x * 4 + threadIdx.x / 64);
        s[0] = c1 - c0;
        s[1] = r1 - r0;
    }
}

struct Res {
    double cyc_per_instr;   // shader cycles per wave-instruction per SIMD (median wave)
    double clock_ghz;       // effective shader clock during the loop
    double event_cyc_24;    // host-event figure at an assumed 2.4 GHz
};

template <int OP>
Res run(int cus, int waves_per_simd, uint32_t *out, uint64_t *stamps) {
    // 256-thread blocks = one wave per SIMD per block
    const int grid = cus * waves_per_simd;
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
    std::vector<double> cyc, clk;
    for (int w = 0; w < waves; ++w) {
        const double c = (double)st[4 * w], r = (double)st[4 * w + 1];
        cyc.push_back(c);
        if (r > 0) clk.push_back(c / r * 0.1);
    }
    std::sort(cyc.begin(), cyc.end());
    std::sort(clk.begin(), clk.end());
    const double per_wave = (double)kIters * 4 * kChainsPerLane;
    Res r;
    // the clock the SIMDs ran at (median over waves of d(memtime)/d(realtime)),
    // applied to the kernel's event time: shader cycles spent per
    // wave-instruction per SIMD, DVFS separated from issue rate
    r.clock_ghz = clk.empty() ? 0 : clk[clk.size() / 2];
    const double wave_instr = (double)waves * per_wave;
    r.cyc_per_instr = ms * 1e-3 * r.clock_ghz * 1e9 * cus * 4 / wave_instr;
    r.event_cyc_24 = ms * 1e-3 * 2.4e9 * cus * 4 / wave_instr;
    hipEventDestroy(a);
    hipEventDestroy(b);
    return r;
}

template <int OP>
Res dispatch(int cus, int w, uint32_t *out, uint64_t *stamps) {
    return run<OP>(cus, w, out, stamps);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *out;
    uint64_t *stamps;
    hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
    hipMalloc(&stamps, (size_t)cus * 8 * 4 * 4 * 8);
    const char *names[kOps] = {"v_add3_u32",    "v_alignbit_b32", "v_bitop3_b32",
                               "v_xor_b32",     "v_fma_f32",      "v_perm_b32",
                               "v_lshl_or_b32", "v_add_u32_e32",  "v_xor_b32_e64"};
    printf("{\"cus\": %d, \"clock\": \"s_memtime cycles; effective GHz from s_memrealtime (100 MHz)\", "
           "\"ops\": {", cus);
    for (int op = 0; op < kOps; ++op) {
        printf("%s\"%s\": {", op ? ", " : "", names[op]);
        for (int w = 1; w <= 8; w *= 2) {
            Res r{};
            switch (op) {
                case 0: r = dispatch<0>(cus, w, out, stamps); break;
                case 1: r = dispatch<1>(cus, w, out, stamps); break;
                case 2: r = dispatch<2>(cus, w, out, stamps); break;
                case 3: r = dispatch<3>(cus, w, out, stamps); break;
                case 4: r = dispatch<4>(cus, w, out, stamps); break;
                case 5: r = dispatch<5>(cus, w, out, stamps); break;
                case 6: r = dispatch<6>(cus, w, out, stamps); break;
                case 7: r = dispatch<7>(cus, w, out, stamps); break;
                default: r = dispatch<8>(cus, w, out, stamps); break;
            }
            printf("%s\"%d\": {\"cyc_per_wave_instr\": %.2f, \"clock_ghz\": %.3f, "
                   "\"event_cyc_at_2.4GHz\": %.2f}",
                   w > 1 ? ", " : "", w, r.cyc_per_instr, r.clock_ghz, r.event_cyc_24);
        }
        printf("}");
    }
    printf("}}\n");
    hipFree(out);
    hipFree(stamps);
    return 0;
}
