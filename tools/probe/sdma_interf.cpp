// sdma_interf.cpp -- does a device-to-host DMA slow a latency-bound kernel
// beside it?  (R7: the walk kernel runs 41 -> 51.6 ms while the contribution
// rows leave the device on an SDMA engine, profiles/r05_r7.)
//
// A pointer-chasing kernel (every lane follows a random chain through a
// 1 GiB device table: one dependent 8-byte load after another, the walk's
// gather pattern) is timed alone and with 4 GiB leaving the device in 64 MiB
// SDMA copies (hsa_amd_memory_async_copy, as the library's DmaD2H does) into
//   a) hipHostMalloc memory (the library's pinned rings),
//   b) 2 MiB-aligned malloc memory advised MADV_HUGEPAGE, then hipHostRegister'd,
//   c) another device buffer (a device-to-device SDMA copy: no host pages).
// If the host pages' translations are what the kernel competes with, b) and
// c) leave it alone while a) slows it.
//   hipcc -O2 --offload-arch=gfx950 sdma_interf.cpp -o bin/sdma_interf -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorName(e_)); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

__global__ __launch_bounds__(256) void chase(const uint64_t *tab, uint64_t mask, uint32_t steps,
                                             uint64_t *out) {
    uint64_t x = (blockIdx.x * 256ull + threadIdx.x) * 0x9E3779B97F4A7C15ull;
    for (uint32_t i = 0; i < steps; ++i) x = tab[x & mask] ^ (x >> 7);
    if (x == 0x1234567ull) out[0] = x;
}

__global__ void fill(uint64_t *tab, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        tab[i] = z ^ (z >> 27);
    }
}

static hsa_agent_t g_gpu{}, g_cpu{};
static hsa_status_t find_agent(hsa_agent_t a, void *) {
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
    return HSA_STATUS_SUCCESS;
}

// total bytes from src to dst in `piece` copies, one in flight after another
static void dma(void *dst, hsa_agent_t dagent, const void *src, size_t total, size_t piece) {
    hsa_signal_t sig;
    if (hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) exit(2);
    for (size_t o = 0; o < total; o += piece) {
        hsa_signal_store_relaxed(sig, 1);
        if (hsa_amd_memory_async_copy((char *)dst + o, dagent, (const char *)src + o, g_gpu, piece, 0,
                                      nullptr, sig) != HSA_STATUS_SUCCESS)
            exit(3);
        hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    }
    hsa_signal_destroy(sig);
}

int main() {
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));   // the HIP runtime initialises HSA
    if (hsa_init() != HSA_STATUS_SUCCESS) return 5;
    if (hsa_iterate_agents(find_agent, nullptr) != HSA_STATUS_SUCCESS) return 4;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint64_t n = (1ull << 30) / 8;
    uint64_t *tab, *out;
    CK(hipMalloc(&tab, n * 8));
    CK(hipMalloc(&out, 64));
    fill<<<4096, 256>>>(tab, n);
    const size_t total = 4ull << 30, piece = 64ull << 20;
    void *dsrc, *ddst;
    CK(hipMalloc(&dsrc, total));
    CK(hipMalloc(&ddst, total));
    CK(hipMemset(dsrc, 1, total));
    void *hpin = nullptr;
    CK(hipHostMalloc(&hpin, total, hipHostMallocDefault));
    void *huge = aligned_alloc(2ull << 20, total);
    madvise(huge, total, MADV_HUGEPAGE);
    for (size_t o = 0; o < total; o += 4096) ((volatile char *)huge)[o] = 0;   // fault in
    CK(hipHostRegister(huge, total, hipHostRegisterDefault));
    void *huge_dev = nullptr;
    CK(hipHostGetDevicePointer(&huge_dev, huge, 0));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t steps = 1500;
    const int grid = cus * 8;
    auto kernel_ms = [&](uint64_t words) {
        CK(hipEventRecord(e0, 0));
        chase<<<grid, 256>>>(tab, words - 1, steps, out);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms;
    };
    kernel_ms(n);   // warm up
    // both tables: 1 GiB (HBM-latency bound) and 64 MiB (cache resident)
    auto both = [&](float *k) {
        k[0] = kernel_ms(n);
        k[1] = kernel_ms((64ull << 20) / 8);
    };
    struct Mode {
        const char *name;
        void *dst;
        hsa_agent_t agent;
    } modes[] = {{"none", nullptr, {}},
                 {"hipHostMalloc", hpin, g_cpu},
                 {"THP malloc + hipHostRegister", huge, g_cpu},
                 {"device to device", ddst, g_gpu}};
    printf("{\"cus\": %d, \"table_GiB\": 1, \"copy_GiB\": 4, \"piece_MiB\": 64, \"results\": [\n", cus);
    for (int rep = 0; rep < 2; ++rep) {
        for (int m = 0; m < 4; ++m) {
            double copy_ms = 0;
            float kms[2];
            if (!modes[m].dst) {
                both(kms);
            } else {
                // copy alone first (its rate), then beside the kernel
                auto t0 = std::chrono::steady_clock::now();
                dma(modes[m].dst, modes[m].agent, dsrc, total, piece);
                copy_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                std::thread th(dma, modes[m].dst, modes[m].agent, dsrc, total, piece);
                std::this_thread::sleep_for(std::chrono::milliseconds(5));
                both(kms);
                th.join();
            }
            printf("%s {\"rep\": %d, \"dst\": \"%s\", \"chase_1GiB_ms\": %.2f, \"chase_64MiB_ms\": %.2f, "
                   "\"copy_alone_ms\": %.1f, \"copy_GBps\": %.1f}\n",
                   rep || m ? "," : "", rep, modes[m].name, kms[0], kms[1], copy_ms,
                   copy_ms > 0 ? total / copy_ms / 1e6 : 0.0);
            fflush(stdout);
        }
    }
    printf("]}\n");
    (void)huge_dev;
    return 0;
}
