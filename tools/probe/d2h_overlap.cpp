// d2h_overlap.cpp -- does a device-to-host read-back run beside a kernel that
// holds every CU?  (R7's contribution rows, 1/16 of the
// source, cross PCIe while the walk kernel occupies the chip.)
//
// A spin kernel (persistent: 8 workgroups of 256 threads per CU, ~60 ms) runs
// on stream A; 4 GiB leave the device on stream B in 16 MiB pieces, by several
// mechanisms.  For each: the copy alone, the spin alone, and both together,
// with the time at which the copies finished measured from the spin's start.
// Copies that need a CU (blit kernels) finish only after the spin; copies on a
// DMA engine finish beside it.
//   hipcc -O2 --offload-arch=gfx950 d2h_overlap.cpp -o bin/d2h_overlap && bin/d2h_overlap
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorName(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ __launch_bounds__(256) void spin(uint32_t *out, uint32_t iters) {
    uint32_t x = threadIdx.x * 2654435761u + blockIdx.x;
    for (uint32_t i = 0; i < iters; ++i) x = x * 1664525u + 1013904223u;
    if (x == 0x12345678u) out[0] = x;
}

// a copy kernel that writes the host buffer through its device-visible address
__global__ __launch_bounds__(256) void copy_to_host(const uint4 *src, uint4 *dst, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
         i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t piece = 16ull << 20, total = 4ull << 30;
    const int np = (int)(total / piece);
    void *dsrc;
    CK(hipMalloc(&dsrc, total));
    CK(hipMemset(dsrc, 1, total));
    uint32_t *dout;
    CK(hipMalloc(&dout, 64));
    void *hpin, *hpin_nc, *hreg;
    CK(hipHostMalloc(&hpin, total, hipHostMallocDefault));
    CK(hipHostMalloc(&hpin_nc, total, hipHostMallocNonCoherent));
    hreg = aligned_alloc(4096, total);
    CK(hipHostRegister(hreg, total, hipHostRegisterDefault));
    void *hpin_dev = nullptr;
    CK(hipHostGetDevicePointer(&hpin_dev, hpin, 0));
    hipStream_t A, B, Blo, Bhi;
    CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
    int least = 0, greatest = 0;
    CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    CK(hipStreamCreateWithPriority(&Blo, hipStreamNonBlocking, least));
    CK(hipStreamCreateWithPriority(&Bhi, hipStreamNonBlocking, greatest));
    hipEvent_t a0, a1, b1;
    CK(hipEventCreate(&a0));
    CK(hipEventCreate(&a1));
    CK(hipEventCreate(&b1));
    const uint32_t iters = 2000000;
    const int grid = cus * 8;
    // warm up
    spin<<<grid, 256, 0, A>>>(dout, 1000);
    CK(hipMemcpyAsync(hpin, dsrc, piece, hipMemcpyDeviceToHost, B));
    CK(hipDeviceSynchronize());

    const char *names[] = {"hipMemcpyAsync D2H -> hipHostMalloc", "hipMemcpyAsync D2H -> non-coherent",
                           "hipMemcpyAsync D2H -> hipHostRegister", "hipMemcpyDtoHAsync -> hipHostMalloc",
                           "copy kernel -> host pointer (1 CU-worth grid)",
                           "hipMemcpyAsync D2H on a lowest-priority stream",
                           "hipMemcpyAsync D2H on a highest-priority stream"};
    printf("{\"cus\": %d, \"piece_MiB\": %zu, \"total_GiB\": %zu, \"results\": [\n", cus, piece >> 20,
           total >> 30);
    for (int mode = 0; mode < 7; ++mode) {
        hipStream_t S = mode == 5 ? Blo : mode == 6 ? Bhi : B;
        auto copies = [&]() {
            for (int k = 0; k < np; ++k) {
                const char *s = (const char *)dsrc + (size_t)k * piece;
                switch (mode) {
                    case 0: CK(hipMemcpyAsync((char *)hpin + (size_t)k * piece, s, piece, hipMemcpyDeviceToHost, B)); break;
                    case 1: CK(hipMemcpyAsync((char *)hpin_nc + (size_t)k * piece, s, piece, hipMemcpyDeviceToHost, B)); break;
                    case 2: CK(hipMemcpyAsync((char *)hreg + (size_t)k * piece, s, piece, hipMemcpyDeviceToHost, B)); break;
                    case 3: CK(hipMemcpyDtoHAsync((char *)hpin + (size_t)k * piece, (hipDeviceptr_t)s, piece, B)); break;
                    case 5:
                    case 6: CK(hipMemcpyAsync((char *)hpin + (size_t)k * piece, s, piece, hipMemcpyDeviceToHost, S)); break;
                    default:
                        copy_to_host<<<64, 256, 0, B>>>((const uint4 *)s, (uint4 *)((char *)hpin_dev + (size_t)k * piece),
                                                        piece / 16);
                }
            }
            CK(hipEventRecord(b1, S));
        };
        // copies alone
        CK(hipDeviceSynchronize());
        auto t0 = std::chrono::steady_clock::now();
        copies();
        CK(hipEventSynchronize(b1));
        const double alone = ms_since(t0);
        // spin alone
        CK(hipEventRecord(a0, A));
        spin<<<grid, 256, 0, A>>>(dout, iters);
        CK(hipEventRecord(a1, A));
        CK(hipEventSynchronize(a1));
        float spin_ms = 0;
        CK(hipEventElapsedTime(&spin_ms, a0, a1));
        // both: spin first, then the copies on the other stream
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a0, A));
        spin<<<grid, 256, 0, A>>>(dout, iters);
        CK(hipEventRecord(a1, A));
        copies();
        CK(hipDeviceSynchronize());
        float spin_both = 0, copies_done = 0;
        CK(hipEventElapsedTime(&spin_both, a0, a1));
        CK(hipEventElapsedTime(&copies_done, a0, b1));
        printf("%s {\"mode\": \"%s\", \"copies_alone_ms\": %.2f, \"GBps_alone\": %.1f, \"spin_alone_ms\": %.2f, "
               "\"spin_with_copies_ms\": %.2f, \"copies_done_after_spin_start_ms\": %.2f}\n",
               mode ? "," : "", names[mode], alone, total / alone / 1e6, spin_ms, spin_both, copies_done);
        fflush(stdout);
    }
    printf("]}\n");
    return 0;
}
