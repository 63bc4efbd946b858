// pin_range.cpp -- which HIP queries report the extent of a page-locked host
// allocation (host_range_pinned in xfer.cpp decides between a direct DMA of
// caller memory and the staging copy on them).
//   hipcc -O2 pin_range.cpp -o pin_range && ./pin_range
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

static void probe(const char *what, void *base, size_t n) {
    for (size_t off : {(size_t)0, n / 2}) {
        void *p = (char *)base + off;
        hipPointerAttribute_t at{};
        hipError_t e1 = hipPointerGetAttributes(&at, p);
        uintptr_t start = 0;
        size_t size = 0;
        hipError_t e2 = hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR,
                                               (hipDeviceptr_t)p);
        hipError_t e3 = hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE,
                                               (hipDeviceptr_t)p);
        hipDeviceptr_t rb = 0;
        size_t rs = 0;
        hipError_t e4 = hipMemGetAddressRange(&rb, &rs, (hipDeviceptr_t)p);
        unsigned int flags = 0;
        hipError_t e5 = hipHostGetFlags(&flags, p);
        (void)hipGetLastError();
        printf("%s +%zu: attrs %s type %d host %p | range_start %s %p range_size %s %zu | "
               "addr_range %s %p %zu | host_flags %s 0x%x | base %p n %zu\n",
               what, off, hipGetErrorName(e1), (int)at.type, at.hostPointer, hipGetErrorName(e2),
               (void *)start, hipGetErrorName(e3), size, hipGetErrorName(e4), (void *)rb, rs,
               hipGetErrorName(e5), flags, base, n);
    }
}

int main() {
    const size_t n = 1ull << 30;
    void *a = nullptr;
    if (hipHostMalloc(&a, n, hipHostMallocDefault) == hipSuccess) probe("hipHostMalloc", a, n);
    void *b = nullptr;
    if (hipHostMalloc(&b, n, hipHostMallocPortable | hipHostMallocMapped) == hipSuccess)
        probe("hipHostMalloc(portable|mapped)", b, n);
    void *c = aligned_alloc(4096, n);
    if (c && hipHostRegister(c, n, hipHostRegisterDefault) == hipSuccess) probe("hipHostRegister", c, n);
    void *d = malloc(1 << 20);
    probe("malloc", d, 1 << 20);
    return 0;
}
