// d2h_numa.cpp -- why does the contribution read-back run at ~55 GB/s in some
// processes and ~30 GB/s in others (profiles/r05_r7/trace: the file-sum jobs
// wait 240-266 ms per 4 GiB on their DMA copies in the slow runs, 3-64 ms in
// the fast ones)?  Candidates: the NUMA node the pinned destination pages sit
// on, and which SDMA engine the copies land on.
//
// For every online NUMA node: 1 GiB bound to it (mmap + mbind, touched,
// hipHostRegister), read back from the device in 16 MiB SDMA copies
// (hsa_amd_memory_async_copy, one in flight: the library's pattern), by one
// thread and by three threads each into its own buffer.  Then the node of a
// hipHostMalloc buffer's pages (move_pages), and the rate per SDMA engine
// (hsa_amd_memory_async_copy_on_engine).
//   hipcc -O2 --offload-arch=gfx950 d2h_numa.cpp -o bin/d2h_numa -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
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

static hsa_agent_t g_gpu{}, g_cpu{};
static hsa_status_t find_agent(hsa_agent_t a, void *) {
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
    return HSA_STATUS_SUCCESS;
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

static const size_t kPiece = 16ull << 20;

// n bytes in kPiece copies, one in flight; engine < 0: the runtime's choice
static bool dma(void *dst, const void *src, size_t n, int engine) {
    hsa_signal_t sig;
    if (hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) return false;
    bool ok = true;
    for (size_t o = 0; o < n && ok; o += kPiece) {
        hsa_signal_store_relaxed(sig, 1);
        hsa_status_t st;
        if (engine < 0)
            st = hsa_amd_memory_async_copy((char *)dst + o, g_cpu, (const char *)src + o, g_gpu, kPiece, 0,
                                           nullptr, sig);
        else
            st = hsa_amd_memory_async_copy_on_engine((char *)dst + o, g_cpu, (const char *)src + o, g_gpu,
                                                     kPiece, 0, nullptr, sig,
                                                     (hsa_amd_sdma_engine_id_t)(1u << engine), true);
        if (st != HSA_STATUS_SUCCESS) {
            ok = false;
            break;
        }
        hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    }
    hsa_signal_destroy(sig);
    return ok;
}

static void *node_buf(size_t n, int node) {
    void *p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) return nullptr;
    if (node >= 0) {
        unsigned long mask[16] = {};
        mask[node / 64] = 1ul << (node % 64);
        if (syscall(SYS_mbind, p, n, 2 /* MPOL_BIND */, mask, 1024, 0) != 0) {
            munmap(p, n);
            return nullptr;
        }
    }
    memset(p, 0, n);
    if (hipHostRegister(p, n, hipHostRegisterDefault) != hipSuccess) {
        (void)hipGetLastError();
        munmap(p, n);
        return nullptr;
    }
    return p;
}

// the node of the page at p (-1: unknown)
static int page_node(void *p) {
    void *pages[1] = {p};
    int status[1] = {-1};
    if (syscall(SYS_move_pages, 0, 1, pages, nullptr, status, 0) != 0) return -1;
    return status[0];
}

int main() {
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));
    if (hsa_init() != HSA_STATUS_SUCCESS || hsa_iterate_agents(find_agent, nullptr) != HSA_STATUS_SUCCESS)
        return 4;
    char bdf[64] = {};
    CK(hipDeviceGetPCIBusId(bdf, sizeof bdf, 0));
    for (char *c = bdf; *c; ++c) *c = (char)tolower(*c);
    std::string gnode = "?", online = "?";
    {
        std::ifstream f(std::string("/sys/bus/pci/devices/") + bdf + "/numa_node");
        if (f) f >> gnode;
        std::ifstream g("/sys/devices/system/node/online");
        if (g) g >> online;
    }
    std::vector<int> nodes;
    for (int n = 0; n < 64; ++n) {
        std::ifstream f("/sys/devices/system/node/node" + std::to_string(n) + "/cpulist");
        if (f) nodes.push_back(n);
    }
    uint32_t engines = 0, preferred = 0;
    hsa_amd_memory_copy_engine_status(g_cpu, g_gpu, &engines);
    const int pst = (int)hsa_amd_memory_get_preferred_copy_engine(g_cpu, g_gpu, &preferred);
    const size_t n = 1ull << 30;
    void *dsrc;
    CK(hipMalloc(&dsrc, 3 * n));
    CK(hipMemset(dsrc, 1, 3 * n));
    printf("{\"gpu_bdf\": \"%s\", \"gpu_numa_node\": \"%s\", \"nodes_online\": \"%s\", "
           "\"sdma_engine_mask_free\": %u, \"preferred_mask\": %u, \"preferred_status\": %d, "
           "\"cpu_of_main\": %d, \"results\": [\n",
           bdf, gnode.c_str(), online.c_str(), engines, preferred, pst, sched_getcpu());
    bool first = true;
    auto line = [&](const std::string &what, double gbps) {
        printf("%s {\"what\": \"%s\", \"GBps\": %.1f}\n", first ? "" : ",", what.c_str(), gbps);
        first = false;
        fflush(stdout);
    };
    for (int node : nodes) {
        void *b[3];
        bool ok = true;
        for (auto &x : b) ok = ok && (x = node_buf(n, node)) != nullptr;
        if (!ok) {
            line("node " + std::to_string(node) + ": allocation failed", 0);
            continue;
        }
        for (int rep = 0; rep < 2; ++rep) {
            double t0 = now_ms();
            dma(b[0], dsrc, n, -1);
            line("node " + std::to_string(node) + " (page on " + std::to_string(page_node(b[0])) +
                     "), one thread, rep " + std::to_string(rep),
                 n / (now_ms() - t0) / 1e6);
            t0 = now_ms();
            std::vector<std::thread> th;
            for (int k = 0; k < 3; ++k) th.emplace_back(dma, b[k], (const char *)dsrc + k * n, n, -1);
            for (auto &t : th) t.join();
            line("node " + std::to_string(node) + ", three threads (aggregate), rep " + std::to_string(rep),
                 3 * n / (now_ms() - t0) / 1e6);
        }
        for (auto &x : b) {
            (void)hipHostUnregister(x);
            munmap(x, n);
        }
    }
    void *hm = nullptr;
    CK(hipHostMalloc(&hm, n, hipHostMallocDefault));
    {
        const double t0 = now_ms();
        dma(hm, dsrc, n, -1);
        line("hipHostMalloc (page on node " + std::to_string(page_node(hm)) + "), one thread",
             n / (now_ms() - t0) / 1e6);
    }
    for (int e = 0; e < 16; ++e) {
        if (!(engines & (1u << e))) continue;
        const double t0 = now_ms();
        const bool ok = dma(hm, dsrc, n, e);
        line("hipHostMalloc, SDMA engine " + std::to_string(e) + (ok ? "" : " (refused)"),
             ok ? n / (now_ms() - t0) / 1e6 : 0);
    }
    // three threads at once on the preferred engine (else engine 1)
    {
        const int e = preferred ? __builtin_ctz(preferred) : 1;
        void *b[3];
        for (auto &x : b) CK(hipHostMalloc(&x, n, hipHostMallocDefault));
        const double t0 = now_ms();
        std::vector<std::thread> th;
        for (int k = 0; k < 3; ++k) th.emplace_back(dma, b[k], (const char *)dsrc + k * n, n, e);
        for (auto &t : th) t.join();
        line("three threads (aggregate), all on SDMA engine " + std::to_string(e), 3 * n / (now_ms() - t0) / 1e6);
        const double t1 = now_ms();
        std::vector<std::thread> th2;
        for (int k = 0; k < 3; ++k) th2.emplace_back(dma, b[k], (const char *)dsrc + k * n, n, -1);
        for (auto &t : th2) t.join();
        line("three threads (aggregate), runtime's choice", 3 * n / (now_ms() - t1) / 1e6);
    }
    printf("]}\n");
    return 0;
}
