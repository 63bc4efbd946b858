// xfer.cpp -- host <-> device copies of caller (pageable) memory, and the
// error plumbing of HIP calls.
//
// The library never page-locks memory it does not own.  Round 2 pinned its
// std::vector read-back storage with hipHostRegister; that storage shares
// pages with the rest of the process heap, and a later pageable hipMemcpy of a
// caller buffer >= 1 MiB -- which the runtime pins on the fly
// (DmaBlitManager's pinned path) -- failed when its pages overlapped a
// registered range.  Now every copy whose host side is not
// hipHostMalloc'd by the library goes through a Stager: two owned pinned
// buffers, the CPU memcpy of chunk k overlapping the DMA of chunk k-1.  The
// runtime is never handed a caller pointer to pin.
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <mutex>

#include "internal.hpp"

namespace vsgpu {

// ---- device-to-host copies on a DMA engine (round 5) ---------------------------
// Inside a PyTorch process the library shares torch's bundled HIP runtime, and
// that runtime performs hipMemcpyAsync device-to-host copies as blit kernels
// (__amd_rocclr_copyBuffer), which need a free CU: behind a persistent kernel
// that holds every CU (the rsync walk) they wait until it ends
// (tools/probe/d2h_apis.py: every hipMemcpy* form but one runs as a blit; the
// HSA runtime's own async copy runs on an SDMA engine, beside anything).  The
// whole-file checksum reads its contribution rows back this way.  HSA is the
// runtime under HIP (already initialised by it; hsa_init only counts a user).
namespace {
struct DmaAgents {
    bool tried = false, ok = false;
    hsa_agent_t gpu{}, cpu{};
};
std::mutex g_dma_mu;
DmaAgents g_dma[64];

struct AgentFind {
    uint32_t bdf = 0, domain = 0;
    hsa_agent_t gpu{}, cpu{};
    bool found = false;
};

hsa_status_t agent_cb(hsa_agent_t a, void *p) {
    AgentFind *f = (AgentFind *)p;
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_CPU && !f->cpu.handle) f->cpu = a;
    if (t == HSA_DEVICE_TYPE_GPU && !f->found) {
        uint32_t bdf = 0, dom = 0;
        if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) == HSA_STATUS_SUCCESS &&
            hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom) == HSA_STATUS_SUCCESS &&
            bdf == f->bdf && dom == f->domain) {
            f->gpu = a;
            f->found = true;
        }
    }
    return HSA_STATUS_SUCCESS;
}

// the HSA agents of HIP device `device` (matched by PCI domain / bus / device
// / function) and a CPU agent; false when they cannot be found
bool dma_agents(int device, hsa_agent_t *gpu, hsa_agent_t *cpu) {
    if (device < 0 || device >= 64) return false;
    std::lock_guard<std::mutex> lk(g_dma_mu);
    DmaAgents &d = g_dma[device];
    if (!d.tried) {
        d.tried = true;
        int bus = 0, dev = 0, dom = 0;
        if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
            hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess ||
            hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) != hipSuccess) {
            (void)hipGetLastError();
        } else if (hsa_init() == HSA_STATUS_SUCCESS) {
            AgentFind f;
            f.bdf = ((uint32_t)bus << 8) | ((uint32_t)dev << 3);
            f.domain = (uint32_t)dom;
            if (hsa_iterate_agents(agent_cb, &f) == HSA_STATUS_SUCCESS && f.found && f.cpu.handle) {
                d.gpu = f.gpu;
                d.cpu = f.cpu;
                d.ok = true;
            }
        }
    }
    *gpu = d.gpu;
    *cpu = d.cpu;
    return d.ok;
}
}  // namespace

bool DmaD2H::init(int device) {
    if (!ready) {
        hsa_agent_t g{}, c{};
        ready = dma_agents(device, &g, &c);
        gpu_ = g.handle;
        cpu_ = c.handle;
        for (int i = 0; ready && i < kSignals; ++i) {
            hsa_signal_t t{};
            if (hsa_signal_create(0, 0, nullptr, &t) != HSA_STATUS_SUCCESS) {
                for (int k = 0; k < i; ++k) hsa_signal_destroy(hsa_signal_t{sig_[k]});
                ready = false;
            }
            sig_[i] = t.handle;
        }
        // The engine: the runtime's recommendation for this direction.  Left
        // to hsa_amd_memory_async_copy, a process's copies landed on whatever
        // engine it assigned, and the engines differ: device to host on an
        // MI355X box, engine 1 52.6 GB/s, engines 0, 2, 3 35-37, engines 4-15
        // 6-11 (tools/probe/d2h_numa.cpp, profiles/r05_r7/numa) -- the R7
        // read-back ran at 55 GB/s in some processes and at a fraction of it
        // in others (profiles/r05_r7/trace).
        uint32_t pref = 0, avail = 0;
        if (ready &&
            hsa_amd_memory_get_preferred_copy_engine(c, g, &pref) == HSA_STATUS_SUCCESS &&
            hsa_amd_memory_copy_engine_status(c, g, &avail) == HSA_STATUS_SUCCESS) {
            const uint32_t m = (pref & avail) ? (pref & avail) : pref;
            engine = m ? __builtin_ctz(m) : -1;
        }
    }
    return ready;
}

void DmaD2H::release() {
    if (!ready) return;
    for (int i = 0; i < kSignals; ++i) hsa_signal_destroy(hsa_signal_t{sig_[i]});
    ready = false;
}

bool DmaD2H::start(int slot, void *dst, const void *src, size_t n) {
    const hsa_signal_t s{sig_[slot]};
    hsa_signal_store_screlease(s, 1);
    const hsa_status_t st =
        engine >= 0
            ? hsa_amd_memory_async_copy_on_engine(dst, hsa_agent_t{cpu_}, src, hsa_agent_t{gpu_}, n, 0,
                                                  nullptr, s, (hsa_amd_sdma_engine_id_t)(1u << engine),
                                                  true)
            : hsa_amd_memory_async_copy(dst, hsa_agent_t{cpu_}, src, hsa_agent_t{gpu_}, n, 0, nullptr, s);
    // not queued: nothing will ever lower the signal, so a later wait on
    // this slot must not block
    if (st != HSA_STATUS_SUCCESS) hsa_signal_store_screlease(s, 0);
    return st == HSA_STATUS_SUCCESS;
}

bool DmaD2H::wait(int slot) {
    const hsa_signal_t s{sig_[slot]};
    hsa_signal_value_t v;
    do {
        v = hsa_signal_wait_scacquire(s, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    } while (v >= 1);   // a spurious wake-up; a negative value is a copy error
    return v == 0;
}

// The staging copies are the host side of every pageable feed (the Go
// Chunker's read buffer is pageable): one thread copies ~20 GB/s, a third of
// what the DMA behind it moves, so large copies are split over four threads.
void par_memcpy(void *dst, const void *src, size_t n) {
    constexpr int threads = 4;
    constexpr size_t kMin = 4u << 20;   // per thread
    const int t = (int)std::min<size_t>((size_t)threads, n / kMin);
    if (t <= 1) {
        memcpy(dst, src, n);
        return;
    }
    const size_t part = (n / (size_t)t + 4095) & ~(size_t)4095;
    std::vector<std::thread> pool;
    pool.reserve((size_t)t - 1);
    for (int i = 1; i < t; ++i) {
        const size_t off = part * (size_t)i;
        if (off >= n) break;
        pool.emplace_back([=] { memcpy((char *)dst + off, (const char *)src + off, std::min(part, n - off)); });
    }
    memcpy(dst, src, std::min(part, n));
    for (auto &th : pool) th.join();
}

int fail_hip(hipError_t e, const char *what, const char *file, int line) {
    (void)hipGetLastError();  // clear the runtime's last error: it is reported here
    const char *base = strrchr(file, '/');
    return fail(VS_ERR_HIP, std::string(what) + ": " + hipGetErrorName(e) + " (" +
                                std::to_string((int)e) + ", " + hipGetErrorString(e) + ") at " +
                                (base ? base + 1 : file) + ":" + std::to_string(line));
}

int enter_device(int device) {
    // the runtime's last error is per thread and sticky until read: an error
    // the caller left (a failed hipMemcpy of its own, say) would otherwise be
    // returned by the hipGetLastError() after this call's first kernel launch
    (void)hipGetLastError();
    const hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(VS_ERR_NO_DEVICE, "hipSetDevice(" + std::to_string(device) + "): " +
                                          hipGetErrorName(e));
    }
    return 0;
}

void *pinned_alloc(size_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, std::max<size_t>(bytes, 64), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return p;
}

void pinned_free(void *p) {
    if (p) (void)hipHostFree(p);
}

bool host_range_pinned(const void *p, size_t n) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (at.type != hipMemoryTypeHost) return false;
    // the whole range must lie in one page-locked allocation: a DMA that runs
    // past a registered range's end fails (hipErrorInvalidValue)
    uintptr_t start = 0;
    size_t size = 0;
    // The range attributes report size 0 for a 64 GiB pinned allocation on
    // ROCm 7 (tools/probe/pin_torch.py, profiles/r03_end/pin_torch64.log);
    // hipMemGetAddressRange reports it right
    if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p) !=
            hipSuccess ||
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p) !=
            hipSuccess ||
        size == 0) {
        // the allocation's extent from the runtime's address-range query
        (void)hipGetLastError();
        hipDeviceptr_t base = 0;
        if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        start = (uintptr_t)base;
    }
    const uintptr_t a = (uintptr_t)p;
    return start <= a && a + n <= start + size;
}

int Stager::init() {
    if (buf[0]) return 0;
    for (int i = 0; i < 2; ++i) {
        buf[i] = (uint8_t *)pinned_alloc(kChunk);
        if (!buf[i] || hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            release();
            return fail(VS_ERR_NOMEM, "pinned staging buffers (2 x " + std::to_string(kChunk) +
                                          " bytes) could not be allocated");
        }
        busy[i] = false;
    }
    return 0;
}

int Stager::wait(int i) {
    if (busy[i]) VS_HIP(hipEventSynchronize(ev[i]));
    busy[i] = false;
    return 0;
}

int Stager::h2d(void *dst, const void *src, size_t n, hipStream_t s) {
    if (!n) return 0;
    VS_TRY(init());
    const uint8_t *p = (const uint8_t *)src;
    uint8_t *d = (uint8_t *)dst;
    for (size_t off = 0; off < n; off += kChunk) {
        const size_t k = std::min(kChunk, n - off);
        VS_TRY(wait(next));
        par_memcpy(buf[next], p + off, k);
        VS_HIP(hipMemcpyAsync(d + off, buf[next], k, hipMemcpyHostToDevice, s));
        VS_HIP(hipEventRecord(ev[next], s));
        busy[next] = true;
        next ^= 1;
    }
    // the caller's bytes are all in staging memory: it may reuse src now; the
    // DMA stays ordered on s, and the next use of a buffer waits for its event
    return 0;
}

int Stager::d2h(void *dst, const void *src, size_t n, hipStream_t s) {
    if (!n) return 0;
    VS_TRY(init());
    const uint8_t *d = (const uint8_t *)src;
    uint8_t *p = (uint8_t *)dst;
    // chunk k's DMA runs while chunk k-1 is copied out of staging
    size_t prev_off = 0, prev_k = 0;
    int prev = -1;
    for (size_t off = 0; off < n; off += kChunk) {
        const size_t k = std::min(kChunk, n - off);
        VS_TRY(wait(next));
        VS_HIP(hipMemcpyAsync(buf[next], d + off, k, hipMemcpyDeviceToHost, s));
        VS_HIP(hipEventRecord(ev[next], s));
        busy[next] = true;
        if (prev >= 0) {
            VS_TRY(wait(prev));
            par_memcpy(p + prev_off, buf[prev], prev_k);
        }
        prev = next;
        prev_off = off;
        prev_k = k;
        next ^= 1;
    }
    VS_TRY(wait(prev));
    par_memcpy(p + prev_off, buf[prev], prev_k);
    return 0;
}

void Stager::release() {
    for (int i = 0; i < 2; ++i) {
        if (ev[i]) {
            (void)hipEventSynchronize(ev[i]);
            (void)hipEventDestroy(ev[i]);
        }
        pinned_free(buf[i]);
        buf[i] = nullptr;
        ev[i] = nullptr;
        busy[i] = false;
    }
    next = 0;
}

}  // namespace vsgpu
