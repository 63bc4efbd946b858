// d2h_apis.cpp -- which device-to-host copy APIs reach a DMA engine inside a
// PyTorch process?  Built as a shared library and loaded after torch (as
// libvsgpu.so is, so it binds to torch's bundled HIP runtime); d2h_apis.py
// calls copy(mode, ...) under rocprofv3 --memory-copy-trace: SDMA copies show
// as MEMORY_COPY_* records, blit copies as __amd_rocclr_copyBuffer kernels.
//   hipcc -O2 --offload-arch=gfx950 -shared -fPIC d2h_apis.cpp -o bin/libd2h_apis.so
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdint>
#include <cstdio>

static hsa_agent_t g_gpu{}, g_cpu{};
static bool g_agents = false;

static hsa_status_t find_agent(hsa_agent_t a, void *) {
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
    return HSA_STATUS_SUCCESS;
}

extern "C" int d2h_copy(int mode, void *host, const void *dev, size_t n, size_t pieces, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const size_t p = n / pieces;
    for (size_t k = 0; k < pieces; ++k) {
        char *h = (char *)host + k * p;
        const char *d = (const char *)dev + k * p;
        hipError_t e = hipSuccess;
        switch (mode) {
            case 0: e = hipMemcpyAsync(h, d, p, hipMemcpyDeviceToHost, s); break;
            case 1: e = hipMemcpyDtoHAsync(h, (hipDeviceptr_t)d, p, s); break;
            case 2: e = hipMemcpy2DAsync(h, p, d, p, p, 1, hipMemcpyDeviceToHost, s); break;
            case 3: e = hipMemcpyAsync(h, d, p, hipMemcpyDefault, s); break;
            case 4: e = hipMemcpyWithStream(h, d, p, hipMemcpyDeviceToHost, s); break;
            case 5: {   // the HSA runtime's DMA copy, ordered on the host
                if (!g_agents) {
                    if (hsa_iterate_agents(find_agent, nullptr) != HSA_STATUS_SUCCESS) return -10;
                    g_agents = true;
                }
                if (k == 0 && hipStreamSynchronize(s) != hipSuccess) return -11;
                hsa_signal_t sig;
                if (hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) return -12;
                if (hsa_amd_memory_async_copy(h, g_cpu, d, g_gpu, p, 0, nullptr, sig) != HSA_STATUS_SUCCESS)
                    return -13;
                hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
                hsa_signal_destroy(sig);
                break;
            }
            default: return -1;
        }
        if (e != hipSuccess) return -(100 + (int)e);
    }
    return 0;
}
