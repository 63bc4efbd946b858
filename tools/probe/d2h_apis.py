"""d2h_apis.py -- drives tools/probe/bin/libd2h_apis.so inside a PyTorch
process: 1 GiB device-to-host in 16 MiB pieces per copy API, alone and beside
a CU-filling kernel (an in-place add over 48 GiB, 4 times), with
the time the copies finished measured from the busy kernel's start.  Under
rocprofv3 --memory-copy-trace the DMA copies show as MEMORY_COPY records."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from volsync_amd import Matcher, sum_sizes_sqroot, synth_fill_device  # noqa: E402

L = ctypes.CDLL(os.path.join(ROOT, "tools", "probe", "bin", "libd2h_apis.so"))
L.d2h_copy.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                       ctypes.c_size_t, ctypes.c_void_p]
dev = torch.device("cuda", 0)
n = 48 << 30
d = torch.empty(n, dtype=torch.uint8, device=dev)
synth_fill_device(d.data_ptr(), 4, 0, n)
hdr = sum_sizes_sqroot(n)
s1 = torch.zeros(hdr.count, dtype=torch.int32, device=dev)
s2 = torch.zeros(hdr.count * hdr.s2length, dtype=torch.uint8, device=dev)
src = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
host = torch.empty(1 << 30, dtype=torch.uint8, pin_memory=True)
A, B = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
m = Matcher(0)
m.set_stream(A.cuda_stream)
names = ["hipMemcpyAsync D2H", "hipMemcpyDtoHAsync", "hipMemcpy2DAsync", "hipMemcpyAsync Default",
         "hipMemcpyWithStream", "hsa_amd_memory_async_copy"]
res = []
for mode, name in enumerate(names):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rc = L.d2h_copy(mode, host.data_ptr(), src.data_ptr(), 1 << 30, 64, B.cuda_stream)
    torch.cuda.synchronize()
    alone = (time.perf_counter() - t0) * 1e3
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(A)
    with torch.cuda.stream(A):   # asynchronous, every CU, HBM-bound
        for _ in range(4):
            d.add_(1)
    e1.record(A)
    rc2 = L.d2h_copy(mode, host.data_ptr(), src.data_ptr(), 1 << 30, 64, B.cuda_stream)
    B.synchronize()
    copies_done = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    res.append({"mode": name, "rc": [rc, rc2], "alone_ms": round(alone, 2),
                "busy_ms": round(e0.elapsed_time(e1), 2),
                "copies_done_from_busy_launch_ms": round(copies_done, 2)})
m.close()
print(json.dumps(res))
