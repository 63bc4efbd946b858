"""What HIP reports for a torch pinned tensor (bench.py --mode host feeds one):
the pointer type, the allocation range attributes and hipMemGetAddressRange --
the queries host_range_pinned (xfer.cpp) uses to choose direct DMA."""
import ctypes

import torch

hip = ctypes.CDLL("libamdhip64.so")
import sys

n = int(float(sys.argv[1]) * (1 << 30)) if len(sys.argv) > 1 else 1 << 30
t = torch.empty(n, dtype=torch.uint8, pin_memory=True)
for off in (0, n // 2, n - (64 << 20)):
    p = ctypes.c_void_p(t.data_ptr() + off)
    start = ctypes.c_uint64(0)
    size = ctypes.c_size_t(0)
    # HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR = 11, RANGE_SIZE = 12 (hip_runtime_api.h)
    e2 = hip.hipPointerGetAttribute(ctypes.byref(start), 11, p)
    e3 = hip.hipPointerGetAttribute(ctypes.byref(size), 12, p)
    rb = ctypes.c_uint64(0)
    rs = ctypes.c_size_t(0)
    e4 = hip.hipMemGetAddressRange(ctypes.byref(rb), ctypes.byref(rs), p)
    fl = ctypes.c_uint(0)
    e5 = hip.hipHostGetFlags(ctypes.byref(fl), p)
    print(f"torch pinned +{off}: range_start rc {e2} {start.value:#x} range_size rc {e3} {size.value} "
          f"| addr_range rc {e4} {rb.value:#x} {rs.value} | host_flags rc {e5} {fl.value:#x} "
          f"| base {t.data_ptr():#x}")
