"""d2h_torch.py -- the d2h_overlap question inside a PyTorch process, whose HIP
runtime (torch's bundled libamdhip64) is the one the library binds to there:
does a pinned device-to-host copy run on a DMA engine beside a kernel that
holds the CUs, or as a blit kernel queued behind it?  The busy kernel is the
library's signature pass over 16 GiB (rs_sig_coop_kernel, every CU); 1 GiB
leaves the device in 16 MiB pieces on another stream, by torch copy_ and by
the library's own file-sum read-back path.  Run it under rocprofv3
--kernel-trace --memory-copy-trace to see which copies are blits."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from volsync_amd import Matcher, sum_sizes_sqroot, synth_fill_device  # noqa: E402

dev = torch.device("cuda", 0)
n = 16 << 30
d = torch.empty(n, dtype=torch.uint8, device=dev)
synth_fill_device(d.data_ptr(), 4, 0, n)
hdr = sum_sizes_sqroot(n)
s1 = torch.zeros(hdr.count, dtype=torch.int32, device=dev)
s2 = torch.zeros(hdr.count * hdr.s2length, dtype=torch.uint8, device=dev)
src = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
host = torch.empty(1 << 30, dtype=torch.uint8, pin_memory=True)
A = torch.cuda.Stream(dev)
B = torch.cuda.Stream(dev)
m = Matcher(0)
m.set_stream(A.cuda_stream)


def busy():
    for _ in range(3):
        m.signatures_device(d.data_ptr(), n, hdr.blength, hdr.s2length, 8, 1, s1.data_ptr(),
                            s2.data_ptr())


def copies():
    with torch.cuda.stream(B):
        for k in range(64):
            host[k << 24:(k + 1) << 24].copy_(src[k << 24:(k + 1) << 24], non_blocking=True)


out = {}
for name, fn in (("copies alone", lambda: copies()), ("busy alone", lambda: busy())):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    out[name + " ms"] = round((time.perf_counter() - t0) * 1e3, 2)
e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
torch.cuda.synchronize()
e0.record(A)
busy()
e1.record(A)
copies()
e2.record(B)
torch.cuda.synchronize()
out["both: busy ms"] = round(e0.elapsed_time(e1), 2)
out["both: copies done after busy start ms"] = round(e0.elapsed_time(e2), 2)
m.close()
print(json.dumps(out))
