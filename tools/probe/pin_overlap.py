"""Probe: does a pageable hipMemcpy fail when the caller buffer shares a page
with a range another part of the process registered (hipHostRegister)?"""
import ctypes, mmap, sys

hip = ctypes.CDLL("libamdhip64.so")
hip.hipGetErrorName.restype = ctypes.c_char_p
vp, sz = ctypes.c_void_p, ctypes.c_size_t
hip.hipHostRegister.argtypes = [vp, sz, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [vp]
hip.hipMemcpy.argtypes = [vp, vp, sz, ctypes.c_int]
hip.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]


def name(e):
    return hip.hipGetErrorName(e).decode()


dev = vp()
assert hip.hipMalloc(ctypes.byref(dev), 128 << 20) == 0
PG = 4096


def region(pages):
    m = mmap.mmap(-1, pages * PG)
    buf = (ctypes.c_char * (pages * PG)).from_buffer(m)
    return m, buf, ctypes.addressof(buf)


def case(label, n, reg_off, reg_len, src_off, pages=None, unregister_first=False):
    pages = pages or (n + src_off + 3 * PG) // PG + 2
    m, buf, base = region(pages)
    ctypes.memset(base, 7, pages * PG)
    r = hip.hipHostRegister(vp(base + reg_off), reg_len, 0)
    if unregister_first and r == 0:
        hip.hipHostUnregister(vp(base + reg_off))
    e = hip.hipMemcpy(dev, vp(base + src_off), n, 1)
    hip.hipGetLastError()
    print(f"{label:58s} n={n:>9d} register={name(r):28s} memcpy={name(e)}", flush=True)
    if r == 0 and not unregister_first:
        hip.hipHostUnregister(vp(base + reg_off))
    del buf
    m.close()
    return e


for n in (512 << 10, 1_061_078, 4 << 20, 64 << 20):
    case("registered 64 B at the start of the first page", n, 0, 64, 128)
    case("registered 64 B in the last page (after the buffer)", n, 128 + n + 16, 64, 128)
    case("registered 64 B, then unregistered", n, 0, 64, 128, unregister_first=True)
    case("registered range overlapping the buffer bytes", n, 64, 256, 128)
    case("no registration", n, 0, 0, 128)


# How a stale registration can arise: two registrations sharing a page.
print("--- two registrations sharing a page", flush=True)
for order in ("low-then-high", "high-then-low"):
    m, buf, base = region(1024)
    A, B = (base + 64, 4096 + 100), (base + 4096 + 512, 8192)   # B starts in A's last page
    first, second = (A, B) if order == "low-then-high" else (B, A)
    r1 = hip.hipHostRegister(vp(first[0]), first[1], 0)
    r2 = hip.hipHostRegister(vp(second[0]), second[1], 0)
    u1 = hip.hipHostUnregister(vp(first[0]))
    u2 = hip.hipHostUnregister(vp(second[0]))
    # after both were "released": a pageable copy over their bytes
    e = hip.hipMemcpy(dev, vp(base + 128), 2 << 20, 1)
    hip.hipGetLastError()
    print(f"{order}: reg1={name(r1)} reg2={name(r2)} unreg1={name(u1)} unreg2={name(u2)} "
          f"memcpy-after={name(e)}", flush=True)
    del buf
    m.close()
