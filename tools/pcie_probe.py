#!/usr/bin/env python3
"""Host<->device copy rates on the GPU box (profiling helper, not product code): pageable vs
pinned (hipHostMalloc) vs registered (hipHostRegister) host buffers, and what registering costs."""
import ctypes
import time

import numpy as np

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
hip.hipDeviceSynchronize.argtypes = []
H2D, D2H = 1, 2


def ck(rc):
    assert rc == 0, rc


def timeit(f, reps=5):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    ts.sort()
    return ts[len(ts) // 2]


N = 256 << 20
d = ctypes.c_void_p()
ck(hip.hipMalloc(ctypes.byref(d), N))
page = np.ones(N, dtype=np.uint8)
pin = ctypes.c_void_p()
ck(hip.hipHostMalloc(ctypes.byref(pin), N, 0))
ctypes.memset(pin, 1, N)
for name, p in (("pageable", page.ctypes.data), ("pinned", pin.value)):
    for dirn, lab in ((H2D, "h2d"), (D2H, "d2h")):
        a, b = (d.value, p) if dirn == H2D else (p, d.value)
        t = timeit(lambda: ck(hip.hipMemcpy(a, b, N, dirn)))
        print("%-10s %s %.1f GB/s" % (name, lab, N / t / 1e9), flush=True)
for mb in (32, 128, 256):
    buf = np.ones(mb << 20, dtype=np.uint8)
    t0 = time.perf_counter()
    ck(hip.hipHostRegister(buf.ctypes.data, buf.nbytes, 0))
    t1 = time.perf_counter()
    th = timeit(lambda: ck(hip.hipMemcpy(d.value, buf.ctypes.data, buf.nbytes, H2D)))
    td = timeit(lambda: ck(hip.hipMemcpy(buf.ctypes.data, d.value, buf.nbytes, D2H)))
    t2 = time.perf_counter()
    ck(hip.hipHostUnregister(buf.ctypes.data))
    t3 = time.perf_counter()
    print("registered %4d MB: register %.2f ms (%.1f GB/s), unregister %.2f ms, h2d %.1f GB/s, d2h %.1f GB/s" % (
        mb, (t1 - t0) * 1e3, buf.nbytes / (t1 - t0) / 1e9, (t3 - t2) * 1e3, buf.nbytes / th / 1e9, buf.nbytes / td / 1e9),
        flush=True)
# memcpy into pinned memory (the staging pipeline's host copy), one thread
src = np.ones(N, dtype=np.uint8)
dst = np.frombuffer((ctypes.c_uint8 * N).from_address(pin.value), dtype=np.uint8)
t = timeit(lambda: np.copyto(dst, src))
print("host memcpy -> pinned, 1 thread: %.1f GB/s" % (N / t / 1e9), flush=True)

# both directions at once, from two host threads on two streams (pageable / registered / pinned)
import threading  # noqa: E402

hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
s1, s2 = ctypes.c_void_p(), ctypes.c_void_p()
ck(hip.hipStreamCreate(ctypes.byref(s1)))
ck(hip.hipStreamCreate(ctypes.byref(s2)))
M = 128 << 20
d2 = ctypes.c_void_p()
ck(hip.hipMalloc(ctypes.byref(d2), M))
up_src = np.ones(M, dtype=np.uint8)
dn_dst = np.ones(M, dtype=np.uint8)


def both(src, dst, split=1):
    def up():
        for i in range(split):
            ck(hip.hipMemcpyAsync(d.value + i * (M // split), src + i * (M // split), M // split, H2D, s1))
        ck(hip.hipStreamSynchronize(s1))

    def dn():
        for i in range(split):
            ck(hip.hipMemcpyAsync(dst + i * (M // split), d2.value + i * (M // split), M // split, D2H, s2))
        ck(hip.hipStreamSynchronize(s2))
    a, b = threading.Thread(target=up), threading.Thread(target=dn)
    a.start(), b.start()
    a.join(), b.join()


for split in (1, 4):
    t = timeit(lambda: both(up_src.ctypes.data, dn_dst.ctypes.data, split))
    print("pageable both ways, %d MB each, %d copies each: %.2f ms (%.1f GB/s per direction)" % (
        M >> 20, split, t * 1e3, M / t / 1e9), flush=True)
ck(hip.hipHostRegister(up_src.ctypes.data, M, 0))
ck(hip.hipHostRegister(dn_dst.ctypes.data, M, 0))
for split in (1, 4):
    t = timeit(lambda: both(up_src.ctypes.data, dn_dst.ctypes.data, split))
    print("registered both ways, %d MB each, %d copies each: %.2f ms (%.1f GB/s per direction)" % (
        M >> 20, split, t * 1e3, M / t / 1e9), flush=True)
ck(hip.hipHostUnregister(up_src.ctypes.data))
ck(hip.hipHostUnregister(dn_dst.ctypes.data))
t = timeit(lambda: both(pin.value, pin.value + M, 1))
print("pinned both ways, %d MB each: %.2f ms (%.1f GB/s per direction)" % (M >> 20, t * 1e3, M / t / 1e9), flush=True)
# first touch: D2H into fresh (never written) pages
for lab in ("fresh pageable", "fresh registered"):
    buf = np.empty(M, dtype=np.uint8)
    t0 = time.perf_counter()
    if lab == "fresh registered":
        ck(hip.hipHostRegister(buf.ctypes.data, M, 0))
    t1 = time.perf_counter()
    ck(hip.hipMemcpy(buf.ctypes.data, d2.value, M, D2H))
    t2 = time.perf_counter()
    print("%s d2h %d MB: register %.2f ms, copy %.2f ms" % (lab, M >> 20, (t1 - t0) * 1e3, (t2 - t1) * 1e3), flush=True)
    if lab == "fresh registered":
        ck(hip.hipHostUnregister(buf.ctypes.data))
