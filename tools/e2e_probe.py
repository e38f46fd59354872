#!/usr/bin/env python3
"""E2E host-buffer encode (ctok_encode_batch) on C2: fresh vs reused output buffers, host thread
counts and chunk sizes (profiling helper, not product code)."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "complexity-tokenizer_amd")]
import numpy as np  # noqa: E402

from complexity_tokenizer import Tokenizer, _native as _n  # noqa: E402
from datagen import corpus  # noqa: E402
from datagen.build_tokenizers import fixture_path  # noqa: E402

tok = Tokenizer.from_file(fixture_path("gpt2_50k", "/tmp"))
print("lib", _n.lib._name, flush=True)
text, off = corpus.corpus_c2()
n_docs, nb = len(off) - 1, int(off[-1])
cap = nb + n_docs + 16
ids = np.empty(cap, dtype=np.uint32)
ids[:] = 0
toff = np.empty(n_docs + 1, dtype=np.uint64)


def call(ids_buf, threads=0, chunk=0, stats=False):
    ex = _n.Exec(0, None, 0)
    ex.host_threads = threads
    ex.chunk_mb = chunk
    st = _n.Stats()
    t = time.perf_counter()
    rc = _n.lib.ctok_encode_batch(tok._h, text.ctypes.data, off.ctypes.data, n_docs, ids_buf.ctypes.data, cap,
                                  toff.ctypes.data, ctypes.byref(ex), ctypes.byref(st) if stats else None)
    assert rc == 0, _n.last_error()
    return time.perf_counter() - t


for _ in range(3):
    call(ids)
for label, fresh, th, ch, stt in [("reused", False, 0, 0, False), ("fresh", True, 0, 0, False),
                                  ("reused_stats", False, 0, 0, True), ("fresh_stats", True, 0, 0, True),
                                  ("reused_c8", False, 0, 8, False), ("reused_c16", False, 0, 16, False),
                                  ("reused_c64", False, 0, 64, False), ("reused_t4", False, 4, 0, False),
                                  ("reused_t16", False, 16, 0, False), ("fresh_t16", True, 16, 0, False)]:
    ts = []
    for _ in range(5):
        buf = np.empty(cap, dtype=np.uint32) if fresh else ids
        ts.append(call(buf, th, ch, stt))
    ts.sort()
    print("%-12s %.2f ms  %.0f MB/s" % (label, ts[2] * 1e3, nb / ts[2] / 1e6), flush=True)
ex = _n.Exec(0, None, 0)
ex.flags = 1  # CTOK_F_TIMING
st = _n.Stats()
for _ in range(2):
    t = time.perf_counter()
    rc = _n.lib.ctok_encode_batch(tok._h, text.ctypes.data, off.ctypes.data, n_docs, ids.ctypes.data, cap,
                                  toff.ctypes.data, ctypes.byref(ex), ctypes.byref(st))
    t = time.perf_counter() - t
print("timed call %.2f ms: first-chunk h2d %.2f ms, last-chunk d2h %.2f ms, device %.2f ms" % (
    t * 1e3, st.ms_h2d, st.ms_d2h, st.ms_device), flush=True)
ts = []
for _ in range(5):
    t = time.perf_counter()
    tok.encode_packed(text, off)
    ts.append(time.perf_counter() - t)
ts.sort()
print("%-12s %.2f ms  %.0f MB/s" % ("encode_packed", ts[2] * 1e3, nb / ts[2] / 1e6), flush=True)

# encode_packed step by step
import ctypes as C
for rep in range(3):
    t0 = time.perf_counter()
    cap2 = int(nb + n_docs + 16)
    ids2 = np.empty(max(cap2, 1), dtype=np.uint32)
    toff2 = np.empty(n_docs + 1, dtype=np.uint64)
    ex = tok._host_exec(False)
    st = _n.Stats()
    t1 = time.perf_counter()
    rc = _n.lib.ctok_encode_batch(tok._h, text.ctypes.data, off.ctypes.data, n_docs, ids2.ctypes.data, cap2,
                                  toff2.ctypes.data, C.byref(ex), C.byref(st))
    t2 = time.perf_counter()
    print("steps: alloc %.2f ms, call %.2f ms, ex=%s dev=%s devices=%s chunk=%s threads=%s" % (
        (t1 - t0) * 1e3, (t2 - t1) * 1e3, ex.device, tok.device, tok.devices, ex.chunk_mb, ex.host_threads), flush=True)
