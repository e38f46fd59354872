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
text, off = corpus.corpus_c2()
n_docs, nb = len(off) - 1, int(off[-1])
cap = nb + n_docs + 16
ids = np.empty(cap, dtype=np.uint32)
ids[:] = 0
toff = np.empty(n_docs + 1, dtype=np.uint64)


def call(ids_buf, threads=0, chunk=0):
    ex = _n.Exec(0, None, 0)
    ex.host_threads = threads
    ex.chunk_mb = chunk
    t = time.perf_counter()
    rc = _n.lib.ctok_encode_batch(tok._h, text.ctypes.data, off.ctypes.data, n_docs, ids_buf.ctypes.data, cap,
                                  toff.ctypes.data, ctypes.byref(ex), None)
    assert rc == 0, _n.last_error()
    return time.perf_counter() - t


for _ in range(3):
    call(ids)
for label, fresh, th, ch in [("reused", False, 0, 0), ("fresh", True, 0, 0), ("reused_t16", False, 16, 0),
                             ("reused_t32", False, 32, 0), ("reused_c64", False, 0, 64), ("reused_c16", False, 0, 16)]:
    ts = []
    for _ in range(5):
        buf = np.empty(cap, dtype=np.uint32) if fresh else ids
        ts.append(call(buf, th, ch))
    ts.sort()
    print("%-12s %.2f ms  %.0f MB/s" % (label, ts[2] * 1e3, nb / ts[2] / 1e6), flush=True)
