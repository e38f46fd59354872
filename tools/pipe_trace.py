#!/usr/bin/env python3
"""One traced host-buffer call on C2 (CTOK_PIPE_TRACE=1 prints the pipeline's per-chunk events)."""
import ctypes
import os
import sys

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
ids = np.zeros(cap, dtype=np.uint32)
toff = np.empty(n_docs + 1, dtype=np.uint64)
for i in range(4):
    if i == 3:
        print("---- traced call", file=sys.stderr, flush=True)
    ex = _n.Exec(0, None, 0)
    rc = _n.lib.ctok_encode_batch(tok._h, text.ctypes.data, off.ctypes.data, n_docs, ids.ctypes.data, cap,
                                  toff.ctypes.data, ctypes.byref(ex), None)
    assert rc == 0
