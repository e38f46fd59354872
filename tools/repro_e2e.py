#!/usr/bin/env python3
"""Host-buffer encode (ctok_encode_batch) of a corpus sample in small chunks, checked against the
device path (debugging helper, not product code).  usage: repro_e2e.py CONFIG N_DOCS CHUNK_MB"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "complexity-tokenizer_amd")]
import numpy as np  # noqa: E402

from complexity_tokenizer import Tokenizer, _native as _n  # noqa: E402
from datagen import corpus  # noqa: E402
from datagen.build_tokenizers import fixture_path  # noqa: E402

cfg, n_docs, chunk = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
fx = {"c2": "gpt2_50k", "c5": "multi_32k", "c5nfc": "multi_32k", "c3": "llama3_128k"}[cfg]
tok = Tokenizer.from_file(fixture_path(fx, "/tmp"))
gen = {"c2": corpus.corpus_c2, "c5": corpus.corpus_c5, "c5nfc": corpus.corpus_c5nfc, "c3": corpus.corpus_c3}[cfg]
text, off = gen(n_docs)
n_docs = len(off) - 1
print("corpus", n_docs, int(off[-1]), flush=True)
if len(sys.argv) > 4 and sys.argv[4] == "device_first":  # as tools/bench_matrix.py: the device path on a torch stream first
    import torch
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    nb = int(off[-1])
    d_text = torch.zeros(nb + 64, dtype=torch.uint8, device=dev)
    d_text[:nb] = torch.from_numpy(text).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    dcap = 3 * nb + n_docs + 16
    d_ids = torch.empty(dcap, dtype=torch.int32, device=dev)
    d_tok = torch.empty(n_docs + 1, dtype=torch.int64, device=dev)
    for _ in range(5):
        n = tok.encode_packed_device(d_text.data_ptr(), d_off.data_ptr(), n_docs, nb, d_ids.data_ptr(), dcap,
                                     d_tok.data_ptr(), stream=stream.cuda_stream, timing=True)
    print("device path tokens", n, flush=True)
    del d_text, d_off, d_ids, d_tok
    torch.cuda.empty_cache()
cap = int(off[-1]) * 3 + n_docs + 16
ids = np.zeros(cap, dtype=np.uint32)
toff = np.zeros(n_docs + 1, dtype=np.uint64)
ex = _n.Exec(0, None, 0)
ex.chunk_mb = chunk
for i in range(5):
    rc = _n.lib.ctok_encode_batch(tok._h, text.ctypes.data, off.ctypes.data, n_docs, ids.ctypes.data, cap,
                                  toff.ctypes.data, ctypes.byref(ex), None)
    print("host path rc", rc, _n.last_error() if rc else "", flush=True)
    assert rc == 0
ref_ids, ref_off = tok.encode_packed(text, off)  # (the same host path, default chunk)
print("tokens", int(toff[-1]), int(ref_off[-1]), flush=True)
assert np.array_equal(toff, ref_off) and np.array_equal(ids[:int(toff[-1])], ref_ids)
print("ok", flush=True)
