#!/usr/bin/env python3
"""Per-call latency of ctok_encode_batch_device on HBM-resident C2 prefixes of several sizes
(profiling helper, not product code): wall time per call, the event-timed device span and the
sum of the kernel spans, so the fixed per-call cost (launches, host round trips) shows up."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "complexity-tokenizer_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from complexity_tokenizer import Tokenizer  # noqa: E402
from datagen import corpus  # noqa: E402
from datagen.build_tokenizers import fixture_path  # noqa: E402

tok = Tokenizer.from_file(fixture_path("gpt2_50k", "/tmp"))
text, off = corpus.corpus_c2(300_000)
for n_docs in (1, 100, 3_000, 30_000, 300_000):
    nb = int(off[n_docs])
    d_text = torch.zeros(nb + 64, dtype=torch.uint8, device="cuda")
    d_text[:nb] = torch.from_numpy(text[:nb]).cuda()
    d_off = torch.from_numpy(off[:n_docs + 1].astype(np.int64)).cuda()
    cap = nb + n_docs + 16
    d_ids = torch.empty(cap, dtype=torch.int32, device="cuda")
    d_toff = torch.empty(n_docs + 1, dtype=torch.int64, device="cuda")
    args = (d_text.data_ptr(), d_off.data_ptr(), n_docs, nb, d_ids.data_ptr(), cap, d_toff.data_ptr())
    for _ in range(3):
        tok.encode_packed_device(*args)
    ts = []
    for _ in range(20):
        t = time.perf_counter()
        tok.encode_packed_device(*args)
        ts.append(time.perf_counter() - t)
    ts.sort()
    tok.encode_packed_device(*args, timing=True)
    st = tok.last_stats
    print("docs %7d bytes %10d: wall %.3f ms  (timed call: device %.3f ms, segment %.3f, short %.3f, emit %.3f)" % (
        n_docs, nb, ts[len(ts) // 2] * 1e3, st["ms_device"], st["ms_segment"], st["ms_bpe_short"], st["ms_emit"]),
        flush=True)
