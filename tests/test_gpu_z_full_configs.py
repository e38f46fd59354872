"""Whole benchmark configs on the GPU against the C oracle's golden digests (tests/golden/digests.json,
sha256 over tok_off u64 LE + ids u32 LE, made by tests/golden/make_golden.py from oracle/ctok_ref.c):
C2 (1M docs, GPT-2-shaped 50k), C5 (1M multilingual docs, 32k) and C5-NFC (C5 with NFC-active
text in 3% of the docs: the NFC splice, ctok_host.cpp nfc_splice).  C3 / C3TT / C4 run whole in
tests/test_gpu_parity.py and tests/test_gpu_c4.py.

Each corpus is built by a background process started when the session collected these tests
(tests/conftest.py, datagen/cache.py); the file sorts last among the GPU tests so that the build
overlaps the others.  Every config runs once through the device-resident path (the bench's) and
once through the host-buffer C ABI (ctok_encode_batch, chunked pipeline)."""
import hashlib
import json
import os

import numpy as np
import pytest

from complexity_tokenizer import Tokenizer
from datagen import cache

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))


def digest(ids, tok_off):
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(tok_off, dtype="<u8").tobytes())
    h.update(np.ascontiguousarray(ids, dtype="<u4").tobytes())
    return h.hexdigest()


def _encode_device(tok, text, off):
    import torch
    dev = torch.device("cuda", 0)
    n_docs, n_bytes = len(off) - 1, int(off[-1])
    d_text = torch.zeros(n_bytes + 16, dtype=torch.uint8, device=dev)
    d_text[:n_bytes].copy_(torch.from_numpy(text[:n_bytes]))
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    cap = 2 * n_bytes + n_docs + 16  # (NFC can grow the text)
    d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
    d_tok_off = torch.empty(n_docs + 1, dtype=torch.int64, device=dev)
    ntok = tok.encode_packed_device(d_text.data_ptr(), d_off.data_ptr(), n_docs, n_bytes, d_ids.data_ptr(), cap,
                                    d_tok_off.data_ptr(), device=0)
    torch.cuda.synchronize(dev)
    ids = d_ids[:ntok].cpu().numpy().view(np.uint32)
    toff = d_tok_off.cpu().numpy().view(np.uint64)
    del d_text, d_off, d_ids, d_tok_off
    torch.cuda.empty_cache()
    return ids, toff


@pytest.mark.timeout(900)
@pytest.mark.parametrize("cfg", ["C2", "C5", "C5NFC"])
def test_full_config_digest(request, cfg):
    gold = GOLD[cfg]
    path = request.getfixturevalue({"gpt2_50k": "gpt2_path", "multi_32k": "multi_path"}[gold["tokenizer"]])
    tok = Tokenizer.from_file(path)
    tok.device = 0
    text, off = cache.wait_load(cache.default_dir(), cfg)
    assert len(off) - 1 == gold["docs"] and int(off[-1]) == gold["bytes"]
    ids, toff = _encode_device(tok, text, off)
    assert len(ids) == gold["tokens"], cfg
    assert digest(ids, toff) == gold["sha256"], "%s (device path) differs from the C-oracle digest" % cfg
    # the first 100k documents against the Python restatement's digest (regex + unicodedata, not
    # the generated tables the C oracle shares with the product: make_golden.py pin_ref_py)
    pin = gold["pin_ref_py"]
    n = pin["docs"]
    assert digest(ids[: int(toff[n])], toff[: n + 1]) == pin["sha256"], "%s: first %d docs differ from ref_py" % (cfg, n)
    if cfg == "C5NFC":
        assert tok.last_stats["nfc_docs"] > 0
    elif cfg == "C5":  # no NFC-active text: nothing flagged (a false flag costs a splice, round 4)
        assert tok.last_stats["nfc_docs"] == 0
    ids, toff = tok.encode_packed(text, off)
    assert digest(ids, toff) == gold["sha256"], "%s (host-buffer path) differs from the C-oracle digest" % cfg
