"""The host-buffer path of ctok_encode_batch: chunked H2D -> encode -> D2H pipeline through
pinned staging, and doc sharding over several devices from one process (include/ctok.h,
ctok_exec.devices / chunk_mb).  The result must not depend on the chunking or the sharding:
bit-exact vs the C oracle and vs the single-chunk, single-device run.  The GPU box has one
device, so multi-device sharding is exercised as several shards on device 0 (the same code
path: one host thread per shard, per-shard regions of the output, rebasing)."""
import ctypes
import json

import numpy as np
import pytest

from complexity_tokenizer import Tokenizer
from complexity_tokenizer import _native as _n
from datagen import corpus
from oracle import ref_c
from tests.test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpt2(gpt2_path):
    with open(gpt2_path) as f:
        obj = json.load(f)
    return Tokenizer.from_file(gpt2_path), ref_c.RefC(obj)


@pytest.fixture(scope="module")
def c2():
    return corpus.corpus_c2(100_000, seed=21)


def run(tok, text, off, devices=None, chunk_mb=0):
    tok.devices, tok.chunk_mb = devices, chunk_mb
    try:
        return tok.encode_packed(text, off, timing=True)
    finally:
        tok.devices, tok.chunk_mb = None, 0


def test_many_chunks_vs_oracle(gpt2, c2):
    tok, rc = gpt2
    text, off = c2
    ref = rc.encode_packed(text, off)
    for mb in (1, 3):  # 12.8 MB of text: 13 and 5 pipeline steps
        assert_same(*run(tok, text, off, chunk_mb=mb), *ref)
    assert tok.last_stats["tokens"] == len(ref[0])


@pytest.mark.parametrize("shards", [2, 3])
def test_shards_on_one_device(gpt2, c2, shards):
    tok, rc = gpt2
    text, off = c2
    ref = rc.encode_packed(text, off)
    assert_same(*run(tok, text, off, devices=[0] * shards, chunk_mb=2), *ref)


def test_shards_with_empty_and_tiny_batches(gpt2):
    tok, rc = gpt2
    for docs in ([], [""], ["", "", "a"], ["hello world"] * 3):
        text, off = corpus.pack([d.encode() for d in docs])
        got = run(tok, text, off, devices=[0, 0, 0, 0])
        assert_same(*got, *rc.encode_packed(text, off))


def test_one_doc_longer_than_a_chunk(gpt2):
    tok, rc = gpt2
    big = ("the quick brown fox jumps over the lazy dog " * 60000).encode()  # 2.6 MB
    docs = [b"a b", big, b"tail", big[:100000]]
    text, off = corpus.pack(docs)
    assert_same(*run(tok, text, off, chunk_mb=1), *rc.encode_packed(text, off))
    assert_same(*run(tok, text, off, devices=[0, 0], chunk_mb=1), *rc.encode_packed(text, off))


def test_nfc_growth_across_shards(gpt2):
    """NFC can grow a doc (U+0958 -> 2 code points, U+FB2C -> 3): ids can exceed bytes + docs,
    so a shard can outgrow its output region and is run again into a private buffer."""
    tok, rc = gpt2
    grow = "क़שּׁ" * 4000
    docs = ["plain ascii %d" % i for i in range(500)] + [grow] * 8 + ["x"] * 10
    text, off = corpus.pack([d.encode() for d in docs])
    ref = rc.encode_packed(text, off)
    for dev in (None, [0, 0], [0, 0, 0]):
        assert_same(*run(tok, text, off, devices=dev, chunk_mb=1), *ref)


def test_capacity_error_reports_size(gpt2, c2):
    tok, _ = gpt2
    text, off = c2
    ids, toff = tok.encode_packed(text, off)
    n_docs = len(off) - 1
    for devs in (None, [0, 0]):
        small = np.empty(len(ids) - 1, dtype=np.uint32)
        out_off = np.empty(n_docs + 1, dtype=np.uint64)
        ex = _n.Exec(0, None, 0)
        if devs:
            arr = (ctypes.c_int * len(devs))(*devs)
            ex.devices, ex.n_devices = ctypes.cast(arr, ctypes.POINTER(ctypes.c_int)), len(devs)
        rc = _n.lib.ctok_encode_batch(tok._h, text.ctypes.data, off.ctypes.data, n_docs, small.ctypes.data,
                                      len(small), out_off.ctypes.data, ctypes.byref(ex), None)
        assert rc == _n.CTOK_E_CAPACITY
        assert int(out_off[-1]) == len(ids)
        # exact capacity succeeds, also when the per-shard regions do not fit (private buffers)
        exact = np.empty(len(ids), dtype=np.uint32)
        rc = _n.lib.ctok_encode_batch(tok._h, text.ctypes.data, off.ctypes.data, n_docs, exact.ctypes.data,
                                      len(exact), out_off.ctypes.data, ctypes.byref(ex), None)
        assert rc == _n.CTOK_OK
        assert np.array_equal(exact, ids) and np.array_equal(out_off, toff)


def test_shards_over_every_visible_device(gpt2, c2):
    """ctok_exec.devices = every visible device (one shard per GPU, one host thread each, each
    thread making its device current); on a 1-GPU box this is one shard, on a node all of them."""
    tok, rc = gpt2
    text, off = c2
    n = _n.lib.ctok_device_count()
    assert n >= 1
    devs = list(range(n))
    assert_same(*run(tok, text, off, devices=devs, chunk_mb=4), *rc.encode_packed(text, off))
    assert_same(*run(tok, text, off, devices=devs + devs, chunk_mb=4), *rc.encode_packed(text, off))
