"""Parity of the HIP decode path with the CPU oracles, through the C ABI.

decode_impl (reference src/huggingface/mod.rs:710-747): byte-exact UTF-8 output required.
Oracles: oracle/ref_py.py (restatement) for small inputs, oracle/ctok_ref.c (faithful C port,
checked against ref_py in tests/test_oracle.py) for large ones; at full size the
encode -> decode round trip (clean-up off) must give back the input bytes.
"""
import json

import numpy as np
import pytest

from complexity_tokenizer import Tokenizer, UnsupportedConfigError
from datagen import corpus
from oracle import ref_c, ref_py
from tests import decode_cases, edge_cases, toys

pytestmark = pytest.mark.gpu

OPTS = [(False, True), (False, False), (True, True), (True, False)]


def load(path):
    with open(path) as f:
        obj = json.load(f)
    return obj, Tokenizer.from_file(path), ref_c.RefC(obj)


@pytest.fixture(scope="module")
def gpt2(gpt2_path):
    return load(gpt2_path)


def check_batch(tok, rc, batch, skip, clean):
    got = tok.decode_batch_with_options(batch, skip, clean)
    want = rc.decode_batch(batch, skip, clean)
    bad = [i for i in range(len(batch)) if got[i] != want[i]]
    assert not bad, "doc %d (skip=%s clean=%s) ids %r: gpu %r ref %r" % (
        bad[0], skip, clean, batch[bad[0]][:20], got[bad[0]], want[bad[0]])


def test_byte_level_decode_kat():
    """reference src/decoders.rs:275-281: ["ĠHello", "Ġworld"] decodes to text containing "Hello"."""
    chars = toys.byte_chars()
    vocab = {c: i for i, c in enumerate(chars)}
    vocab["ĠHello"] = 256
    vocab["Ġworld"] = 257
    tok = Tokenizer.from_str(json.dumps(toys.tok_json(vocab, [])))
    out = tok.decode([256, 257])
    assert "Hello" in out and out == "Hello world"
    assert tok.decode_with_options([256, 257], False, False) == " Hello world"


def test_cleanup_texts_vs_oracles(gpt2):
    obj, tok, rc = gpt2
    py = ref_py.RefTokenizer(obj)
    batch = [py.encode(t) for t in decode_cases.CLEANUP_TEXTS + edge_cases.EDGE]
    for skip, clean in OPTS:
        got = tok.decode_batch_with_options(batch, skip, clean)
        want = py.decode_batch(batch, skip, clean)
        assert got == want
    # clean-up off: the round trip gives the text back (NFC-stable docs, every byte in vocab)
    raw = tok.decode_batch_with_options(batch, False, False)
    texts = decode_cases.CLEANUP_TEXTS + edge_cases.EDGE
    for t, r in zip(texts, raw):
        if ref_py.unicodedata.normalize("NFC", t) == t:
            assert r == t


@pytest.mark.parametrize("seed", [1, 2])
def test_random_ids_gpt2(gpt2, seed):
    obj, tok, rc = gpt2
    special = [v for k, v in rc.py.special_tokens.items()]
    batch = decode_cases.random_batches(len(rc.py.id_to_token_map), 3000, seed, special_ids=special)
    for skip, clean in OPTS:
        check_batch(tok, rc, batch, skip, clean)
    split = decode_cases.split_docs(batch[:500], seed)
    for skip, clean in OPTS:
        check_batch(tok, rc, split, skip, clean)


def test_multilingual_round_trip_and_split(multi_path):
    obj, tok, rc = load(multi_path)
    text, off = corpus.corpus_c5(3000, seed=5)
    docs = [d.decode() for d in corpus.unpack(text, off)]
    ids, tok_off = rc.encode_packed(text, off, 8)
    out, out_off = tok.decode_packed(ids, tok_off, False, False)
    assert np.array_equal(out_off, off.astype(np.uint64)) and out.tobytes() == text[: int(off[-1])].tobytes()
    o = tok_off.tolist()
    batch = [ids[o[i]:o[i + 1]].tolist() for i in range(len(o) - 1)]
    for skip, clean in OPTS:
        check_batch(tok, rc, batch, skip, clean)
    split = decode_cases.split_docs(batch[:400], 3)  # cuts inside multi-byte characters
    for skip, clean in OPTS:
        check_batch(tok, rc, split, skip, clean)
    rnd = decode_cases.random_batches(len(rc.py.id_to_token_map), 2000, 9)
    for skip, clean in OPTS:
        check_batch(tok, rc, rnd, skip, clean)
    assert docs  # the corpus is non-empty


def test_llama3_added_tokens_not_in_model_vocab(llama3_path):
    """Added tokens outside model.vocab are dropped by decode (Vocab::get_token, src/vocab.rs:91-93)."""
    obj, tok, rc = load(llama3_path)
    special = [a["id"] for a in obj.get("added_tokens", [])]
    batch = decode_cases.random_batches(len(rc.py.id_to_token_map), 2000, 4, special_ids=special)
    for skip, clean in OPTS:
        check_batch(tok, rc, batch, skip, clean)


def test_empty_inputs(gpt2):
    obj, tok, rc = gpt2
    assert tok.decode_batch([]) == []
    assert tok.decode_batch([[], [], []]) == ["", "", ""]
    assert tok.decode([]) == ""
    sp = tok.token_to_id("<|endoftext|>")
    assert tok.decode_with_options([sp, sp], True, True) == ""
    assert tok.decode_batch_with_options([[sp], [], [sp]], True, False) == ["", "", ""]


def test_long_runs_and_whitespace(gpt2):
    obj, tok, rc = gpt2
    py = ref_py.RefTokenizer(obj)
    texts = [" ." * 500, " - " * 300, '" ' * 400, " " * 5000, "x" + " " * 3000 + ".", "\n" * 2000 + "y" + "\t" * 999,
             "( " * 200 + "x" + " )" * 200, " - - " * 100 + "end"]
    batch = [py.encode(t) for t in texts]
    for skip, clean in OPTS:
        assert tok.decode_batch_with_options(batch, skip, clean) == py.decode_batch(batch, skip, clean)


def test_raw_and_unsupported_decoders(gpt2):
    obj, tok, rc = gpt2
    raw_obj = toys.derived(obj, lambda o: o.__setitem__("decoder", {"type": "SomethingElse"}))
    seq_obj = toys.derived(obj, lambda o: o.__setitem__("decoder", {"type": "Sequence", "decoders": [
        {"type": "ByteLevel"}, {"type": "Fuse"}]}))
    bad_obj = toys.derived(obj, lambda o: o.__setitem__("decoder", {"type": "Metaspace"}))
    batch = decode_cases.random_batches(len(rc.py.id_to_token_map), 500, 11)
    for o in (raw_obj, seq_obj):
        t = Tokenizer.from_str(json.dumps(o))
        py = ref_py.RefTokenizer(o)
        for skip, clean in OPTS:
            assert t.decode_batch_with_options(batch, skip, clean) == py.decode_batch(batch, skip, clean)
    t = Tokenizer.from_str(json.dumps(bad_obj))
    with pytest.raises(UnsupportedConfigError):
        t.decode([1, 2])
    assert t.encode("still encodes") == tok.encode("still encodes")


def test_bad_offsets_and_capacity(gpt2):
    import torch
    obj, tok, rc = gpt2
    dev = torch.device("cuda", 0)
    ids = torch.tensor([10, 20, 30, 40], dtype=torch.int32, device=dev)
    off = torch.tensor([0, 3, 2, 4], dtype=torch.int64, device=dev)  # not non-decreasing
    out = torch.empty(64, dtype=torch.uint8, device=dev)
    out_off = torch.empty(4, dtype=torch.int64, device=dev)
    with pytest.raises(ValueError):
        tok.decode_packed_device(ids.data_ptr(), off.data_ptr(), 3, 4, out.data_ptr(), 64, out_off.data_ptr())
    off = torch.tensor([0, 1, 2, 4], dtype=torch.int64, device=dev)
    with pytest.raises(ValueError, match="bytes needed"):
        tok.decode_packed_device(ids.data_ptr(), off.data_ptr(), 3, 4, out.data_ptr(), 1, out_off.data_ptr())
    need = tok.last_decode_needed
    n = tok.decode_packed_device(ids.data_ptr(), off.data_ptr(), 3, 4, out.data_ptr(), 64, out_off.data_ptr())
    assert n == need
    want = tok.decode_batch([[10], [20], [30, 40]])
    got = out[:n].cpu().numpy().tobytes()
    o = out_off.cpu().numpy().tolist()
    assert [got[o[i]:o[i + 1]].decode() for i in range(3)] == want


def test_c2_full_round_trip_and_sample(gpt2):
    """Full C2 (1M docs): encode on the GPU, decode with clean-up off gives the input back
    byte for byte (size-independent property); clean-up on matches the C oracle on a sample."""
    import torch
    obj, tok, rc = gpt2
    text, off = corpus.corpus_c2(1_000_000, seed=2)
    dev = torch.device("cuda", 0)
    n_docs, n_bytes = len(off) - 1, int(off[-1])
    d_text = torch.from_numpy(np.concatenate([text[:n_bytes], np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    cap = n_bytes + n_docs + 16
    d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
    d_tok_off = torch.empty(n_docs + 1, dtype=torch.int64, device=dev)
    ntok = tok.encode_packed_device(d_text.data_ptr(), d_off.data_ptr(), n_docs, n_bytes, d_ids.data_ptr(), cap,
                                    d_tok_off.data_ptr())
    d_out = torch.empty(n_bytes + 64, dtype=torch.uint8, device=dev)
    d_out_off = torch.empty(n_docs + 1, dtype=torch.int64, device=dev)
    nb = tok.decode_packed_device(d_ids.data_ptr(), d_tok_off.data_ptr(), n_docs, ntok, d_out.data_ptr(),
                                  n_bytes + 64, d_out_off.data_ptr(), False, False)
    assert nb == n_bytes
    assert torch.equal(d_out[:nb], d_text[:n_bytes])
    assert torch.equal(d_out_off, d_off)
    nb = tok.decode_packed_device(d_ids.data_ptr(), d_tok_off.data_ptr(), n_docs, ntok, d_out.data_ptr(),
                                  n_bytes + 64, d_out_off.data_ptr(), False, True)
    got = d_out[:nb].cpu().numpy()
    got_off = d_out_off.cpu().numpy().view(np.uint64)
    ids = d_ids[:ntok].cpu().numpy().view(np.uint32)
    toff = d_tok_off.cpu().numpy().view(np.uint64)
    k = 50_000
    want, want_off = rc.decode_packed(ids[: int(toff[k])], toff[: k + 1], False, True, 16)
    assert np.array_equal(got_off[: k + 1], want_off)
    assert got[: int(want_off[-1])].tobytes() == want.tobytes()
