"""GPU added-token split against both oracles.

Reference: src/huggingface/mod.rs:566-610 (the word loop), :616-634
(find_next_added_token_in_word), :637-675 (find_added_token).  Every variant of
tests/added_cases.py has tokens that match inside pieces, so the HIP path runs its added-token
split in all three places: k_bpe_generic (pieces <= 32 B, thread per piece), k_bpe_long<false>
(33..2048 B, LDS linked list) and k_bpe_long<true> (> 2048 B, global-memory list).
"""
import json

import pytest

from complexity_tokenizer import Tokenizer
from datagen import corpus
from oracle import ref_c, ref_py
from tests import added_cases
from tests.test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def base(gpt2_path):
    with open(gpt2_path) as f:
        return json.load(f)


def run(obj, docs, py_check=200):
    tok = Tokenizer.from_str(json.dumps(obj))
    assert tok.num_piece_added_tokens() > 0  # the split really runs on the GPU
    rc = ref_c.RefC(obj)
    text, off = corpus.pack([d.encode() for d in docs])
    ids, toff = tok.encode_packed(text, off, timing=True)
    assert_same(ids, toff, *rc.encode_packed(text, off))
    py = ref_py.RefTokenizer(obj)
    for i in range(min(py_check, len(docs))):
        if len(docs[i]) > 1200:  # the Python merge loop is quadratic: long pieces vs the C oracle only
            continue
        assert ids[toff[i]:toff[i + 1]].tolist() == py.encode(docs[i]), repr(docs[i])
    return tok.last_stats, ids


@pytest.mark.parametrize("variant", sorted(added_cases.VARIANTS))
def test_added_short_pieces(base, variant):
    obj = added_cases.with_added(base, variant)
    docs = added_cases.short_docs(4000, seed=sum(map(ord, variant)))
    _, ids = run(obj, docs)
    nid = max(base["model"]["vocab"].values()) + 1
    assert (ids >= nid).any()  # some added token was emitted


@pytest.mark.parametrize("variant", sorted(added_cases.VARIANTS))
def test_added_long_pieces(base, variant):
    obj = added_cases.with_added(base, variant)
    docs = added_cases.long_piece_docs(seed=3)
    st, _ = run(obj, docs, py_check=len(docs))
    assert st["long_pieces"] > 0


def test_added_special_flag_and_edges(base):
    # special=True changes nothing on the encode path; edge docs (empty, NFC-free unicode,
    # contractions) go through the same split
    from tests import edge_cases
    obj = added_cases.with_added(base, "mixed", special=True)
    docs = edge_cases.EDGE + added_cases.short_docs(500, seed=9)
    run(obj, docs, py_check=len(docs))


def test_added_c2_sample(base):
    # English-like text with "ing" / "ll" / "the" inside most words
    obj = added_cases.with_added(base, "plain")
    text, off = corpus.corpus_c2(20_000, seed=21)
    tok = Tokenizer.from_str(json.dumps(obj))
    ids, toff = tok.encode_packed(text, off)
    assert_same(ids, toff, *ref_c.RefC(obj).encode_packed(text, off))
