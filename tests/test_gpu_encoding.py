"""Padded batch encode and Encoding objects through the C ABI against the
Python oracle (oracle/ref_py.py encode_to_encoding / encode_from_ids / call, a restatement of
src/huggingface/mod.rs:340-545, src/encoding.rs, src/postprocessors.rs).  Ids, type ids,
tokens, attention / special masks, sequence ids and overflowing windows must be identical."""
import json

import numpy as np
import pytest

from complexity_tokenizer import PanicException, Tokenizer
from oracle import ref_py
from tests import encoding_cases

pytestmark = pytest.mark.gpu

KINDS = ["template", "template_twice", "bert", "roberta", "sequence", "none"]


@pytest.fixture(scope="module")
def base(gpt2_path):
    with open(gpt2_path) as f:
        return json.load(f)


def pair_of(obj):
    return Tokenizer.from_str(json.dumps(obj)), ref_py.RefTokenizer(obj)


def enc_dict(e):
    return {"ids": e.ids, "type_ids": e.type_ids, "tokens": e.tokens, "attention_mask": e.attention_mask,
            "special_tokens_mask": e.special_tokens_mask, "sequence_ids": e.sequence_ids,
            "overflowing": [enc_dict(o) for o in e.overflowing]}


def same(got, want, what):
    for k, (g, w) in enumerate(zip(got, want)):
        assert enc_dict(g) == w.as_dict(), "%s: encoding %d differs" % (what, k)
    assert len(got) == len(want)


@pytest.mark.parametrize("kind", KINDS)
def test_encode_batch_to_encoding(base, kind):
    tok, ref = pair_of(encoding_cases.with_post_processor(base, kind))
    ts = encoding_cases.texts()
    same(tok.encode_batch_to_encoding(ts), [ref.encode_to_encoding(t) for t in ts], kind)
    assert tok.num_special_tokens_to_add() == {"template": 2, "template_twice": 2, "bert": 2, "roberta": 2}.get(kind, 0)


@pytest.mark.parametrize("kind", ["template", "bert", "none"])
def test_pairs(base, kind):
    tok, ref = pair_of(encoding_cases.with_post_processor(base, kind))
    ts = encoding_cases.texts()
    prs = list(zip(ts, reversed(ts)))
    same(tok.encode_batch_pairs_to_encoding(prs), [ref.encode_to_encoding(a, b) for a, b in prs], kind)
    e = tok.encode_pair_to_encoding("first part", "second part")
    assert enc_dict(e) == ref.encode_to_encoding("first part", "second part").as_dict()


@pytest.mark.parametrize("kind", ["template", "roberta", "none"])
@pytest.mark.parametrize("opts", [dict(), dict(padding="longest"), dict(padding="max_length", max_length=24),
                                  dict(truncation=True, max_length=7), dict(truncation=True, max_length=9, stride=3),
                                  dict(padding="left"), dict(add_special_tokens=False, padding="longest"),
                                  dict(add_special_tokens=False, truncation=True, max_length=5)])
def test_call_batch(base, kind, opts):
    tok, ref = pair_of(encoding_cases.with_post_processor(base, kind))
    ts = encoding_cases.texts()
    try:
        want = ref.call(ts, **opts)
    except ref_py.PanicException:
        with pytest.raises(PanicException):
            tok(ts, **opts).encodings()
        return
    got = tok(ts, **opts)
    same(got.encodings(), want, "%s %s" % (kind, opts))
    assert got.input_ids == [w.ids for w in want]
    assert got.keys() == ["input_ids", "attention_mask", "token_type_ids"]


def test_call_pairs_and_single(base):
    tok, ref = pair_of(encoding_cases.with_post_processor(base, "bert"))
    ts = encoding_cases.texts()
    got = tok(ts, text_pair=ts[::-1], padding="longest", truncation=True, max_length=30)
    same(got.encodings(), ref.call(ts, pairs=ts[::-1], padding="longest", truncation=True, max_length=30), "pairs")
    one = tok("hello world", padding="max_length", max_length=8)
    want = ref.call(["hello world"], padding="max_length", max_length=8)
    same(one.encodings(), want, "single")
    with pytest.raises(TypeError):
        tok(123)


@pytest.mark.parametrize("kind", ["template", "bert", "none"])
def test_encode_padded_arrays(base, kind):
    tok, ref = pair_of(encoding_cases.with_post_processor(base, kind))
    ts = encoding_cases.texts()
    for opts in (dict(padding="longest"), dict(padding="max_length", max_length=40, truncation=True),
                 dict(padding="longest", pad_left=True, truncation=True, max_length=12)):
        r = tok.encode_padded(ts, **opts)
        ml = opts.get("max_length", 512)
        want = [ref.encode_to_encoding(t) for t in ts]
        for e in want:
            if opts.get("truncation") and len(e.ids) > ml:
                e.truncate(ml)
        target = ml if opts["padding"] == "max_length" else max(len(e.ids) for e in want)
        pid, ptok = ref.pad_id_token()
        for e in want:
            e.pad(target, pid, ptok, opts.get("pad_left", False))
        for i, e in enumerate(want):
            L = int(r["row_len"][i])
            assert L == len(e.ids)
            assert r["input_ids"][i, :L].tolist() == e.ids
            assert r["attention_mask"][i, :L].tolist() == e.attention_mask
            assert r["token_type_ids"][i, :L].tolist() == e.type_ids
            assert r["special_tokens_mask"][i, :L].tolist() == e.special_tokens_mask


def test_encode_batch_with_padding(base):
    tok, ref = pair_of(encoding_cases.with_post_processor(base, "template"))
    ts = encoding_cases.texts()
    for ml, left in ((None, False), (50, True), (3, False)):
        got = tok.encode_batch_with_padding(ts, max_length=ml, pad_left=left)
        want = [ref.encode_to_encoding(t) for t in ts]
        target = ml if ml is not None else max(len(e.ids) for e in want)
        pid, ptok = ref.pad_id_token()
        for e in want:
            e.pad(target, pid, ptok, left)
        same(got, want, "padding %r %r" % (ml, left))


def test_truncation_panics_like_the_reference(base):
    """tokens are not extended by the post-processor, so truncating between the token count and
    the id count slices past the end of tokens: a panic in the reference."""
    tok, ref = pair_of(encoding_cases.with_post_processor(base, "bert"))
    e = tok.encode_to_encoding("hello world")
    n_tokens = len(e.tokens)
    assert len(e.ids) == n_tokens + 2
    with pytest.raises(ref_py.PanicException):
        ref.encode_to_encoding("hello world").truncate(n_tokens + 1)
    with pytest.raises(PanicException):
        e.truncate(n_tokens + 1)


def test_template_without_sequence(base):
    tok, ref = pair_of(encoding_cases.with_post_processor(base, "template_no_a"))
    assert tok.encode_to_encoding("").ids == ref.encode_to_encoding("").ids
    with pytest.raises(PanicException):
        tok.encode_batch_to_encoding(["hello there world"])
    with pytest.raises(ref_py.PanicException):
        ref.encode_to_encoding("hello there world")


def test_special_mask_helpers(base):
    tok, ref = pair_of(encoding_cases.with_post_processor(base, "bert"))
    ids = tok.encode_to_encoding("hi there").ids
    assert tok.get_special_tokens_mask(ids) == [0] * len(ids)  # specials outside model.vocab
    assert tok.get_special_tokens_mask(ids, already_has_special_tokens=False) == [0] * len(ids)
    arr = tok.encode_padded(["a b", "c"], padding="longest")
    assert arr["input_ids"].dtype == np.uint32 and arr["input_ids"].shape[0] == 2
