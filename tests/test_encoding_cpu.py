"""CPU tests of the Encoding path's host side: the reference's known-answer tests for Encoding
(src/encoding.rs:462-577) and the post-processors (src/postprocessors.rs:294-356) on both the
oracle and the product's Encoding class, the two Encoding classes against each other under
random pad / truncate sequences, and the loader's post-processor compilation (no GPU needed)."""
import json
import random

import pytest

from complexity_tokenizer import Encoding, PanicException, Tokenizer
from complexity_tokenizer import _native as _n
from oracle import ref_py
from tests import encoding_cases


def test_kat_encoding_from_ids():
    e = Encoding.from_ids([1, 2, 3], ["a", "b", "c"])
    assert len(e) == 3 and e.attention_mask == [1, 1, 1] and e.type_ids == [0, 0, 0]
    assert e.sequence_ids == [0, 0, 0]


def test_kat_padding():
    e = Encoding.from_ids([1, 2], ["a", "b"])
    e.pad(5, 0, "<pad>", False)
    assert len(e) == 5 and e.attention_mask == [1, 1, 0, 0, 0]
    assert e.sequence_ids == [0, 0, None, None, None]


def test_kat_truncation():
    e = Encoding.from_ids([1, 2, 3, 4, 5], list("abcde"))
    e.truncate(3)
    assert len(e) == 3 and e.n_overflowing == 1 and len(e.overflowing[0]) == 2


def test_kat_char_and_word_lookups():
    e = Encoding.from_ids([1, 2, 3], ["hello", " ", "world"])
    e._offsets = [(0, 5), (5, 6), (6, 11)]
    assert [e.char_to_token(i) for i in (0, 4, 5, 6, 11)] == [0, 0, 1, 2, None]
    assert e.token_to_chars(1) == (5, 6) and e.token_to_chars(3) is None
    w = Encoding.from_ids([1, 2, 3, 4], ["hel", "lo", "wor", "ld"])
    w._word_ids = [0, 0, 1, 1]
    w._offsets = [(0, 3), (3, 5), (6, 9), (9, 11)]
    assert w.word_to_tokens(0) == (0, 2) and w.word_to_tokens(1) == (2, 4) and w.word_to_tokens(2) is None
    assert w.word_to_chars(0) == (0, 5) and w.word_to_chars(1) == (6, 11)
    assert w.n_words == 2


def test_kat_post_processors():
    assert ref_py.process_post(("bert", 101, 102), [1, 2, 3]) == [101, 1, 2, 3, 102]
    assert ref_py.process_post(("roberta", 0, 2), [1, 2, 3]) == [0, 1, 2, 3, 2]


def _pair(rng):
    n = rng.randrange(0, 12)
    ids = [rng.randrange(100) for _ in range(n)]
    toks = ["t%d" % i for i in ids][: max(0, n - rng.randrange(0, 3))]  # tokens may be shorter
    extra = rng.randrange(0, 3)
    args = (ids + [7] * extra, [0] * (n + extra), toks, [1] * (n + extra), [0] * n + [1] * extra, [0] * n)
    mine = Encoding(*[list(a) for a in args[:5]], [], [], list(args[5]))
    return mine, ref_py.RefEncoding(*[list(a) for a in args])


def test_encoding_ops_match_oracle_deterministic():
    rng = random.Random(11)
    for _ in range(300):
        mine, ref = _pair(rng)
        ops = [(rng.choice(["pad", "truncate", "stride"]), rng.randrange(1, 14), rng.random() < 0.5)
               for _ in range(3)]
        for op, m, left in ops:
            res = []
            for obj, exc in ((mine, PanicException), (ref, ref_py.PanicException)):
                try:
                    if op == "pad":
                        obj.pad(m, 0, "<pad>", left)
                    elif op == "truncate":
                        obj.truncate(m)
                    else:
                        obj.truncate_with_stride(m, m // 2)
                    res.append("ok")
                except exc:
                    res.append("panic")
            assert res[0] == res[1], (op, m)
            if res[0] == "panic":
                break
            d = ref.as_dict()
            assert mine.ids == d["ids"] and mine.tokens == d["tokens"] and mine.type_ids == d["type_ids"]
            assert mine.attention_mask == d["attention_mask"]
            assert mine.special_tokens_mask == d["special_tokens_mask"]
            assert mine.sequence_ids == d["sequence_ids"]
            assert [o.ids for o in mine.overflowing] == [o["ids"] for o in d["overflowing"]]


@pytest.mark.parametrize("kind,items,n_single", [
    ("template", ["<|bos|>", "A", "[SEP]"], 2), ("template_twice", ["A", "[CLS]", "A"], 2),
    ("bert", ["[CLS]", "A", "[SEP]"], 2), ("roberta", ["<s>", "A", "</s>"], 2),
    ("template_no_a", ["[CLS]"], 1), ("sequence", None, 0), ("none", None, 0)])
def test_loader_post_processor(gpt2_path, kind, items, n_single):
    with open(gpt2_path) as f:
        obj = encoding_cases.with_post_processor(json.load(f), kind)
    tok = Tokenizer.from_str(json.dumps(obj))
    sp = {a["content"]: a["id"] for a in obj["added_tokens"] if a["special"]}
    want = None if items is None else [_n.CTOK_PP_SEQUENCE if i == "A" else sp[i] for i in items]
    assert tok._pp_items() == want
    assert tok.num_special_tokens_to_add(False) == n_single
    assert tok.model_max_length == 512
    ref = ref_py.RefTokenizer(obj)
    assert tok._pad_id_token()[0] == ref.pad_id_token()[0]


def test_kat_words_with_offsets():
    """pre_tokenize_with_offsets (src/huggingface/mod.rs:448-480) on hand-checked cases: find after
    the leading 'Ġ' is trimmed, the byte-length fallback for words not in the text, the panic on a
    fallback that ends inside a UTF-8 character."""
    w = ref_py.RefTokenizer.words_with_offsets
    assert [x[1:] for x in w(["hello", "\u0120world"], "hello world")] == [(0, 5), (6, 11)]
    # '\n' -> 'Ċ' (2 bytes) is not in the text: start at the search point, end clipped
    assert [x[1:] for x in w(["a", "\u010a", "b"], "a\nb")] == [(0, 1), (1, 3), (3, 3)]
    with pytest.raises(ref_py.PanicException):
        w(["\u00c3\u00a9", "\u00e2\u0082\u00ac"], "\u00e9\u20ac")
