"""CPU side of the added-token split (src/huggingface/mod.rs:566-675).

1. The load-time predicate that keeps an added token for the device split only when it can
   occur inside one GPT2_PATTERN piece (ctok_piece_can_contain) is sound against the `regex`
   module: whenever some piece of a probe text contains the token's raw bytes, the predicate
   says yes.  A wrong "no" would silently drop a token from the GPU split.
2. The loader keeps every token of the tests/added_cases.py variants (they are all reachable).
3. The two oracles (ref_py, ctok_ref.c) agree on every variant and text set the GPU tests use.
"""
import itertools
import json
import random

import pytest

from complexity_tokenizer import Tokenizer
from complexity_tokenizer import _native
from datagen import corpus
from oracle import ref_c, ref_py
from tests import added_cases, edge_cases

CONTEXTS = ["", " ", "  ", "a", "Z", "1", ".", "'", "\n", "\t", "é", "世", "😀", " a", "a ", "'s", "x'", " "]


def can_contain(raw: bytes) -> bool:
    r = _native.lib.ctok_piece_can_contain(raw, len(raw))
    assert r in (0, 1)
    return r == 1


def regex_reachable(raw: bytes) -> bool:
    """Does some piece of c1 + raw + c2 contain raw, for contexts c1, c2?"""
    try:
        s = raw.decode("utf-8")
    except UnicodeDecodeError:
        return True  # a partial code point: the predicate keeps those (unknown class)
    py = ref_py.RefTokenizer.__new__(ref_py.RefTokenizer)
    py.pre_tokenizer = ("ByteLevel", False)
    for c1, c2 in itertools.product(CONTEXTS, CONTEXTS):
        text = c1 + s + c2
        if any(raw in p for p in py.pieces(text)):
            return True
    return False


def candidates(seed, n):
    rng = random.Random(seed)
    alpha = ["a", "b", "Z", "1", "9", " ", "  ", "\n", "\t", "'", ".", "!", "-", "é", "世", "😀", " ", "s",
             "t", "re", "ll", "d", "m", "ve"]
    out = set()
    for _ in range(n):
        out.add("".join(rng.choice(alpha) for _ in range(rng.randint(1, 4))))
    out |= {"<|endoftext|>", "[CLS]", "<s>", "ing", " the", "'s", "'ll", "s'", "a b", " 1", "1a", "..", " \n",
            "\n ", "  x", "x ", "'", "''", "'t", "'re", "e'", "😀😀", " 😀", "世界", " 世"}
    return sorted(out)


def test_predicate_is_sound_vs_regex():
    for cand in candidates(1, 600):
        raw = cand.encode()
        if regex_reachable(raw):
            assert can_contain(raw), repr(cand)


def test_predicate_rejects_bracketed_specials():
    for s in ["<|endoftext|>", "[CLS]", "<s>", "</s>", "<|reserved_special_token_0|>", "a b", "x ", "1a", "a.",
              "'s'", "s'"]:
        assert not can_contain(s.encode()), s
        assert not regex_reachable(s.encode()), s


@pytest.fixture(scope="module")
def gpt2_obj(gpt2_path):
    with open(gpt2_path) as f:
        return json.load(f)


@pytest.mark.parametrize("variant", sorted(added_cases.VARIANTS))
def test_loader_keeps_variant_tokens(gpt2_obj, variant):
    tok = Tokenizer.from_str(json.dumps(added_cases.with_added(gpt2_obj, variant)))
    distinct = {c for c, *_ in added_cases.VARIANTS[variant]}
    base = {a["content"] for a in gpt2_obj.get("added_tokens", [])}
    kept = tok.num_piece_added_tokens()
    # every variant token is reachable inside a piece; the fixture's own specials are not
    assert kept == len(distinct - base), (kept, distinct)


@pytest.mark.parametrize("variant", sorted(added_cases.VARIANTS))
def test_two_oracles_agree(gpt2_obj, variant):
    obj = added_cases.with_added(gpt2_obj, variant)
    py = ref_py.RefTokenizer(obj)
    rc = ref_c.RefC(obj)
    docs = (added_cases.short_docs(300, seed=sum(map(ord, variant))) + added_cases.long_piece_docs(3, lengths=(33, 100, 700))
            + edge_cases.EDGE)
    assert rc.encode_batch(docs) == py.encode_batch(docs)
    # the split actually fired: an added id appears
    nid = max(gpt2_obj["model"]["vocab"].values()) + 1
    assert any(i >= nid for ids in py.encode_batch(docs[:300]) for i in ids)


def test_first_occurrence_only(gpt2_obj):
    """find_added_token checks the flags at the first occurrence only (mod.rs:637-675), on
    byte-mapped chars.  With single_word "ab": "éab" is one letter piece, mapped "Ã©ab", and '©'
    (U+00A9) is not alphanumeric, so "ab" matches; in "xabéab" the first "ab" follows 'x' and
    fails, so the token is not found at all although its second occurrence would pass."""
    obj = added_cases.with_added(gpt2_obj, "single_word")
    py = ref_py.RefTokenizer(obj)
    rc = ref_c.RefC(obj)
    ab = py.added_tokens["ab"]
    assert ab in py.encode("ab")
    assert ab in py.encode("x-ab")
    assert ab in py.encode("éab")
    assert ab not in py.encode("xabéab")
    assert ab not in py.encode("abxab")  # first occurrence at 0 fails: 'x' follows
    for s in ["ab", "x-ab", "éab", "xabéab", "abxab", "ab ab", "ab-ab"]:
        assert py.encode(s) == rc.encode_batch([s])[0], s
