"""Padded batch encode and Encoding objects through the C ABI against the
Python oracle (oracle/ref_py.py encode_to_encoding / encode_from_ids / call, a restatement of
src/huggingface/mod.rs:340-545, src/encoding.rs, src/postprocessors.rs).  Ids, type ids,
tokens, attention / special masks, sequence ids and overflowing windows must be identical."""
import json

import numpy as np
import pytest

from complexity_tokenizer import PanicException, Tokenizer
from oracle import ref_py
from tests import encoding_cases, toys

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
            "offsets": e.offsets, "word_ids": e.word_ids, "overflowing": [enc_dict(o) for o in e.overflowing]}


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


def _offset_texts():
    """Texts for the offsets walk: the Encoding cases, whitespace runs (words whose byte-level form
    is not in the text: the fallback), accents, CJK, emoji, and seeded random mixes."""
    import random
    out = encoding_cases.texts() + ["hello world\tfoo\nbar  baz", "  leading", "trailing   ", "a\n\n\nb",
                                    "caf\u00e9 na\u00efve", "\u4f60\u597d\u4e16\u754c", "emoji \U0001F600 here",
                                    "x\u00e9y", "\u00e9 x", "'s 're it's", "1,234.56 %"]
    rng = random.Random(5)
    alphabet = ["a", "b", " ", "  ", "\n", "\t", "\u00e9", "\u4e16", "\U0001F600", "1", "!", "'s", "\u20ac", "x y"]
    out += ["".join(rng.choice(alphabet) for _ in range(rng.randrange(1, 12))) for _ in range(300)]
    return out


@pytest.mark.parametrize("variant", ["plain", "prefix_space", "nfc", "invalid_merges"])
def test_offsets_and_word_ids(base, variant):
    """ctok_encode_offsets vs the oracle's encode_single_to_encoding: ids, per-token byte ranges
    and word indices equal, texts whose walk panics in the reference raise PanicException.
    invalid_merges: the rank-shift quirk (src/bpe.rs:60-69) makes some ids' token strings differ
    from their word's bytes, so ids are attributed to words by the device's per-piece counts."""
    obj = json.loads(json.dumps(base))
    if variant == "invalid_merges":
        obj = toys.with_invalid_merges(obj, seed=2, n_bad=30)
    if variant == "prefix_space":
        obj["pre_tokenizer"]["add_prefix_space"] = True
    if variant == "nfc":
        obj["normalizer"] = {"type": "NFC"}
    tok, ref = pair_of(obj)
    ok, bad = [], []
    texts = _offset_texts() + (["e\u0301 x \u00e9\u0301", "A\u030a\u0301b", "n\u0303o"] if variant == "nfc" else [])
    for t in texts:
        try:
            ok.append((t, ref.encode_single_to_encoding(t, 0)))
        except ref_py.PanicException:
            bad.append(t)
    got = tok.encode_offsets([t for t, _ in ok])
    for (t, want), (ids, offs, wids) in zip(ok, got):
        assert ids == want.ids, repr(t)
        assert offs == want.offsets, repr(t)
        assert wids == want.word_ids, repr(t)
    assert len(bad) > 0 or variant != "plain"  # the random mixes reach the reference's panic
    for t in bad[:5]:
        with pytest.raises(PanicException):
            tok.encode_offsets([t])
        with pytest.raises(PanicException):
            tok.encode_to_encoding(t)


def test_offsets_many_tiles_long_pieces(base):
    """the offsets walk over a batch of many pre-tokenizer tiles (~500 KB, 3968-byte
    tiles), with pieces longer than 64 B (the long-piece records) and pieces crossing tile
    boundaries, enough documents that the host walk is split over its threads mid-tile."""
    import random
    tok, ref = pair_of(base)
    rng = random.Random(17)
    words = ["the", "quick", "brown", "fox", "jumps", "over", "lazy", "dog", "caf\u00e9", "na\u00efve", "1234",
             "it's", "we're", "!!", "...", "\u4e16\u754c"]
    texts = []
    for k in range(2500):
        parts = []
        for _ in range(rng.randrange(5, 60)):
            r = rng.random()
            if r < 0.03:
                parts.append("".join(rng.choice("abcdefgh") for _ in range(rng.randrange(65, 400))))
            elif r < 0.05:
                parts.append(" " * rng.randrange(2, 90))
            elif r < 0.06:
                parts.append(str(rng.randrange(10 ** 12)) * rng.randrange(6, 12))
            else:
                parts.append(rng.choice(words))
        texts.append(rng.choice([" ", "\n", "  "]).join(parts))
    ok = []
    for t in texts:
        try:
            ok.append((t, ref.encode_single_to_encoding(t, 0)))
        except ref_py.PanicException:
            pass
    assert len(ok) > 1200 and sum(len(t.encode()) for t, _ in ok) > 400_000
    got = tok.encode_offsets([t for t, _ in ok])
    for (t, want), (ids, offs, wids) in zip(ok, got):
        assert ids == want.ids, repr(t[:80])
        assert offs == want.offsets, repr(t[:80])
        assert wids == want.word_ids, repr(t[:80])


def test_offsets_lookups(base):
    """char / word lookups over the GPU offsets, as the reference computes them."""
    tok, ref = pair_of(encoding_cases.with_post_processor(base, "bert"))
    e = tok.encode_to_encoding("hello world foo")
    w = ref.encode_to_encoding("hello world foo")
    assert e.offsets == w.offsets and e.word_ids == w.word_ids
    assert e.char_to_token(0) == 0 and e.token_to_word(0) == 0
    assert e.word_to_tokens(1) is not None and e.n_words == 3
    p = tok.encode_pair_to_encoding("ab cd", "ef")
    q = ref.encode_to_encoding("ab cd", "ef")
    assert p.offsets == q.offsets and p.word_ids == q.word_ids


def test_encode_padded_concurrent_threads(base):
    """Two threads calling encode_padded on one device (ctypes releases the GIL): each call holds
    the device's lock from staging its inputs to reading back its outputs."""
    import threading
    tok, _ = pair_of(encoding_cases.with_post_processor(base, "bert"))
    a = ["hello world %d" % i for i in range(300)]
    b = ["a much longer text number %d with more words in it" % i for i in range(500)]
    want = {0: tok.encode_padded(a, padding="longest"), 1: tok.encode_padded(b, padding="longest")}
    errs = []

    def work(k, texts):
        try:
            for _ in range(20):
                got = tok.encode_padded(texts, padding="longest")
                for key in want[k]:
                    assert np.array_equal(np.asarray(got[key]), np.asarray(want[k][key])), key
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=work, args=(0, a)), threading.Thread(target=work, args=(1, b))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs[0]


def test_padded_nfc_splice_keeps_no_added_split(base):
    """encode_to_encoding's words skip the added-token split (src/huggingface/mod.rs:395-420); the
    NFC splice re-encodes flagged docs as a sub-batch, which must keep that rule.
    Docs hold an added token's text inside a piece beside a decomposed accent (NFC-flagged), among
    unflagged docs; the padded rows and the plain encode (which does split) against the oracle."""
    obj = encoding_cases.with_post_processor(base, "template")
    nid = max(max(obj["model"]["vocab"].values()), max(a["id"] for a in obj["added_tokens"])) + 1
    for k, content in enumerate(["hello", "ing"]):
        obj["added_tokens"].append({"id": nid + k, "content": content, "single_word": False, "lstrip": False,
                                    "rstrip": False, "normalized": False, "special": False})
    tok, ref = pair_of(obj)
    ts = ["helloé singing", "plain hello text", "xhello café thing", "", "nothing flagged here",
          "abc éabc hellohello"] + ["filler doc %d with words" % i for i in range(50)]
    r = tok.encode_padded(ts, padding="longest")
    want = [ref.encode_to_encoding(t) for t in ts]
    for i, e in enumerate(want):
        n = len(e.ids)  # (the row's content; padding follows)
        assert r["input_ids"][i, :n].tolist() == e.ids, repr(ts[i])
        assert int(r["attention_mask"][i].sum()) == n, repr(ts[i])
    got = tok.encode_batch_to_encoding(ts)
    assert [g.ids for g in got] == [e.ids for e in want]
    assert tok.encode_batch(ts) == [ref.encode(t) for t in ts]
