"""Parity of the HIP path (libctok.so through the C ABI) with the CPU oracle.

Bit-exact token ids are required (integer work).  Oracle: oracle/ref_py.py (Python
restatement of the reference) for small inputs, oracle/ctok_ref.c (faithful C port, checked
against ref_py in tests/test_oracle.py) for large ones, plus the committed golden vectors.
"""
import json
import os

import numpy as np
import pytest

from complexity_tokenizer import PanicException, Tokenizer
from datagen import corpus
from oracle import ref_c, ref_py
from tests import edge_cases, toys

pytestmark = pytest.mark.gpu


def gpu_tok(obj):
    return Tokenizer.from_str(json.dumps(obj))


def assert_same(gpu_ids, gpu_off, ref_ids, ref_off):
    assert len(gpu_off) == len(ref_off)
    if not (np.array_equal(gpu_off, ref_off) and np.array_equal(gpu_ids, ref_ids)):
        bad = np.flatnonzero(gpu_off != ref_off)
        d = int(bad[0]) - 1 if len(bad) else -1
        if d < 0:
            d = next(i for i in range(len(gpu_off) - 1)
                     if not np.array_equal(gpu_ids[gpu_off[i]:gpu_off[i + 1]], ref_ids[ref_off[i]:ref_off[i + 1]]))
        raise AssertionError("doc %d differs: gpu %s ref %s" % (
            d, gpu_ids[gpu_off[d]:gpu_off[d + 1]].tolist(), ref_ids[ref_off[d]:ref_off[d + 1]].tolist()))


@pytest.fixture(scope="module")
def gpt2(gpt2_path):
    with open(gpt2_path) as f:
        obj = json.load(f)
    return obj, Tokenizer.from_file(gpt2_path), ref_c.RefC(obj)


def test_hello_kat():
    assert gpu_tok(toys.hello_kat()).encode("hello") == [8]


def test_edge_cases_vs_python_oracle(gpt2):
    obj, tok, _ = gpt2
    py = ref_py.RefTokenizer(obj)
    got = tok.encode_batch(edge_cases.EDGE)
    for s, g in zip(edge_cases.EDGE, got):
        assert g == py.encode(s), repr(s)


def test_c1_vs_oracles(gpt2):
    obj, tok, rc = gpt2
    text, off = corpus.corpus_c1()
    ids, toff = tok.encode_packed(text, off)
    rids, rtoff = rc.encode_packed(text, off)
    assert_same(ids, toff, rids, rtoff)
    py = ref_py.RefTokenizer(obj)
    docs = [d.decode() for d in corpus.unpack(text, off)]
    assert [ids[toff[i]:toff[i + 1]].tolist() for i in range(len(docs))] == py.encode_batch(docs)


def test_c2_sample_vs_c_oracle(gpt2):
    _, tok, rc = gpt2
    text, off = corpus.corpus_c2(100_000)
    ids, toff = tok.encode_packed(text, off)
    assert_same(ids, toff, *rc.encode_packed(text, off))


@pytest.mark.parametrize("which", ["c1", "c2"])
def test_stats_pieces(gpt2, which):
    """last_stats["pieces"] (the tile scan's sum of k_segment's per-tile piece counts) equals the
    C oracle's pre-tokenizer piece count; C2's first 200k docs span two scan blocks (> 4096 tiles)."""
    _, tok, rc = gpt2
    text, off = corpus.corpus_c1() if which == "c1" else corpus.corpus_c2(200_000)
    ids, toff = tok.encode_packed(text, off)
    assert_same(ids, toff, *rc.encode_packed(text, off))
    want = sum(len(ref_c.pieces(d)) for d in corpus.unpack(text, off))
    assert tok.last_stats["pieces"] == want


def test_megabyte_documents(gpt2):
    """Documents of 1.3 MB and 2.6 MB (C2 text joined) among small ones: tiles whose context word
    lies more than 64 tiles inside a document get their first document from k_segment's own
    search (k_tilefirst writes 64 tiles per document)."""
    _, tok, rc = gpt2
    text, off = corpus.corpus_c2(30_000)
    small = corpus.unpack(text, off)
    big1 = b" ".join(small[:10_000])
    big2 = b"\n".join(small[10_000:30_000])
    docs = small[:50] + [big1] + small[50:60] + [b"", big2, b""] + small[60:100]
    t2, o2 = corpus.pack(docs)
    ids, toff = tok.encode_packed(t2, o2)
    assert_same(ids, toff, *rc.encode_packed(t2, o2))


def test_long_pieces(gpt2):
    obj, tok, rc = gpt2
    docs = edge_cases.long_docs()
    text, off = corpus.pack([d.encode() for d in docs])
    ids, toff = tok.encode_packed(text, off)
    assert_same(ids, toff, *rc.encode_packed(text, off))
    assert tok.last_stats["long_pieces"] > 0


def test_random_unicode(gpt2):
    obj, tok, rc = gpt2
    docs = edge_cases.random_unicode_docs(20_000, seed=11)
    text, off = corpus.pack([d.encode() for d in docs])
    ids, toff = tok.encode_packed(text, off)
    assert_same(ids, toff, *rc.encode_packed(text, off))
    py = ref_py.RefTokenizer(obj)
    for i in range(0, 2000):
        assert ids[toff[i]:toff[i + 1]].tolist() == py.encode(docs[i]), repr(docs[i])


def test_empty_batch_and_empty_docs(gpt2):
    _, tok, _ = gpt2
    assert tok.encode_batch([]) == []
    assert tok.encode_batch(["", "", ""]) == [[], [], []]
    assert tok.encode("") == []
    r = tok.encode_batch(["", "a b", "", "", "c"])
    assert r[0] == [] and r[2] == [] and r[3] == [] and len(r[1]) > 0 and len(r[4]) > 0


def test_llama3_sample(llama3_path):
    with open(llama3_path) as f:
        obj = json.load(f)
    tok = Tokenizer.from_file(llama3_path)
    rc = ref_c.RefC(obj)
    text, off = corpus.corpus_c3(3000, seed=33)
    ids, toff = tok.encode_packed(text, off)
    assert_same(ids, toff, *rc.encode_packed(text, off))


@pytest.mark.parametrize("fx", ["llama3_path", "llama3_tt_path"])
def test_long_piece_tiers_and_order(request, fx):
    """Long pieces of every tier in one batch: lengths at the tier bounds (<= 256 B dense tier,
    257..1024 and 1025..4096 B segmented tiers, > 4096 B global-memory tier) and random ones, as
    random letters, concatenated words and single-letter repeats.  Exercises k_long_len /
    k_long_order (length buckets, longest-first order) and the per-tier dynamic take
    (kernels.hip), against the C oracle.  llama3_tt_path: the same vocab with the tiktoken-style
    merge list (several merges per token, not rank-monotone): the rounds of eager merges apply
    their sites up to the first cascade (kernels.hip first_cascade)."""
    path = request.getfixturevalue(fx)
    with open(path) as f:
        obj = json.load(f)
    tok = Tokenizer.from_file(path)
    rc = ref_c.RefC(obj)
    rng = np.random.default_rng(77)
    words = [w.encode() for w in "the of and tokenizer merge piece order round wave tier bucket".split()]
    def run(n, kind):
        if kind == 0:
            return bytes(rng.integers(ord("a"), ord("z") + 1, size=n).astype(np.uint8))
        if kind == 1:
            b = b""
            while len(b) < n:
                b += words[int(rng.integers(len(words)))]
            return b[:n]
        return bytes([int(rng.integers(ord("a"), ord("z") + 1))]) * n
    lengths = [63, 64, 65, 255, 256, 257, 1023, 1024, 1025, 2048, 4095, 4096, 4097, 5000]
    lengths += [int(x) for x in rng.integers(65, 1500, size=150)]
    docs = []
    for i, n in enumerate(lengths):
        for kind in range(3):
            docs.append(b"x " + run(n, kind) + b" y")
        docs.append(b"short doc %d" % i)  # ordinary pieces between the long ones
    rng.shuffle(docs)
    text, off = corpus.pack(docs)
    ids, toff = tok.encode_packed(text, off, timing=True)
    assert tok.last_stats["long_pieces"] >= 3 * 150
    assert_same(ids, toff, *rc.encode_packed(text, off))


def test_c3_tiktoken_layout_full_corpus(llama3_tt_path):
    """C3 (100k docs, 76 MB, 1% with 1-4 KiB runs) with the Llama-3-shaped tokenizer whose merge
    list is laid out as the tiktoken conversion of the real Llama-3 file does it: 304k merges,
    several per token (the loader's rank-valued wide table), not rank-monotone (src/bpe.rs:52-79
    keeps every one with its own rank).  The whole corpus against the C oracle's digest
    (tests/golden/digests.json C3TT; it equals C3's: the two merge lists encode the same BPE)."""
    import hashlib
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "digests.json")))["C3TT"]
    tok = Tokenizer.from_file(llama3_tt_path)
    text, off = corpus.corpus_c3()
    assert int(off[-1]) == gold["bytes"]
    ids, toff = tok.encode_packed(text, off, timing=True)
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(toff, dtype="<u8").tobytes())
    h.update(np.ascontiguousarray(ids, dtype="<u4").tobytes())
    assert len(ids) == gold["tokens"]
    assert h.hexdigest() == gold["sha256"]
    assert tok.last_stats["long_pieces"] >= 1000  # (the 1% of docs with a 1-4 KiB run)


@pytest.mark.parametrize("seed", range(6))
def test_window_rounds_random_proper(seed):
    """Window rounds of the segmented tiers (kernels.hip bpe_wave_seg, Tables::window) on random
    rank-monotone tables with tokens up to 8..23 letters (wide windows, model and CPU check in
    tests/test_window_rule.py): pieces of 2-3 letters at every tier's lengths, against the C
    oracle; the same table with an invalid merge in front (window rounds off) too."""
    alpha = b"abc"[: 2 + seed % 2]
    obj = toys.random_proper(seed, alphabet=alpha.decode(), max_len=8 + 3 * seed)
    rng = np.random.default_rng(seed)
    docs = []
    for n in [40, 70, 129, 200, 256, 257, 300, 700, 1024, 1025, 1500, 2500, 4000, 4096, 5000]:
        for _ in range(3):
            docs.append(b"x " + bytes(rng.choice(list(alpha), size=n).astype(np.uint8)) + b" y")
    text, off = corpus.pack(docs)
    tok, rc = gpu_tok(obj), ref_c.RefC(obj)
    ids, toff = tok.encode_packed(text, off)
    assert_same(ids, toff, *rc.encode_packed(text, off))
    assert len(ids) < 0.8 * len(text)  # (the table merges these runs: toys.byte_map, round 4)
    # an invalid merge in front: ranks shift, window rounds off; the last valid merge panics when
    # used, in the reference too (src/bpe.rs:141)
    bad = toys.with_invalid_merge_in_front(obj)
    _parity_or_panic(gpu_tok(bad), ref_c.RefC(bad), text, off)


@pytest.mark.parametrize("alpha", ["日本語", "かなカ", "한국어", "日a本", "\U0001F600\U0001F601", "éßø", "中文字符"])
def test_window_rounds_random_proper_multibyte(alpha):
    """Window rounds on random rank-monotone tables over the UTF-8 bytes of multi-byte chars
    (the C5 path of the dense tier's position windows, kernels.hip bpe_wave_dense): runs of 1..1500
    random chars of the alphabet (3- and 4-byte chars: pieces at every tier, most in the <= 256 B
    dense tier), against the C oracle; the same table with an invalid merge in front (rules off)."""
    seed = sum(map(ord, alpha)) % 1000
    rng = np.random.default_rng(seed)
    chars = list(alpha)
    obj = toys.random_proper_from_text(seed, "".join(rng.choice(chars, size=3000)).encode(), n_merges=150,
                                       max_len=12 + seed % 9)
    docs = []
    for n in [1, 2, 5, 10, 15, 21, 22, 30, 40, 60, 63, 64, 70, 85, 86, 100, 200, 341, 500, 1000, 1400]:
        for _ in range(4):
            docs.append(b"x " + "".join(rng.choice(chars, size=n)).encode() + b" y")
    rng.shuffle(docs)
    text, off = corpus.pack(docs)
    tok, rc = gpu_tok(obj), ref_c.RefC(obj)
    ids, toff = tok.encode_packed(text, off)
    assert_same(ids, toff, *rc.encode_packed(text, off))
    assert len(ids) < 0.7 * len(text)  # (the table really merges these runs)
    bad = toys.with_invalid_merge_in_front(obj)  # (window rounds off; may panic, as the reference)
    _parity_or_panic(gpu_tok(bad), ref_c.RefC(bad), text, off)


@pytest.mark.parametrize("seed", range(8))
def test_window_rounds_non_monotone(seed):
    """Window rounds on tables that are not rank-monotone (round 4: eager candidates checked
    against their neighbours, kernels.hip bpe_wave_seg / bpe_wave_dense): a random proper table's
    merges shuffled, and re-laid out tiktoken-style (tests/test_window_rule.py _non_monotone), with
    runs at every long-piece tier's lengths, against the C oracle."""
    from tests.test_window_rule import _non_monotone
    alpha, rng, objs = _non_monotone(seed)
    chars = list(alpha)
    docs = []
    for n in [5, 20, 40, 63, 64, 65, 86, 100, 200, 256, 257, 400, 700, 1024, 1025, 1400, 3000, 4096, 5000]:
        for _ in range(3):
            docs.append(b"x " + "".join(rng.choice(chars, size=max(1, n // len(chars[0].encode())))).encode() + b" y")
    rng.shuffle(docs)
    text, off = corpus.pack(docs)
    fewer = []
    for o in objs:
        tok, rc = gpu_tok(o), ref_c.RefC(o)
        ids, toff = tok.encode_packed(text, off, timing=True)
        assert_same(ids, toff, *rc.encode_packed(text, off))
        # the window rounds ran: fewer rounds than with them switched off at load
        rounds = tok.last_stats["long_rounds"]
        os.environ["CTOK_NO_WINDOW"] = "1"
        try:
            plain = gpu_tok(o)
        finally:
            del os.environ["CTOK_NO_WINDOW"]
        ids2, toff2 = plain.encode_packed(text, off, timing=True)
        assert_same(ids2, toff2, ids, toff)
        assert 0 < rounds <= plain.last_stats["long_rounds"], (rounds, plain.last_stats["long_rounds"])
        fewer.append(rounds < plain.last_stats["long_rounds"])
    assert any(fewer), "window rounds never fired"


def test_c3_full_corpus(llama3_path):
    """C3 (100k docs, 76 MB, 1% with 1-4 KiB runs of letters, digits, words or one repeated
    letter) with the rank-monotone Llama-3-shaped fixture, whose long pieces take the window
    rounds, against the C oracle's digest (tests/golden/digests.json C3)."""
    import hashlib
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "digests.json")))["C3"]
    tok = Tokenizer.from_file(llama3_path)
    text, off = corpus.corpus_c3()
    assert int(off[-1]) == gold["bytes"]
    ids, toff = tok.encode_packed(text, off, timing=True)
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(toff, dtype="<u8").tobytes())
    h.update(np.ascontiguousarray(ids, dtype="<u4").tobytes())
    assert len(ids) == gold["tokens"]
    assert h.hexdigest() == gold["sha256"]


def test_eager_cascade_rounds():
    """toys.eager_cascade: after an "a b" merges, ("ab", "a") ranks below ("a", "b"), so a round
    of that merge must stop at its first site whose new pairs rank lower (kernels.hip
    first_cascade) -- in pieces of every long-piece tier (dense <= 256 B, segmented 257..4096 B,
    global-memory > 4096 B) and in the register passes, against the C oracle."""
    obj = toys.eager_cascade()
    tok, rc = gpu_tok(obj), ref_c.RefC(obj)
    rng = np.random.default_rng(5)
    docs = []
    for n in [2, 3, 4, 7, 20, 40, 63, 64, 65, 127, 200, 255, 256, 257, 600, 1024, 1500, 2047, 2048, 2049, 4100, 6000]:
        docs += [b"ab" * n, b"x " + b"ab" * n + b"c" * (n % 13) + b"ab" * 3, b"ba" + b"ab" * n,
                 bytes(rng.choice(list(b"abc"), size=2 * n).astype(np.uint8))]
    text, off = corpus.pack(docs)
    ids, toff = tok.encode_packed(text, off)
    assert_same(ids, toff, *rc.encode_packed(text, off))
    assert tok.encode("abab") == [obj["model"]["vocab"]["aba"], obj["model"]["vocab"]["b"]]


def _consonant_pair_docs(n, seed=8):
    """Docs of " qx" pieces (two consonants: ~94% are not single tokens of the gpt2 fixture), about
    1250 class-0 pieces per 3968-byte tile."""
    rng = np.random.default_rng(seed)
    cons = np.frombuffer(b"bcdfghjklmnpqrstvwxz", dtype=np.uint8)
    return [b" " + b" ".join(bytes(x) for x in rng.choice(cons, size=(1500, 2))) for _ in range(n)]


def test_class0_list_spill_to_long_list(gpt2):
    """Tiles with more than kCap0Lean (1040) pieces of <= 8 B that are not single tokens: the
    class-0 list keeps 1040 of a tile's pieces, the rest go to the long list and its dense wave
    tier (ctok_internal.h kCap0Lean); against the C oracle.  40 such docs among 2.5 MB of C2 text
    spill ~10k pieces, within the lean long list (B/32 entries)."""
    _, tok, rc = gpt2
    text, off = corpus.corpus_c2(20_000, seed=12)
    docs = [bytes(text[off[i]:off[i + 1]]) for i in range(len(off) - 1)]
    tok.encode_packed(text, off, timing=True)
    base = tok.last_stats["long_pieces"]  # the corpus's own long pieces
    adv = _consonant_pair_docs(40)
    docs = docs[:5000] + adv[:20] + docs[5000:] + adv[20:]
    text, off = corpus.pack(docs)
    ids, toff = tok.encode_packed(text, off, timing=True)
    assert tok.last_stats["long_pieces"] > base + 5000  # the spilled pieces (3 bytes each)
    assert_same(ids, toff, *rc.encode_packed(text, off))


def test_class0_spill_overflow_reruns_safe(gpt2):
    """Only such docs: the spilled pieces outgrow the lean long list, the call runs again with the
    safe capacities (every class-0 piece listed; no spill, so no long pieces)."""
    _, tok, rc = gpt2
    text, off = corpus.pack(_consonant_pair_docs(300))
    ids, toff = tok.encode_packed(text, off, timing=True)
    assert tok.last_stats["long_pieces"] == 0
    assert_same(ids, toff, *rc.encode_packed(text, off))


@pytest.mark.parametrize("n_docs", [20_000, 200_000])
def test_dropped_byte_chars(gpt2, n_docs):
    """A vocab without the byte chars of 'q', 'x', 'z': the reference drops those chars
    (src/bpe.rs:94-97), so pieces holding them take the dropped-byte pass (k_bpe_generic MID: ids
    in the tile's class region after the merge passes' ids).  200k docs overflow the lean
    dropped-byte list (65536 entries): the call runs again with the safe capacities."""
    obj, _, _ = gpt2
    obj = json.loads(json.dumps(obj))
    for c in "qxz":
        del obj["model"]["vocab"][c]
    tok, rc = gpu_tok(obj), ref_c.RefC(obj)
    text, off = corpus.corpus_c2(n_docs, seed=41)
    ids, toff = tok.encode_packed(text, off)
    assert_same(ids, toff, *rc.encode_packed(text, off))


def test_multi_sample(multi_path):
    with open(multi_path) as f:
        obj = json.load(f)
    tok = Tokenizer.from_file(multi_path)
    rc = ref_c.RefC(obj)
    text, off = corpus.corpus_c5(20_000, seed=55)
    ids, toff = tok.encode_packed(text, off, timing=True)
    assert_same(ids, toff, *rc.encode_packed(text, off))
    # C5 holds no code point NFC changes: the speculation flags no document (k_segment decodes each
    # code point from LDS, including one that starts at the end of the look-ahead word)
    assert tok.last_stats["nfc_docs"] == 0


def test_multi_nfc_sample(multi_path):
    """C5-NFC: 5% of 20k multilingual docs carry NFC-active text (decomposed Latin, conjoining
    jamo, Devanagari / Arabic / Hebrew / Thai marks): the k_segment speculation flags them, and
    the flagged docs are normalised (k_nfc_check -> k_norm) and encoded again as a sub-batch
    whose ids are spliced into the speculative pass's output."""
    with open(multi_path) as f:
        obj = json.load(f)
    tok = Tokenizer.from_file(multi_path)
    rc = ref_c.RefC(obj)
    text, off = corpus.corpus_c5nfc(20_000, seed=56, frac=0.05)
    ids, toff = tok.encode_packed(text, off, timing=True)
    assert tok.last_stats["nfc_docs"] > 0
    assert_same(ids, toff, *rc.encode_packed(text, off))


def test_improper_table(gpt2):
    obj, _, _ = gpt2
    sh = toys.shuffled_merges(obj, seed=3)
    tok, rc = gpu_tok(sh), ref_c.RefC(sh)
    docs = edge_cases.long_docs() + edge_cases.EDGE
    text, off = corpus.pack([d.encode() for d in docs])
    ids, toff = tok.encode_packed(text, off)
    assert_same(ids, toff, *rc.encode_packed(text, off))
    text, off = corpus.corpus_c2(20_000, seed=9)
    ids, toff = tok.encode_packed(text, off)
    assert_same(ids, toff, *rc.encode_packed(text, off))


def _parity_or_panic(tok, rc, text, off):
    try:
        want = rc.encode_packed(text, off)
    except ref_py.PanicException:
        with pytest.raises(PanicException):
            tok.encode_packed(text, off)
        return "panic"
    assert_same(*tok.encode_packed(text, off), *want)
    return "ok"


def test_invalid_merges_shift_and_panic(gpt2):
    obj, _, _ = gpt2
    text, off = corpus.corpus_c2(20_000, seed=12)
    seen = set()
    for seed in range(3):
        bad = toys.with_invalid_merges(obj, seed=seed, n_bad=30)
        seen.add(_parity_or_panic(gpu_tok(bad), ref_c.RefC(bad), text, off))
    # invalid merges only at the tail: indices of valid merges unchanged, never a panic
    tail = toys.with_invalid_merges(obj, seed=4, n_bad=30, tail_only=True)
    assert _parity_or_panic(gpu_tok(tail), ref_c.RefC(tail), text, off) == "ok"


def test_panic_toy():
    # rank of (a, b) is 1 but only one merge is valid: BpeTokenizer.merges[1] is out of range
    bc = toys.byte_chars()
    vocab = {c: i for i, c in enumerate(bc)}
    vocab["ab"] = 256
    obj = toys.tok_json(vocab, [("x", "yy"), ("a", "b")])
    tok = gpu_tok(obj)
    assert tok.encode("ba") == ref_py.RefTokenizer(obj).encode("ba")
    with pytest.raises(PanicException):
        tok.encode("ab")
    with pytest.raises(ref_py.PanicException):
        ref_py.RefTokenizer(obj).encode("ab")


def test_nfd_only_panic_pair_does_not_panic(gpt2):
    """A merge ranked past the valid merges (src/bpe.rs:60-69, :141 panics on it) whose pair exists
    only in decomposed text: the reference normalises first (NFC, src/normalizers.rs:45-47) and
    never sees it.  The speculative pass over the raw bytes does; its panic flag must not survive
    into the result."""
    obj, _, _ = gpt2
    pair = (toys.byte_char(0xCC), toys.byte_char(0x81))  # the bytes of U+0301, byte-mapped: one piece of their own
    obj = json.loads(json.dumps(obj))
    assert "%s %s" % pair not in obj["model"]["merges"]
    obj["model"]["vocab"][pair[0] + pair[1]] = max(obj["model"]["vocab"].values()) + 1
    ms = list(obj["model"]["merges"]) + ["zzq%d qqz%d" % (k, k) for k in range(3)] + ["%s %s" % pair]
    obj["model"]["merges"] = ms
    tok, rc = gpu_tok(obj), ref_c.RefC(obj)
    text, off = corpus.corpus_c2(2_000, seed=79)
    docs = [d.decode() for d in corpus.unpack(text, off)]
    docs[5] = "cafe\u0301 and re\u0301sume\u0301"
    docs[1500] = "e\u0301" * 30
    want = rc.encode_batch(docs)
    assert tok.encode_batch(docs) == want
    ids, toff = tok.encode_packed(*corpus.pack([d.encode() for d in docs]))
    assert_same(ids, toff, *rc.encode_packed(*corpus.pack([d.encode() for d in docs])))
    # U+0301 after a char it does not compose with survives NFC: both panic
    for d in (docs[:10] + ["q\u0301"], ["x q\u0301 y"]):
        with pytest.raises(ref_py.PanicException):
            rc.encode_batch(d)
        with pytest.raises(PanicException):
            tok.encode_batch(d)


def test_wide_table_mode(gpt2, monkeypatch):
    """The rank-valued (wide) merge table must give the same ids as the compact one."""
    obj, _, rc = gpt2
    monkeypatch.setenv("CTOK_FORCE_WIDE", "1")
    tok = gpu_tok(obj)
    monkeypatch.delenv("CTOK_FORCE_WIDE")
    text, off = corpus.corpus_c2(30_000, seed=21)
    assert_same(*tok.encode_packed(text, off), *rc.encode_packed(text, off))
    docs = edge_cases.long_docs() + edge_cases.EDGE
    text, off = corpus.pack([d.encode() for d in docs])
    assert_same(*tok.encode_packed(text, off), *rc.encode_packed(text, off))


def test_without_piece_table(gpt2, monkeypatch):
    """Disabling the whole-piece table (every piece through the merge loop) gives the same ids."""
    obj, _, rc = gpt2
    monkeypatch.setenv("CTOK_NO_PIECE_TABLE", "1")
    tok = gpu_tok(obj)
    monkeypatch.delenv("CTOK_NO_PIECE_TABLE")
    text, off = corpus.corpus_c2(30_000, seed=22)
    assert_same(*tok.encode_packed(text, off), *rc.encode_packed(text, off))


def test_nfc_speculation_redo(gpt2):
    """NFC is speculated away for text without NFC-unstable code points; one such code point
    anywhere in the batch (here: only in the last doc, far from the first tile) makes the
    library check, normalise and run again.  Both batches must match the oracle exactly."""
    obj, tok, rc = gpt2
    text, off = corpus.corpus_c2(20_000, seed=77)
    ascii_docs = [d.decode() for d in corpus.unpack(text, off)]
    for tail in ("", "café Å"):
        docs = ascii_docs + ([tail] if tail else [])
        got = tok.encode_batch(docs)
        want = rc.encode_batch(docs)
        assert got == want, "batch with tail %r differs" % tail
        # (nfc_docs: the docs normalised again; flags are per 64-byte word, so the doc sharing the
        # tail's first word is re-encoded too -- a superset, with the same ids)
        n = 0 if tok.last_stats is None else tok.last_stats.get("nfc_docs", 0)
        assert (1 <= n <= 2) if tail else n == 0


@pytest.mark.parametrize("mode", ["splice", "rerun"])
def test_nfc_splice_positions(gpt2, monkeypatch, mode):
    """NFC-active docs (decomposed accents that NFC composes: fewer bytes, other tokens; marks
    that stay) at the first, last and middle positions, in runs, beside empty docs, among ASCII
    docs: the speculative pass finishes and only the flagged docs are encoded again, normalised,
    and spliced in (ctok_host.cpp nfc_splice); "rerun" is the whole-batch path it replaces.
    Both against the C oracle."""
    obj, tok, rc = gpt2
    if mode == "rerun":
        monkeypatch.setenv("CTOK_NFC_RERUN", "1")
    text, off = corpus.corpus_c2(5_000, seed=78)
    base = [d.decode() for d in corpus.unpack(text, off)]
    act = ["cafe\u0301 A\u030a", "n\u0303o e\u0301e\u0301 \u1100\u1161\u11a8", "\u0915\u093c x",
           "\u00e9\u0301", "plain e\u0301" * 40]
    docs = [act[0]] + base[:100] + [act[1], act[2]] + base[100:2000] + ["", act[3], ""] + base[2000:] + [act[4]]
    got = tok.encode_batch(docs)
    assert got == rc.encode_batch(docs)
    assert tok.last_stats is None or tok.last_stats.get("nfc_docs", 0) >= 5
    ids, toff = tok.encode_packed(*corpus.pack([d.encode() for d in docs]), timing=True)
    assert tok.last_stats["nfc_docs"] >= 5
    assert_same(ids, toff, *rc.encode_packed(*corpus.pack([d.encode() for d in docs])))
    only = [act[1], act[4], act[0]]  # every doc flagged
    assert tok.encode_batch(only) == rc.encode_batch(only)


def test_from_tables_encodes_like_from_file(gpt2_path):
    """ctok_create_from_tables on the fixture's tables (normalizer null = NFC, parsing.rs:89)."""
    from tests.test_native_cpu import _tables_of
    with open(gpt2_path) as f:
        obj = json.load(f)
    a = Tokenizer.from_file(gpt2_path)
    b = Tokenizer.from_tables(*_tables_of(obj), nfc=True)
    text, off = corpus.corpus_c1()
    docs = [d.decode() for d in corpus.unpack(text, off)] + edge_cases.EDGE
    assert a.encode_batch(docs) == b.encode_batch(docs)
