"""CPU tests of the oracle (oracle/ref_py.py, oracle/ctok_ref.c): pinned against the reference's
own known-answer tests, the committed golden vectors, the `regex` module, and HF `tokenizers` on
the input domain where the two provably agree.  Also pins, on the CPU, the
piece-start rules the HIP pre-tokenizer kernel evaluates, per code point and in the
bit-parallel form of kernels.hip k_segment."""
import hashlib
import json
import os
import random
import unicodedata

import numpy as np
import pytest

from datagen import corpus
from oracle import ref_c, ref_py
from tests import edge_cases, toys

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def gpt2_obj(gpt2_path):
    with open(gpt2_path) as f:
        return json.load(f)


# ----------------------------------------------------------------- reference known-answer tests

def test_kat_bpe_hello():
    """src/bpe.rs:219-250: lowest rank first, encode("hello") == [8]."""
    obj = toys.hello_kat()
    assert ref_py.RefTokenizer(obj).encode("hello") == [8]
    assert ref_c.RefC(obj).encode_batch(["hello"]) == [[8]]


def test_kat_bytes_to_unicode():
    """src/models.rs:955-969 and src/trainer.rs:659-667."""
    enc = ref_py.bytes_to_unicode()
    assert len(enc) == 256
    assert enc[ord(" ")] == "Ġ"
    assert enc[ord("a")] == "a" and enc[ord("Z")] == "Z"
    dec = {v: k for k, v in enc.items()}
    assert all(dec[enc[b]] == b for b in range(256))


def test_kat_nfc():
    """src/normalizers.rs:223-230."""
    assert unicodedata.normalize("NFC", "é") == "é"
    assert ref_c.nfc_bytes("é".encode()) == "é".encode()


def test_kat_loader_vocab_size():
    """src/huggingface/mod.rs:1566-1592."""
    assert ref_py.RefTokenizer(toys.loader_kat()).vocab_size == 8


def test_kat_gpt2_split():
    """src/pretokenizers.rs:625-630 (the reference only asserts > 1 piece); exact pieces here."""
    pcs = [m.group(0) for m in ref_py.GPT2_PATTERN.finditer("Hello, world!")]
    assert pcs == ["Hello", ",", " world", "!"]


# ----------------------------------------------------------------- golden vectors

def test_golden_c1(gpt2_obj):
    g = np.load(os.path.join(GOLDEN, "c1_gpt2_50k.npz"))
    text, off = corpus.corpus_c1()
    assert np.array_equal(text, g["text"]) and np.array_equal(off, g["off"]), "C1 generator drifted"
    py = ref_py.RefTokenizer(gpt2_obj)
    docs = [d.decode() for d in corpus.unpack(text, off)]
    got = py.encode_batch(docs)
    ids, toff = g["ids"], g["tok_off"]
    assert got == [ids[toff[i]:toff[i + 1]].tolist() for i in range(len(docs))]
    cids, coff = ref_c.RefC(gpt2_obj).encode_packed(text, off)
    assert np.array_equal(cids, ids) and np.array_equal(coff, toff)


def test_golden_edge(gpt2_obj):
    with open(os.path.join(GOLDEN, "edge_gpt2_50k.json")) as f:
        cases = json.load(f)
    py = ref_py.RefTokenizer(gpt2_obj)
    rc = ref_c.RefC(gpt2_obj)
    docs = [c[0] for c in cases]
    assert py.encode_batch(docs) == [c[1] for c in cases]
    assert rc.encode_batch(docs) == [c[1] for c in cases]


def _digest(ids, tok_off):
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(tok_off, dtype="<u8").tobytes())
    h.update(np.ascontiguousarray(ids, dtype="<u4").tobytes())
    return h.hexdigest()


def test_golden_c2_first_100k_c_oracle(gpt2_obj):
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        gold = json.load(f)["C2"]
    text, off = corpus.corpus_c2()
    n = gold["first_docs"]
    ids, toff = ref_c.RefC(gpt2_obj).encode_packed(text[: int(off[n])], off[: n + 1])
    assert len(ids) == gold["first_tokens"] and _digest(ids, toff) == gold["first_sha256"]


@pytest.mark.parametrize("cfg", ["C2", "C5", "C5NFC"])
def test_golden_digests_pinned_to_ref_py(cfg):
    """The C oracle writes every full-config digest; tests/golden/make_golden.py first runs the
    Python restatement (`regex` + `unicodedata`, no generated table) on the config's first 100k
    documents and stores its digest (pin_ref_py), which must equal the C oracle's digest of the
    same documents (first_sha256, recomputed for C2 by test_golden_c2_first_100k_c_oracle; the GPU
    full-config tests compare the product's first 100k documents with it too)."""
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        gold = json.load(f)[cfg]
    pin = gold["pin_ref_py"]
    assert pin["docs"] >= 100_000 and pin["docs"] == gold["first_docs"]
    assert pin["sha256"] == gold["first_sha256"] and pin["tokens"] == gold["first_tokens"]


# ----------------------------------------------------------------- the two oracles agree

def test_c_oracle_matches_python_oracle(gpt2_obj):
    docs = edge_cases.EDGE + edge_cases.long_docs() + edge_cases.random_unicode_docs(4000, seed=5)
    assert ref_c.RefC(gpt2_obj).encode_batch(docs) == ref_py.RefTokenizer(gpt2_obj).encode_batch(docs)


@pytest.mark.parametrize("variant", ["shuffled", "invalid_tail", "invalid_mixed"])
def test_oracles_agree_on_quirky_tables(gpt2_obj, variant):
    if variant == "shuffled":
        obj = toys.shuffled_merges(gpt2_obj, seed=1)
    elif variant == "invalid_tail":
        obj = toys.with_invalid_merges(gpt2_obj, seed=2, n_bad=40, tail_only=True)
    else:
        obj = toys.with_invalid_merges(gpt2_obj, seed=3, n_bad=40)
    docs = edge_cases.EDGE + edge_cases.random_unicode_docs(1500, seed=6)
    py, rc = ref_py.RefTokenizer(obj), ref_c.RefC(obj)
    try:
        want = py.encode_batch(docs)
    except ref_py.PanicException:
        with pytest.raises(ref_py.PanicException):
            rc.encode_batch(docs)
        return
    assert rc.encode_batch(docs) == want


def test_nfc_matches_unicodedata():
    rng = random.Random(9)
    pool = [chr(c) for c in list(range(0x20, 0x250)) + list(range(0x300, 0x370)) + list(range(0x1100, 0x1176))
            + list(range(0x11A8, 0x11C3)) + list(range(0xAC00, 0xAC40)) + list(range(0x1E00, 0x1F00))
            + [0xF900, 0xFA10, 0x212B, 0x2126, 0x0F73, 0x0F75, 0x1D160, 0x0344, 0x0958, 0x09DC]]
    for _ in range(3000):
        s = "".join(rng.choice(pool) for _ in range(rng.randint(0, 12)))
        assert ref_c.nfc_bytes(s.encode()) == unicodedata.normalize("NFC", s).encode(), repr(s)


def test_piece_boundaries_match_regex():
    for s in edge_cases.EDGE + edge_cases.random_unicode_docs(3000, seed=8):
        assert [p.decode() for p in ref_c.pieces(s.encode())] == [m.group(0) for m in ref_py.GPT2_PATTERN.finditer(s)]


# ----------------------------------------------------------------- the GPU segmentation rules

def _cls(c):
    if ref_py._rust_ws(c):
        return 0
    import regex
    if regex.match(r"\p{L}", c):
        return 1
    if regex.match(r"\p{N}", c):
        return 2
    return 3


def gpu_rule_pieces(s):
    """Per-code-point form of the run-class segmentation rules that k_segment
    evaluates bit-parallel (bitparallel_starts below)."""
    u = list(s)
    c = [_cls(x) for x in u]
    n = len(u)

    def prev(i):
        return i - 1 if i > 0 else -1

    def nxt(i):
        return i + 1 if i + 1 < n else -1

    def attached(i):
        if u[i] != " ":
            return False
        j = nxt(i)
        if j < 0 or c[j] == 0:
            return False
        p = prev(i)
        return p < 0 or c[p] != 0

    def con_len(i):
        if u[i] != "'":
            return 0
        n1 = nxt(i)
        if n1 < 0 or c[n1] != 1:
            return 0
        p = prev(i)
        if p >= 0 and (c[p] == 3 or attached(p)):
            return 0
        a = u[n1]
        if a in "stmd":
            return 1
        n2 = nxt(n1)
        if n2 < 0:
            return 0
        return 2 if a + u[n2] in ("re", "ve", "ll") else 0

    def start(i):
        if i == 0:
            return True
        p = prev(i)
        if c[i] != c[p]:
            return not (attached(p) or con_len(p) > 0)
        if c[i] == 1:
            pp = prev(p)
            if pp >= 0:
                if con_len(pp) == 1:
                    return True
                ppp = prev(pp)
                if ppp >= 0 and con_len(ppp) == 2:
                    return True
        return False

    cuts = [i for i in range(n) if start(i)] + [n]
    return ["".join(u[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]


def test_gpu_segmentation_rules_equal_regex():
    docs = edge_cases.EDGE + edge_cases.random_unicode_docs(20000, seed=10, max_len=24)
    for s in docs:
        assert gpu_rule_pieces(s) == [m.group(0) for m in ref_py.GPT2_PATTERN.finditer(s)], repr(s)


def bitparallel_starts(text, docstart):
    """Python transcription of kernels.hip k_segment: the piece-start predicate evaluated on
    64-bit masks of 64-byte words (SegMasks / seg_derive), word neighbours carried across edges."""
    M = (1 << 64) - 1
    B = len(text)

    def masks(g):
        m = dict.fromkeys(("W", "L", "N", "S", "Q", "T1", "R", "Le", "V", "LL", "D"), 0)
        if g < 0:
            return m
        for k in range(64):
            x = g * 64 + k
            if x >= B:
                m["D"] |= 1 << k
                continue
            b = text[x]
            j = x
            while (text[j] & 0xC0) == 0x80:
                j -= 1
            c = _cls(text[j:j + 4].decode("utf-8", errors="ignore")[:1])
            for key, hit in (("W", c == 0), ("L", c == 1), ("N", c == 2), ("S", b == 32), ("Q", b == 39),
                             ("T1", b in b"stmd"), ("R", b == 114), ("Le", b == 101), ("V", b == 118),
                             ("LL", b == 108), ("D", docstart[x])):
                if hit:
                    m[key] |= 1 << k
        return m

    def p(c, q, k):
        return ((c << k) | (q >> (64 - k))) & M

    def n(c, q, k):
        return ((c >> k) | (q << (64 - k))) & M

    def derive(rp, rc, rn, a_prev):
        P = ~(rc["W"] | rc["L"] | rc["N"]) & M
        Pp = ~(rp["W"] | rp["L"] | rp["N"]) & M
        E = n(rc["D"], rn["D"], 1)
        A = rc["S"] & ~E & ~n(rc["W"], rn["W"], 1) & (rc["D"] | ~p(rc["W"], rp["W"], 1)) & M
        Cb = rc["Q"] & ~E & n(rc["L"], rn["L"], 1) & (rc["D"] | (~p(P, Pp, 1) & ~p(A, a_prev, 1))) & M
        t1 = n(rc["T1"], rn["T1"], 1)
        C2 = Cb & ~t1 & ~n(rc["D"], rn["D"], 2) & (
            ((n(rc["R"], rn["R"], 1) | n(rc["V"], rn["V"], 1)) & n(rc["Le"], rn["Le"], 2))
            | (n(rc["LL"], rn["LL"], 1) & n(rc["LL"], rn["LL"], 2))) & M
        return A, Cb & t1, C2

    out = []
    rp, rc, rn = masks(-2), masks(-1), masks(0)
    a_p, c1_p, c2_p = derive(rp, rc, rn, 0)
    rp, rc = rc, rn
    for g in range((B + 63) // 64):
        rn = masks(g + 1)
        A, C1, C2 = derive(rp, rc, rn, a_p)
        chg = 0
        for key in ("W", "L", "N"):
            chg |= rc[key] ^ p(rc[key], rp[key], 1)
        st = rc["D"] | (chg & ~p(A, a_p, 1) & ~p(C1 | C2, c1_p | c2_p, 1) & M) | (
            ~chg & rc["L"] & (p(C1, c1_p, 2) | p(C2, c2_p, 3)) & M)
        out += [g * 64 + k for k in range(64) if (st >> k) & 1 and g * 64 + k < B]
        rp, rc = rc, rn
        a_p, c1_p, c2_p = A, C1, C2
    return out


def test_gpu_bitparallel_segmentation_equals_regex():
    rng = random.Random(11)
    for trial in range(150):
        docs = edge_cases.EDGE if trial == 0 else edge_cases.random_unicode_docs(
            rng.randint(1, 40), seed=rng.randint(0, 10 ** 9), max_len=40)
        text = b"".join(d.encode() for d in docs)
        ds = [0] * len(text)
        want, o = [], 0
        for d in docs:
            e = d.encode()
            if e:
                ds[o] = 1
            want += [o + len(d[:m.start()].encode()) for m in ref_py.GPT2_PATTERN.finditer(d)]
            o += len(e)
        assert bitparallel_starts(text, ds) == want, docs


@pytest.fixture(scope="module")
def seg_lane_lib(tmp_path_factory):
    """tools/seg_lane_check.cpp (the kernel's per-lane SWAR logic, csrc/seg_lane.h) built with g++."""
    import ctypes
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = os.path.join(root, "complexity-tokenizer_amd", "tools", "seg_lane_check.cpp")
    so = str(tmp_path_factory.mktemp("seg") / "libseglane.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", src, "-o", so], check=True)
    lib = ctypes.CDLL(so)
    lib.seg_lane_starts.restype = ctypes.c_int
    lib.seg_lane_starts.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_void_p]
    return lib


def _lane_starts(lib, docs):
    text = b"".join(d.encode() for d in docs)
    ds = bytearray(len(text) + 1)
    want, o = [], 0
    for d in docs:
        e = d.encode()
        if e:
            ds[o] = 1
        want += [o + len(d[:m.start()].encode()) for m in ref_py.GPT2_PATTERN.finditer(d)]
        o += len(e)
    words = np.zeros((len(text) + 63) // 64 + 1, dtype=np.uint64)
    assert lib.seg_lane_starts(text, len(text), bytes(ds), words.ctypes.data) == 0, "look-ahead word disagrees"
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[: len(text)]
    return np.nonzero(bits)[0].tolist(), want


def test_gpu_swar_lane_segmentation_equals_regex(seg_lane_lib):
    rng = random.Random(13)
    for trial in range(400):
        if trial == 0:
            docs = edge_cases.EDGE
        elif trial % 5 == 0:  # several tiles of short docs
            docs = edge_cases.random_unicode_docs(rng.randint(50, 400), seed=rng.randint(0, 10 ** 9), max_len=60)
        else:
            docs = edge_cases.random_unicode_docs(rng.randint(1, 40), seed=rng.randint(0, 10 ** 9), max_len=40)
        got, want = _lane_starts(seg_lane_lib, docs)
        assert got == want, docs
    text, off = corpus.corpus_c1()
    docs = [d.decode() for d in corpus.unpack(text, off)]
    got, want = _lane_starts(seg_lane_lib, docs)
    assert got == want


# ----------------------------------------------------------------- independent BPE cross-check

def test_hf_tokenizers_agree_on_shared_domain(gpt2_path, gpt2_obj):
    """HF `tokenizers` (Rust) BPE equals the oracle where both apply the same split: single spaces
    between words, no other whitespace, NFC-stable text, no added-token strings."""
    tokenizers = pytest.importorskip("tokenizers")
    hf = tokenizers.Tokenizer.from_file(gpt2_path)
    py = ref_py.RefTokenizer(gpt2_obj)
    rng = random.Random(12)
    words = ["the", "and", "of", "don't", "it's", "12", "3456", "hello", "world", "!", "?!", ".", "café",
             "naïve", "x1", "a", "I", "we'll", "(", ")", "世界", "\U0001f600"]
    text, off = corpus.corpus_c1()
    lex = [w for d in corpus.unpack(text, off) for w in d.decode().split() if w.isascii()][:3000]
    for _ in range(1500):
        k = rng.randint(1, 12)
        s = " ".join(rng.choice(words + lex) for _ in range(k))
        if rng.random() < 0.5:
            s = " " + s
        assert hf.encode(s, add_special_tokens=False).ids == py.encode(s), repr(s)


# ----------------------------------------------------------------------------- decode oracles


def test_decode_kat_byte_level():
    """reference src/decoders.rs:275-281."""
    out = ref_py.byte_level_decode(["\u0120Hello", "\u0120world"])
    assert "Hello" in out and out == " Hello world"


def test_from_utf8_lossy_matches_python_codec():
    """Rust from_utf8_lossy and CPython's 'replace' error handler both substitute one U+FFFD per
    maximal subpart (Unicode 'best practice'); checked on random and adversarial byte strings."""
    import random
    rng = random.Random(3)
    special = [0x80, 0xBF, 0xC0, 0xC1, 0xC2, 0xDF, 0xE0, 0xED, 0xEF, 0xF0, 0xF4, 0xF5, 0xFF, 0x9F, 0xA0, 0x90, 0x8F]
    for _ in range(100000):
        b = bytes(rng.choice(special) if rng.random() < 0.6 else rng.randrange(256) for _ in range(rng.randint(0, 9)))
        assert ref_py.from_utf8_lossy(b) == b.decode("utf-8", "replace"), b


def test_cleanup_rules():
    f = ref_py.clean_up_tokenization_spaces_
    assert f("a , b . c") == "a, b. c"
    assert f(" - - ") == "--"
    assert f('say " hi " now') == 'say"hi"now'
    assert f("x\u001cy z") == "x\u001cy z"  # U+001C is not White_Space (Python's split would split)
    assert f("\u3000x\u00a0\u0085y ") == "x y"


def test_parse_decoder_variants():
    pd = ref_py.parse_decoder
    assert pd(None) == ("ByteLevel",) and pd("x") == ("ByteLevel",) and pd({}) == ("ByteLevel",)
    assert pd({"type": "ByteLevel"}) == ("ByteLevel",)
    assert pd({"type": "Unknown"}) == ("Raw",) and pd({"type": 3}) == ("Raw",)
    assert pd({"type": "Fuse"}) == ("Raw",)
    assert pd({"type": "Metaspace"})[0] == "unsupported"
    assert pd({"type": "Sequence", "decoders": [{"type": "ByteLevel"}, {"type": "Fuse"}]}) == ("ByteLevel",)
    assert pd({"type": "Sequence", "decoders": [{"type": "Nope"}]}) == ("Raw",)
    assert pd({"type": "Sequence", "decoders": ["x"]}) == ("ByteLevel",)
    assert pd({"type": "Sequence", "decoders": [{"type": "ByteLevel"}, {}]})[0] == "unsupported"
    assert pd({"type": "Sequence", "decoders": [{"type": "WordPiece"}]})[0] == "unsupported"


@pytest.mark.parametrize("name", ["gpt2_50k", "multi_32k", "llama3_128k"])
def test_decode_oracles_agree(name, fixture_dir):
    from datagen.build_tokenizers import fixture_path
    from tests import decode_cases
    with open(fixture_path(name, fixture_dir)) as f:
        obj = json.load(f)
    py = ref_py.RefTokenizer(obj)
    rc = ref_c.RefC(obj)
    special = list(py.special_tokens.values())
    batch = decode_cases.random_batches(len(py.id_to_token_map), 400, 5, special_ids=special)
    batch += decode_cases.split_docs(batch[:100], 6)
    batch += [py.encode(t) for t in decode_cases.CLEANUP_TEXTS]
    for skip in (False, True):
        for clean in (False, True):
            assert rc.decode_batch(batch, skip, clean, threads=4) == py.decode_batch(batch, skip, clean)


def _eager_values(rt):
    """Tables::eager on the oracle's tables: rank r is eager when a merge consuming its token ranks
    before r (ctok_host.cpp's eager_bits for a rank-valued table)."""
    mincons = {}
    for (a, b), r in rt.merge_ranks.items():
        if r < len(rt.merge_new_ids):
            for c in (a, b):
                mincons[c] = min(mincons.get(c, r), r)
    return {r for r in set(rt.merge_ranks.values()) if r < len(rt.merge_new_ids)
            and mincons.get(rt.merge_new_ids[r], 1 << 60) < r}


def _rounds_bpe(rt, eager, text):
    """The long-piece kernels' round structure in Python (kernels.hip first_cascade): per round
    the minimum rank r and its sites; a non-eager r merges every site at once ((x, x) runs: the
    1st, 3rd, ...); an eager r merges the sites left to right up to and including the first whose
    sequential new pairs -- (left neighbour, or nid after a merged site two tokens before; nid)
    and (nid, the next token as it is) -- include a rank below r; an eager (x, x) run merges its
    leftmost site only."""
    toks = [rt.vocab[c] for c in text if c in rt.vocab]
    while True:
        rk = [rt.merge_ranks.get((toks[i], toks[i + 1])) for i in range(len(toks) - 1)]
        live = [r for r in rk if r is not None]
        if not live:
            return toks
        r = min(live)
        nid = rt.merge_new_ids[r]
        first = rk.index(r)
        chain = toks[first] == toks[first + 1]
        sites, i = [], 0
        while i < len(rk):
            if rk[i] == r:
                sites.append(i)
                i += 2
            else:
                i += 1
        if r in eager and chain:
            sites = sites[:1]
        elif r in eager:
            for k, p in enumerate(sites):
                left = nid if (k and sites[k - 1] == p - 2) else (toks[p - 1] if p else None)
                rl = rt.merge_ranks.get((left, nid)) if left is not None else None
                rr = rt.merge_ranks.get((nid, toks[p + 2])) if p + 2 < len(toks) else None
                if (rl is not None and rl < r) or (rr is not None and rr < r):
                    sites = sites[:k + 1]
                    break
        S = set(sites)
        out, i = [], 0
        while i < len(toks):
            if i in S:
                out.append(nid)
                i += 2
            else:
                out.append(toks[i])
                i += 1
        toks = out


def test_parallel_rounds_with_eager_rule_equal_sequential_bpe(tmp_path):
    """The tiktoken-style Llama-3 table (several merges per token, not rank-monotone): rounds that
    apply every site of a non-eager merge at once give the reference's sequential ids
    (src/bpe.rs:88-153) on long letter / digit / word runs; with every merge treated as non-eager
    (the old global rule) some pieces differ, so the eager bits are what keeps them exact."""
    from datagen.build_tokenizers import fixture_path
    with open(fixture_path("llama3_tt_128k", str(tmp_path))) as f:
        rt = ref_py.RefTokenizer(json.load(f))
    eager = _eager_values(rt)
    assert eager, "the tiktoken-style table should have eager merges"
    rng = random.Random(9)
    bm = ref_py.bytes_to_unicode()
    words = ["the", "quick", "brown", "information", "tion", "ing", "abc", "aaaa", "1234567"]
    wrong_without = 0
    for k in range(400):
        kind = k % 4
        n = rng.randrange(20, 300)
        if kind == 0:
            s = "".join(rng.choice("abcdefghij") for _ in range(n))
        elif kind == 1:
            s = "".join(rng.choice("0123456789") for _ in range(n))
        elif kind == 2:
            s = "".join(rng.choice(words) for _ in range(n // 5))
        else:
            s = rng.choice("ab") * n + "".join(rng.choice("ab") for _ in range(n))
        text = "".join(bm[b] for b in s.encode())
        want = rt.bpe(text)
        assert _rounds_bpe(rt, eager, text) == want, s[:60]
        wrong_without += _rounds_bpe(rt, set(), text) != want
    # (on this BPE-trained vocab the all-at-once rule happens to agree too; the toy table of
    # toys.eager_cascade is one where it does not)
    rt = ref_py.RefTokenizer(toys.eager_cascade())
    eager = _eager_values(rt)
    ab = rt.merge_ranks[(rt.vocab["a"], rt.vocab["b"])]
    assert ab in eager
    for s in ("abab", "ababab", "xabababab", "abcabab", "ab" * 40 + "c" * 9 + "ba" * 7):
        want = rt.bpe(s)
        assert _rounds_bpe(rt, eager, s) == want, s
    assert _rounds_bpe(rt, set(), "abab") != rt.bpe("abab")
