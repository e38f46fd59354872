"""CPU tests of the product's host side: the C-ABI library loads and exports every entry point
declared in include/ctok.h, the tokenizer.json loader reproduces the reference's accept/reject
decisions and getters, and encode fails loudly (no CPU fallback) when no GPU is visible."""
import ctypes
import json
import os
import re

import numpy as np
import pytest

import complexity_tokenizer as ct
from complexity_tokenizer import Tokenizer, UnsupportedConfigError
from complexity_tokenizer import _native
from oracle import ref_py
from tests import toys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_exports_every_declared_symbol():
    hdr = ""
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if h.endswith(".h"):
            with open(os.path.join(ROOT, "include", h)) as f:
                hdr += f.read()
    names = sorted(set(re.findall(r"\b(ctok_[a-z_0-9]+)\s*\(", hdr)))
    assert len(names) >= 25 and "ctok_trainer_train" in names
    lib = ctypes.CDLL(_native.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) <= set(_native.SIGS), set(names) - set(_native.SIGS)


def test_version():
    assert ct.__version__ == "0.3.3"
    assert _native.lib.ctok_version().startswith(b"0.3.3")


@pytest.mark.parametrize("fixture", ["gpt2_path", "llama3_path", "multi_path"])
def test_loader_getters_match_oracle(fixture, request):
    path = request.getfixturevalue(fixture)
    with open(path) as f:
        obj = json.load(f)
    tok = Tokenizer.from_file(path)
    py = ref_py.RefTokenizer(obj)
    assert tok.vocab_size == py.vocab_size
    assert tok.special_tokens == py.special_tokens
    for s in list(obj["model"]["vocab"])[:2000:7] + ["Ġthe", "nonexistent-token", ""]:
        assert tok.token_to_id(s) == py.token_to_id(s), s
    for i in list(range(0, 300)) + [len(obj["model"]["vocab"]) - 1, 10 ** 7]:
        assert tok.id_to_token(i) == py.id_to_token(i), i


def test_loader_kat_and_from_str():
    assert Tokenizer.from_str(json.dumps(toys.loader_kat())).vocab_size == 8


def test_load_errors(tmp_path):
    with pytest.raises(IOError):
        Tokenizer.from_file(str(tmp_path / "missing.json"))
    bad = tmp_path / "bad.json"
    bad.write_text("{not json")
    with pytest.raises(IOError):
        Tokenizer.from_file(str(bad))
    for broken in ({}, {"model": {}}, {"model": {"vocab": {"a": -1}}}, {"model": {"vocab": {"a": 1.5}}},
                   {"model": {"vocab": {"a": 0}, "merges": 3}},
                   {"model": {"vocab": {"a": 0}}, "added_tokens": [{"id": 1, "content": "x"}]}):
        with pytest.raises(IOError):
            Tokenizer.from_str(json.dumps(broken))


@pytest.mark.parametrize("pre,norm", [
    ({"type": "Metaspace"}, None),
    ({"type": "Whitespace"}, None),
    ({"type": "Split", "pattern": {"Regex": "\\s+"}, "behavior": "Isolated"}, None),
    (None, {"type": "Lowercase"}),
    (None, {"type": "NFKC"}),
])
def test_unsupported_components_fail_loudly(pre, norm):
    obj = toys.tok_json({"a": 0}, [], normalizer=norm, pre_tokenizer=pre)
    with pytest.raises(UnsupportedConfigError):
        Tokenizer.from_str(json.dumps(obj))
    with pytest.raises(ref_py.UnsupportedConfig):
        ref_py.RefTokenizer(obj)


def test_supported_shapes_load():
    vocab = {c: i for i, c in enumerate(toys.byte_chars())}
    llama_split = {"type": "Split", "pattern": {"Regex": "\\s+(?!\\S)|\\s+"}, "behavior": "Isolated"}
    for pre in (None, {"type": "ByteLevel", "add_prefix_space": True},
                {"type": "Sequence", "pretokenizers": [llama_split, {"type": "ByteLevel", "use_regex": False}]}):
        for norm in (None, {"type": "NFC"}, {"type": "Sequence", "normalizers": [{"type": "NFC"}]}, {"type": "Foo"}):
            Tokenizer.from_str(json.dumps(toys.tok_json(vocab, [], normalizer=norm, pre_tokenizer=pre)))


def test_empty_added_token_rejected():
    obj = toys.tok_json({"a": 0}, [], added=[{"id": 1, "content": "", "special": True}])
    with pytest.raises(UnsupportedConfigError):
        Tokenizer.from_str(json.dumps(obj))


def test_from_pretrained_local_cache(tmp_path, monkeypatch, gpt2_path):
    monkeypatch.setenv("XDG_CACHE_HOME", str(tmp_path))
    d = tmp_path / "huggingface" / "hub" / "org--name"
    d.mkdir(parents=True)
    with open(gpt2_path, "rb") as f:
        (d / "tokenizer.json").write_bytes(f.read())
    assert Tokenizer.from_pretrained("org/name", local_files_only=True).vocab_size == 50257
    with pytest.raises(IOError):
        Tokenizer.from_pretrained("org/other", local_files_only=True)
    with pytest.raises(IOError):
        Tokenizer.from_pretrained("org/name")  # network fetch: unavailable


def test_pack_texts_type_errors():
    with pytest.raises(TypeError):
        ct.pack_texts("not a list")
    with pytest.raises(TypeError):
        ct.pack_texts(["ok", 3])
    text, off = ct.pack_texts(["ab", "", "é"])
    assert off.tolist() == [0, 2, 2, 4] and text[:4].tobytes() == "abé".encode()


@pytest.mark.skipif(ct.device_count() > 0, reason="a HIP device is present")
def test_encode_without_gpu_fails_loudly(gpt2_path):
    tok = Tokenizer.from_file(gpt2_path)
    with pytest.raises(ct.DeviceError):
        tok.encode("hello world")


@pytest.mark.skipif(ct.device_count() > 0, reason="a HIP device is present")
def test_decode_without_gpu_fails_loudly(gpt2_path):
    tok = Tokenizer.from_file(gpt2_path)
    with pytest.raises(ct.DeviceError):
        tok.decode([1, 2, 3])
    with pytest.raises(ct.DeviceError):
        tok.decode_batch([[1], []])


def test_pack_ids_type_errors():
    ids, off = ct.pack_ids([[1, 2], [], [3]])
    assert ids.tolist() == [1, 2, 3] and off.tolist() == [0, 2, 2, 3]
    with pytest.raises(TypeError):
        ct.pack_ids("abc")
    with pytest.raises(TypeError):
        ct.pack_ids([[1, "x"]])
    with pytest.raises(OverflowError):
        ct.pack_ids([[-1]])
    with pytest.raises(OverflowError):
        ct.pack_ids([[2 ** 32]])


def test_shard_bounds_cover_and_balance():
    from complexity_tokenizer.parallel import concat_results, shard_bounds
    rng = np.random.default_rng(0)
    lens = rng.integers(0, 300, size=1001)
    lens[::17] = 0
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    for world in (1, 2, 3, 8):
        ranges = [shard_bounds(off, world, r) for r in range(world)]
        assert ranges[0][0] == 0 and ranges[-1][1] == len(lens)
        assert all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
        sizes = [int(off[b] - off[a]) for a, b in ranges]
        assert max(sizes) - min(sizes) <= 2 * 300 + int(off[-1]) // world // 10 + 1
    parts = [(np.array([1, 2], np.uint32), np.array([0, 2], np.uint64)),
             (np.array([3], np.uint32), np.array([0, 0, 1], np.uint64))]
    ids, toff = concat_results(parts)
    assert ids.tolist() == [1, 2, 3] and toff.tolist() == [0, 2, 2, 3]


# Split patterns and whether Rust's regex crate compiles them (regex-syntax grammar; the reference
# drops a Split it cannot compile, src/pretokenizers.rs:298-302).  A compiling one is refused here.
SPLIT_PATTERNS = [
    ("\\s+(?!\\S)|\\s+", False),             # look-ahead: the Llama-3 / GPT-4 style patterns
    ("(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\\r\\n\\p{L}\\p{N}]?\\p{L}+|\\p{N}{1,3}| ?[^\\s\\p{L}\\p{N}]+[\\r\\n]*|\\s*[\\r\\n]+|\\s+(?!\\S)|\\s+",
     False),
    ("(?<=a)b", False), ("(?<!a)b", False), ("a(?=b)", False),  # look-behind / look-ahead
    ("(?>ab)", False),                       # atomic group
    ("(\\w)\\1", False), ("(?P<x>a)(?P=x)", False), ("(?<x>a)\\k<x>", False),  # backreferences
    ("(?|a|b)", False), ("(?#note)a", False), ("(?(1)a|b)", False),  # branch reset, comment, conditional
    ("\\p{Foo}+", False), ("\\p{sc=Nope}", False), ("\\p{InBasicLatin}", False),  # unknown \p names
    ("a\\Z", False), ("\\Ga", False),          # escapes the crate does not have
    ("*a", False), ("a|+b", False), ("(?:*)", False), ("a{3,2}", False),  # nothing to repeat, bad range
    ("[[:foo:]]", True),                     # unknown [:name:]: a nested class of ':', 'f', 'o' (regex-syntax backtracks)
    ("[[:^bar:]x]", True),
    ("(?R)a", True), ("(?Rm:a)b", True),      # R: the CRLF-mode flag (regex >= 1.8)
    ("a{99999999999999999999}", False),      # a count past u32: invalid decimal
    ("a{2,4294967296}", False),
    ("(ab", False), ("ab)", False), ("[ab", False),  # unbalanced
    ("[(?=]x", True),                        # '(?=' inside a character class is literal
    ("\\(?=x", True),                        # escaped '(' : a literal paren, then an optional '='
    ("[^]](?=x)", False), ("(?<name>a)b", True), ("(?P<n>a)", True), ("\\s+", True),
    ("(a[)]b)", True), ("\\p{L}+|\\p{N}+", True), ("\\p{Greek}\\p{IsLatin}\\pL", True),
    ("\\p{Script=Han}|\\p{gc=Lu}|\\p{scx:Kana}", True), ("[\\p{L}&&\\p{Greek}]", True),
    ("a++b*+", True),                        # possessive: a repetition of a repetition to regex-syntax
    ("(?i)abc(?-i:d)", True), ("x{2,}y{,}z{3}", True), ("[[:alpha:][:digit:]]", True),
    ("(?x) a # (?= comment", True),          # verbose mode: not walked, taken as compiling
]


@pytest.mark.parametrize("pattern,compiles", SPLIT_PATTERNS)
def test_split_pattern_compilability(pattern, compiles):
    """A Split whose pattern Rust's regex compiles would split (unsupported here: loud error); one it
    cannot compile is skipped by the reference (src/pretokenizers.rs:298-330): the tokenizer loads.
    The product and the oracle agree with each other on which is which."""
    vocab = {c: i for i, c in enumerate(toys.byte_chars())}
    split = {"type": "Split", "pattern": {"Regex": pattern}, "behavior": "Isolated"}
    obj = toys.tok_json(vocab, [], pre_tokenizer={"type": "Sequence", "pretokenizers": [
        split, {"type": "ByteLevel", "use_regex": False}]})
    assert ref_py.rust_regex_compiles(pattern) == compiles
    if compiles:
        with pytest.raises(UnsupportedConfigError, match="taken as compiling.*pattern: "):  # (names the pattern)
            Tokenizer.from_str(json.dumps(obj))
    else:
        Tokenizer.from_str(json.dumps(obj))


def _tables_of(obj):
    vocab = obj["model"]["vocab"]
    merges = []
    for m in obj["model"]["merges"]:
        a, b = m.split(" ") if isinstance(m, str) else m
        merges.append((vocab[a], vocab[b]))
    return vocab, merges, obj.get("added_tokens", [])


def test_create_from_tables_matches_json(gpt2_path):
    """ctok_create_from_tables: the same loader on tables instead of JSON text."""
    with open(gpt2_path) as f:
        obj = json.load(f)
    vocab, merges, added = _tables_of(obj)
    a = Tokenizer.from_file(gpt2_path)
    b = Tokenizer.from_tables(vocab, merges, added, nfc=True)
    assert a.vocab_size == b.vocab_size and a.special_tokens == b.special_tokens
    for tok in list(vocab)[:: max(1, len(vocab) // 500)]:
        assert a.token_to_id(tok) == b.token_to_id(tok)
    for i in range(0, a.vocab_size, 97):
        assert a.id_to_token(i) == b.id_to_token(i)
    with pytest.raises(ValueError):
        Tokenizer.from_tables(vocab, [(0, 10 ** 9)])


def test_create_from_tables_rejects_tokens_with_spaces():
    """A merge of a token whose string contains ' ' cannot be written as the reference's "a b"
    merge string: the reference would drop it and shift every later rank
    (src/huggingface/mod.rs:252-264), so ctok_create_from_tables refuses the table (CTOK_E_ARG)."""
    vocab = {c: i for i, c in enumerate(toys.byte_chars())}
    n = len(vocab)
    vocab.update({"a b": n, "a bc": n + 1, "ab": n + 2})
    with pytest.raises(ValueError, match="contains ' '"):
        Tokenizer.from_tables(vocab, [(vocab["a b"], vocab["c"])])
    # tokens without spaces still load, and a vocab entry with a space that no merge joins is fine
    t = Tokenizer.from_tables(vocab, [(vocab["a"], vocab["b"])])
    assert t.token_to_id("a b") == n


def _c_array(src, name):
    import re
    m = re.search(r"%s\[\d+\] = \{(.*?)\};" % name, src, re.S)
    return [int(x, 0) for x in m.group(1).replace("\n", " ").split(",") if x.strip()]


def test_cp_range_classes_match_tables():
    """k_segment classifies CJK / Hangul / kana / emoji code points by range tests (ctok_internal.h
    cp_range_class, round 4) instead of the two-level tables: every code point of those ranges must
    have that class and no NFC flag in gen/unicode_data.h (the host re-checks this at upload,
    cp_fast_ok), and the classes must be the regex module's (\\p{L} / other)."""
    import regex
    src = open(os.path.join(ROOT, "complexity-tokenizer_amd", "csrc", "gen", "unicode_data.h")).read()
    c1, c2 = _c_array(src, "ct_cls_stage1"), _c_array(src, "ct_cls_stage2")
    n1, n2 = _c_array(src, "ct_nfc_stage1"), _c_array(src, "ct_nfc_stage2")
    ranges = [(0x4E00, 0x9FFF, 1), (0xAC00, 0xD7A3, 1), (0x3041, 0x3096, 1), (0x30A1, 0x30FA, 1),
              (0x1F300, 0x1F64F, 3)]
    rl, rn, rs = regex.compile(r"\p{L}"), regex.compile(r"\p{N}"), regex.compile(r"\s")
    for lo, hi, want in ranges:
        for cp in range(lo, hi + 1):
            cl = (c2[c1[cp >> 8] * 64 + ((cp & 255) >> 2)] >> ((cp & 3) * 2)) & 3
            assert cl == want, hex(cp)
            assert n2[n1[cp >> 8] * 256 + (cp & 255)] == 0, hex(cp)
            ch = chr(cp)
            assert (1 if rl.match(ch) else 0 if rs.match(ch) else 2 if rn.match(ch) else 3) == want, hex(cp)
