"""The generated Unicode tables (complexity-tokenizer_amd/csrc/gen/unicode_data.h) against their
sources, over every code point 0 .. 0x10FFFF (CPU only).

The product (k_segment, k_norm, nfc_splice) and the C oracle (oracle/ctok_ref.c) both read these
tables, so a wrong entry would pass every full-config digest test (common mode).  This test reads
the header as data and checks it against independent sources:

* classes of the pre-tokenizer regex (reference src/pretokenizers.rs:11-15): the `regex` module's
  ``\\p{L}``, ``\\p{N}`` and ``\\s`` (its ``\\s`` is exactly Rust's 25 White_Space code points);
* NFC data (reference src/normalizers.rs:45-47, crate unicode-normalization): `unicodedata`'s
  canonical combining class, NFC(c) == c, canonical decompositions (NFD) and primary compositions
  (NFC of the pair), each derived here afresh.

Version boundary: the classes follow the `regex` module's Unicode tables, the NFC data
`unicodedata` (13.0 in this image).  The reference's crates carry their own versions (regex-syntax
and unicode-normalization, semver ranges only: SURVEY.md 8c).  Code points whose class differs
between `regex` and Unicode 13's General Category (assigned or changed after 13.0), and whose
normalisation changed after 13.0, are parity-unpinned; test_version_boundary_recorded counts the
first set so the number in DESIGN.md section 2 stays true.
"""
import os
import re
import unicodedata

import numpy as np
import pytest
import regex

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "complexity-tokenizer_amd", "csrc", "gen", "unicode_data.h")
NCP = 0x110000


def _arrays():
    src = open(HDR).read()
    out = {}
    for m in re.finditer(r"static const (\w+) (\w+)\[(\d+)\] = \{(.*?)\};", src, re.S):
        vals = [int(v.rstrip("ul").rstrip("u"), 0) for v in m.group(4).replace("\n", " ").split(",") if v.strip()]
        assert len(vals) == int(m.group(3)), m.group(2)
        out[m.group(2)] = vals
    for m in re.finditer(r"#define (CT_\w+) (\S+)", src):
        out[m.group(1)] = m.group(2).strip('"')
    return out


@pytest.fixture(scope="module")
def tab():
    return _arrays()


@pytest.fixture(scope="module")
def all_cps():
    return "".join(map(chr, range(NCP)))


def _two_level(s1, s2, per_byte):
    s1 = np.asarray(s1, dtype=np.int64)
    s2 = np.asarray(s2, dtype=np.int64)
    cp = np.arange(NCP, dtype=np.int64)
    blk = s1[cp >> 8]
    if per_byte == 4:  # 2 bits per code point, 4 per byte (kernels.hip cls_of)
        return (s2[blk * 64 + ((cp & 255) >> 2)] >> ((cp & 3) * 2)) & 3
    return s2[blk * 256 + (cp & 255)]


def _matches(pattern, text):
    hit = np.zeros(NCP, dtype=bool)
    hit[[m.start() for m in regex.finditer(pattern, text)]] = True
    return hit


def test_classes_match_regex_for_every_code_point(tab, all_cps):
    cls = _two_level(tab["ct_cls_stage1"], tab["ct_cls_stage2"], 4)
    ws, let, num = _matches(r"\s", all_cps), _matches(r"\p{L}", all_cps), _matches(r"\p{N}", all_cps)
    want = np.where(ws, 0, np.where(let, 1, np.where(num, 2, 3)))
    bad = np.nonzero(cls != want)[0]
    assert bad.size == 0, "class differs from regex at %s" % [hex(c) for c in bad[:20]]
    # Rust's \s (White_Space): exactly these 25 code points
    rust_ws = [0x9, 0xA, 0xB, 0xC, 0xD, 0x20, 0x85, 0xA0, 0x1680] + list(range(0x2000, 0x200B)) + \
              [0x2028, 0x2029, 0x202F, 0x205F, 0x3000]
    assert sorted(np.nonzero(cls == 0)[0].tolist()) == rust_ws


def test_version_boundary_recorded(tab, all_cps):
    """Classes where `regex` (the tables' source) and Unicode 13 (`unicodedata`) disagree: the
    parity-unpinned set of the pre-tokenizer (DESIGN.md section 2 quotes this count)."""
    cls = _two_level(tab["ct_cls_stage1"], tab["ct_cls_stage2"], 4)
    cat = [unicodedata.category(c) for c in all_cps]
    u13 = np.array([0 if i in (0x9, 0xA, 0xB, 0xC, 0xD, 0x20, 0x85, 0xA0, 0x1680, 0x2028, 0x2029, 0x202F, 0x205F, 0x3000)
                    or 0x2000 <= i <= 0x200A else 1 if c[0] == "L" else 2 if c[0] == "N" else 3
                    for i, c in enumerate(cat)])
    diff = np.nonzero(cls != u13)[0]
    # every difference is a code point unassigned in Unicode 13 (new letters / digits since)
    assert all(unicodedata.category(chr(c)) == "Cn" for c in diff)
    assert tab["CT_UNIDATA_VERSION"] == unicodedata.unidata_version == "13.0.0"
    # 14,574 code points unassigned in Unicode 13 that `regex` classes as \p{L} (14,431: CJK
    # extensions G-J, Tangut, Khitan, Kawi, Garay, ...) or \p{N} (143); none is White_Space
    assert diff.size == 14574, diff.size
    assert int((cls[diff] == 1).sum()) == 14431 and int((cls[diff] == 2).sum()) == 143


def test_nfc_ccc_and_quick_check_for_every_code_point(tab):
    v = _two_level(tab["ct_nfc_stage1"], tab["ct_nfc_stage2"], 1)
    ccc, qc = v & 255, v >> 8
    bad_ccc, bad_qc = [], []
    # second elements of primary compositions (NFC_QC = Maybe), derived here from unicodedata
    second = set()
    for cp in range(NCP):
        if 0xD800 <= cp <= 0xDFFF:
            continue
        c = chr(cp)
        if ccc[cp] != unicodedata.combining(c):
            bad_ccc.append(cp)
        d = unicodedata.decomposition(c)
        if d and not d.startswith("<"):
            parts = [int(x, 16) for x in d.split()]
            if len(parts) == 2 and unicodedata.normalize("NFC", c) == c:
                second.add(parts[1])
    second |= set(range(0x1161, 0x1176)) | set(range(0x11A8, 0x11C3))  # Hangul V / T jamo
    for cp in range(NCP):
        if 0xD800 <= cp <= 0xDFFF:
            continue
        c = chr(cp)
        want = 1 if unicodedata.normalize("NFC", c) != c else 2 if cp in second else 0
        if qc[cp] != want:
            bad_qc.append(cp)
    assert not bad_ccc, [hex(c) for c in bad_ccc[:20]]
    assert not bad_qc, [hex(c) for c in bad_qc[:20]]


def test_decompositions_match_nfd_for_every_code_point(tab):
    cps, offs, data = tab["ct_decomp_cp"], tab["ct_decomp_off"], tab["ct_decomp_data"]
    table = {cp: data[offs[i]:offs[i + 1]] for i, cp in enumerate(cps)}
    assert cps == sorted(cps)
    for cp in range(NCP):
        if 0xD800 <= cp <= 0xDFFF or 0xAC00 <= cp <= 0xD7A3:  # Hangul syllables: algorithmic
            continue
        c = chr(cp)
        nfd = unicodedata.normalize("NFD", c)
        if nfd == c:
            assert cp not in table, hex(cp)
            continue
        got = table.get(cp)
        assert got is not None, hex(cp)
        # the table keeps the mapping order; NFD also orders marks canonically: equal after the
        # canonical ordering (stable sort by combining class of the non-starters)
        assert unicodedata.normalize("NFD", "".join(map(chr, got))) == nfd, hex(cp)
        assert sorted(got) == sorted(map(ord, nfd)), hex(cp)


def test_compositions_match_nfc(tab):
    keys, vals = tab["ct_comp_key"], tab["ct_comp_val"]
    comp = {(k >> 21, k & ((1 << 21) - 1)): v for k, v in zip(keys, vals)}
    assert keys == sorted(keys)
    for (a, b), c in comp.items():
        assert unicodedata.normalize("NFC", chr(a) + chr(b)) == chr(c), (hex(a), hex(b))
    # completeness: every primary composite (two-element canonical decomposition, NFC-stable)
    for cp in range(NCP):
        if 0xD800 <= cp <= 0xDFFF or 0xAC00 <= cp <= 0xD7A3:
            continue
        d = unicodedata.decomposition(chr(cp))
        if not d or d.startswith("<"):
            continue
        parts = [int(x, 16) for x in d.split()]
        if len(parts) == 2 and unicodedata.normalize("NFC", chr(cp)) == chr(cp):
            assert comp.get(tuple(parts)) == cp, hex(cp)


def test_bytemap_alnum(tab):
    # the 256 GPT-2 byte-map chars (src/pretokenizers.rs:130-153): Rust char::is_alphanumeric
    bs = list(range(0x21, 0x7F)) + list(range(0xA1, 0xAD)) + list(range(0xAE, 0x100))
    cs, n = list(bs), 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    bmap = dict(zip(bs, cs))
    want = [1 if regex.match(r"[\p{Alphabetic}\p{Nd}\p{Nl}\p{No}]", chr(bmap[b])) else 0 for b in range(256)]
    assert tab["ct_bytemap_alnum"] == want
