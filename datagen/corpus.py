"""Seeded, deterministic synthetic corpora for the benchmark configs.

Everything is vectorised numpy so the 1M-document configs build in seconds on the GPU box.
A corpus is returned packed the way the C ABI consumes it: ``(text: np.uint8[B], off: np.uint64[D+1])``.

Configs:
  C1  1,000 docs, uniform 1-64 B, ASCII English-like                         seed 1
  C2  1,000,000 docs, uniform 96-160 B (mean 128), ASCII English-like          seed 2
  C3  100,000 docs, log-uniform 16 B-4 KiB, ASCII + Latin-1; 1% carry >=1 KiB letter/digit runs  seed 3
  C4  10,000,000 docs as C2, in independent 1M-doc blocks (sharded over GPUs)  seed 4
  C5  1,000,000 docs, uniform 64-512 B: 40% CJK/kana/Hangul, 20% emoji, 40% ASCII   seed 5
"""
from __future__ import annotations

import numpy as np

# ----------------------------------------------------------------------------- surface table


class Surface:
    """A table of byte strings addressed by id, flattened for vectorised gathers."""

    def __init__(self):
        self.items: list[bytes] = []

    def add(self, b: bytes) -> int:
        self.items.append(b)
        return len(self.items) - 1

    def add_many(self, bs) -> np.ndarray:
        i0 = len(self.items)
        self.items.extend(bs)
        return np.arange(i0, len(self.items), dtype=np.int64)

    def freeze(self):
        lens = np.array([len(b) for b in self.items], dtype=np.int64)
        self.lens = lens
        self.starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        self.flat = np.frombuffer(b"".join(self.items), dtype=np.uint8)
        return self

    def assemble(self, ids: np.ndarray) -> np.ndarray:
        """Concatenate the surfaces `ids` (int64 array) into one uint8 stream."""
        lens = self.lens[ids]
        total = int(lens.sum())
        out_off = np.cumsum(lens) - lens
        src = np.repeat(self.starts[ids] - out_off, lens) + np.arange(total, dtype=np.int64)
        return self.flat[src]


_ONSETS = ["", "b", "c", "d", "f", "g", "h", "j", "k", "l", "m", "n", "p", "r", "s", "t", "v", "w", "y", "z",
           "br", "ch", "cl", "cr", "dr", "fl", "fr", "gl", "gr", "pl", "pr", "sc", "sh", "sl", "sm", "sn", "sp",
           "st", "str", "th", "tr", "wh", "wr"]
_VOWELS = ["a", "e", "i", "o", "u", "ai", "ea", "ee", "ie", "oo", "ou", "y", "io", "ue"]
_CODAS = ["", "", "", "n", "r", "s", "t", "l", "m", "d", "ng", "st", "nt", "ck", "ll", "ss", "rd", "th", "ld"]


def lexicon(n_words: int, seed: int) -> list[str]:
    rng = np.random.default_rng(seed)
    words, seen = [], set()
    nsyl_p = np.array([0.30, 0.42, 0.20, 0.08])
    while len(words) < n_words:
        k = n_words - len(words)
        nsyl = rng.choice(4, size=k, p=nsyl_p) + 1
        on = rng.integers(0, len(_ONSETS), size=(k, 4))
        vo = rng.integers(0, len(_VOWELS), size=(k, 4))
        co = rng.integers(0, len(_CODAS), size=(k, 4))
        for i in range(k):
            w = "".join(_ONSETS[on[i, s]] + _VOWELS[vo[i, s]] + _CODAS[co[i, s]] for s in range(nsyl[i]))
            if w not in seen:
                seen.add(w)
                words.append(w)
    # Zipf rank follows length, so the most frequent words are the short ones (as in English)
    words.sort(key=len)
    return words


def _zipf_ids(rng, n, k, s=1.1):
    """n draws from Zipf(s) over ranks [0, k)."""
    w = 1.0 / np.power(np.arange(1, k + 1, dtype=np.float64), s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    return np.minimum(np.searchsorted(cdf, rng.random(n)), k - 1)


def _cut_docs(stream: np.ndarray, lengths: np.ndarray, utf8: bool) -> tuple[np.ndarray, np.ndarray]:
    """Cut `stream` into docs of the given byte lengths (moved forward to char boundaries)."""
    off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    assert off[-1] <= len(stream), (off[-1], len(stream))
    if utf8:
        lead = np.flatnonzero((stream & 0xC0) != 0x80)
        lead = np.concatenate([lead, [len(stream)]])
        off = lead[np.searchsorted(lead, off)]
        off = np.maximum.accumulate(off)
    text = stream[: off[-1]].copy()
    return text, off.astype(np.uint64)


# ----------------------------------------------------------------------------- English-like ASCII

_PUNCT = [b",", b".", b"!", b"?", b";", b":", b"-", b"...", b"\"", b")", b"(", b"'", b"--", b"/", b"%"]
_CONTR = [b"'s", b"'t", b"'re", b"'ve", b"'m", b"'ll", b"'d"]
_SEPS = [(b" ", 0.88), (b"  ", 0.02), (b"\n", 0.03), (b"\n\n", 0.01), (b" \n", 0.01), (b"\t", 0.005),
         (b"   ", 0.005), (b"", 0.04)]


class EnglishGen:
    def __init__(self, seed: int, n_words: int = 200_000, latin1: bool = False):
        self.rng = np.random.default_rng(seed)
        words = lexicon(n_words, seed + 1000)
        sf = Surface()
        self.w_lower = sf.add_many(w.encode() for w in words)
        self.w_cap = sf.add_many((w[:1].upper() + w[1:]).encode() for w in words)
        nums = [str(x).encode() for x in self.rng.integers(0, 10 ** self.rng.integers(1, 7, size=20000))]
        self.nums = sf.add_many(nums)
        self.punct = sf.add_many(_PUNCT)
        self.contr = sf.add_many(_CONTR)
        self.seps = sf.add_many(s for s, _ in _SEPS)
        self.sep_p = np.array([p for _, p in _SEPS])
        self.sep_p /= self.sep_p.sum()
        self.empty = sf.add(b"")
        self.latin1 = latin1
        if latin1:
            acc = "éèêëáàâäíìîïóòôöúùûüçñÉÈÀÇÑßøåæ"
            lw = []
            for w in words[:50000]:
                pos = len(w) // 2
                lw.append((w[:pos] + acc[sum(map(ord, w)) % len(acc)] + w[pos:]).encode())
            self.w_lat = sf.add_many(lw)
        self.sf = sf.freeze()
        self.n_words = n_words

    def stream(self, n_bytes: int) -> np.ndarray:
        rng = self.rng
        k = int(n_bytes / 5.0) + 1024
        out = []
        total = 0
        while total < n_bytes:
            wid = _zipf_ids(rng, k, self.n_words)
            word = np.where(rng.random(k) < 0.10, self.w_cap[wid], self.w_lower[wid])
            if self.latin1:
                lat = rng.random(k) < 0.15
                word = np.where(lat, self.w_lat[wid % len(self.w_lat)], word)
            isnum = rng.random(k) < 0.05
            word = np.where(isnum, self.nums[rng.integers(0, len(self.nums), k)], word)
            contr = np.where((rng.random(k) < 0.02) & ~isnum, self.contr[rng.integers(0, len(self.contr), k)], self.empty)
            punct = np.where(rng.random(k) < 0.10, self.punct[rng.integers(0, len(self.punct), k)], self.empty)
            sep = self.seps[rng.choice(len(self.seps), size=k, p=self.sep_p)]
            ids = np.stack([word, contr, punct, sep], axis=1).reshape(-1)
            s = self.sf.assemble(ids)
            out.append(s)
            total += len(s)
        return np.concatenate(out)[:n_bytes]


def _docs_from_lengths(gen_stream, lengths, utf8):
    need = int(lengths.sum()) + 64 * 1024
    stream = gen_stream(need)
    return _cut_docs(stream, lengths, utf8)


def corpus_c1(n_docs: int = 1000, seed: int = 1):
    g = EnglishGen(seed)
    lengths = g.rng.integers(1, 65, size=n_docs)
    return _docs_from_lengths(g.stream, lengths, False)


def corpus_c2(n_docs: int = 1_000_000, seed: int = 2):
    g = EnglishGen(seed)
    lengths = g.rng.integers(96, 161, size=n_docs)
    return _docs_from_lengths(g.stream, lengths, False)


# C4: 10M C2-style docs, built in blocks of C4_BLOCK docs so that any doc range (a rank's shard)
# is generated without the rest: the doc lengths of the whole corpus come from one cheap RNG
# stream (seed), block b's text from the C2 generator re-seeded with (seed, b).  Blocks are
# independent, so they are built by a process pool.
C4_DOCS = 10_000_000
C4_BLOCK = 1_000_000


def c4_lengths(n_docs: int = C4_DOCS, seed: int = 4) -> np.ndarray:
    return np.random.default_rng([seed, 0x4C454E]).integers(96, 161, size=n_docs)


def c4_offsets(n_docs: int = C4_DOCS, seed: int = 4) -> np.ndarray:
    """Byte offsets[D+1] of the whole C4 corpus (what parallel.shard_bounds cuts)."""
    return np.concatenate([[0], np.cumsum(c4_lengths(n_docs, seed))]).astype(np.uint64)


_C4_GEN = {}


def _c4_block(args):
    seed, b, lengths = args
    g = _C4_GEN.get(seed)
    if g is None:
        g = _C4_GEN[seed] = EnglishGen(seed)  # lexicon and surfaces shared by every block
    g.rng = np.random.default_rng([seed, b])
    return _docs_from_lengths(g.stream, lengths, False)[0]


def corpus_c4_range(d0: int, d1: int, n_docs: int = C4_DOCS, seed: int = 4, workers: int = 1):
    """Docs [d0, d1) of C4 as (text, offsets rebased to 0)."""
    lengths = c4_lengths(n_docs, seed)
    off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    b0, b1 = d0 // C4_BLOCK, (max(d1, d0 + 1) - 1) // C4_BLOCK + 1
    jobs = [(seed, b, lengths[b * C4_BLOCK: min((b + 1) * C4_BLOCK, n_docs)]) for b in range(b0, b1) if d1 > d0]
    if workers > 1 and len(jobs) > 1:
        import multiprocessing as mp
        with mp.get_context("fork").Pool(min(workers, len(jobs))) as pool:
            parts = pool.map(_c4_block, jobs)
    else:
        parts = [_c4_block(j) for j in jobs]
    text = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    base = int(off[b0 * C4_BLOCK]) if jobs else 0
    a, z = int(off[d0]) - base, int(off[d1]) - base
    return text[a:z].copy(), (off[d0:d1 + 1] - off[d0]).astype(np.uint64)


def corpus_c4(n_docs: int = C4_DOCS, seed: int = 4, workers: int = 1):
    return corpus_c4_range(0, n_docs, n_docs, seed, workers)


def corpus_c3(n_docs: int = 100_000, seed: int = 3):
    g = EnglishGen(seed, latin1=True)
    rng = g.rng
    lengths = np.exp(rng.uniform(np.log(16), np.log(4096), size=n_docs)).astype(np.int64)
    text, off = _docs_from_lengths(g.stream, lengths, True)
    # 1% of docs get a >= 1 KiB letter or digit run spliced in
    docs = [text[off[i]:off[i + 1]].tobytes() for i in range(n_docs)]
    pick = rng.choice(n_docs, size=max(1, n_docs // 100), replace=False)
    for j, d in enumerate(pick):
        n = int(rng.integers(1024, 4097))
        kind = j % 4
        if kind == 0:
            run = bytes(rng.integers(ord("a"), ord("z") + 1, size=n).astype(np.uint8))
        elif kind == 1:
            run = bytes(rng.integers(ord("0"), ord("9") + 1, size=n).astype(np.uint8))
        elif kind == 2:
            ws = g.sf.assemble(g.w_lower[_zipf_ids(rng, n // 3, g.n_words)])
            run = ws.tobytes()[:n]
        else:
            ch = bytes([int(rng.integers(ord("a"), ord("z") + 1))])
            run = ch * n
        cut = len(docs[d]) // 2
        while cut > 0 and (docs[d][cut] & 0xC0) == 0x80:  # split at a character boundary
            cut -= 1
        docs[d] = docs[d][:cut] + b" " + run + b" " + docs[d][cut:]
    return pack(docs)


# ----------------------------------------------------------------------------- multilingual

def _cps_to_utf8_table(cps):
    return [chr(c).encode("utf-8") for c in cps]


class MultiGen:
    def __init__(self, seed: int):
        self.rng = np.random.default_rng(seed)
        self.eng = EnglishGen(seed + 77, n_words=50_000)
        sf = Surface()
        cjk = list(range(0x4E00, 0x9FA6))
        kana = list(range(0x3041, 0x3097)) + list(range(0x30A1, 0x30FB))
        hangul = list(range(0xAC00, 0xD7A4))
        self.cjk = sf.add_many(_cps_to_utf8_table(cjk))
        self.kana = sf.add_many(_cps_to_utf8_table(kana))
        self.hangul = sf.add_many(_cps_to_utf8_table(hangul))
        self.cjk_p = sf.add_many(_cps_to_utf8_table([0x3001, 0x3002, 0xFF01, 0xFF1F, 0x300C, 0x300D]))
        emo = list(range(0x1F300, 0x1F650))
        self.emoji = sf.add_many(_cps_to_utf8_table(emo))
        self.skin = sf.add_many(_cps_to_utf8_table(range(0x1F3FB, 0x1F400)))
        self.zwj = sf.add("\u200d".encode())
        self.vs16 = sf.add("\ufe0f".encode())
        self.space = sf.add(b" ")
        self.empty = sf.add(b"")
        self.sf = sf.freeze()

    def cjk_stream(self, n_bytes):
        rng = self.rng
        k = n_bytes // 3 + 256
        script = rng.random(k)
        cid = np.where(script < 0.6, self.cjk[_zipf_ids(rng, k, len(self.cjk), 1.05)],
                       np.where(script < 0.8, self.kana[_zipf_ids(rng, k, len(self.kana), 1.0)],
                                self.hangul[_zipf_ids(rng, k, len(self.hangul), 1.05)]))
        tail = np.where(rng.random(k) < 0.08, self.cjk_p[rng.integers(0, len(self.cjk_p), k)],
                        np.where(rng.random(k) < 0.05, self.space, self.empty))
        return self.sf.assemble(np.stack([cid, tail], 1).reshape(-1))

    def emoji_stream(self, n_bytes):
        rng = self.rng
        k = n_bytes // 4 + 256
        e = self.emoji[_zipf_ids(rng, k, len(self.emoji), 1.0)]
        mod = np.where(rng.random(k) < 0.15, self.skin[rng.integers(0, len(self.skin), k)],
                       np.where(rng.random(k) < 0.10, self.vs16, self.empty))
        join = np.where(rng.random(k) < 0.10, self.zwj, np.where(rng.random(k) < 0.3, self.space, self.empty))
        return self.sf.assemble(np.stack([e, mod, join], 1).reshape(-1))


def corpus_c5(n_docs: int = 1_000_000, seed: int = 5):
    g = MultiGen(seed)
    rng = g.rng
    lengths = rng.integers(64, 513, size=n_docs)
    kind = rng.random(n_docs)
    parts = []
    # build per-doc by mixing segments: 40% CJK, 20% emoji, 40% ASCII bytes overall
    total = int(lengths.sum())
    cjk = g.cjk_stream(int(total * 0.45) + 4096)
    emo = g.emoji_stream(int(total * 0.25) + 4096)
    eng = g.eng.stream(int(total * 0.45) + 4096)
    pc = pe = pa = 0
    docs = []
    for i in range(n_docs):
        L = int(lengths[i])
        segs = []
        got = 0
        while got < L:
            r = rng.random()
            n = int(rng.integers(8, 96))
            if r < 0.4:
                src, p = cjk, pc
            elif r < 0.6:
                src, p = emo, pe
            else:
                src, p = eng, pa
            q = p + n
            while q < len(src) and (src[q] & 0xC0) == 0x80:
                q += 1
            seg = src[p:q].tobytes()
            if r < 0.4:
                pc = q
            elif r < 0.6:
                pe = q
            else:
                pa = q
            if pc > len(cjk) - 1024:
                pc = 0
            if pe > len(emo) - 1024:
                pe = 0
            if pa > len(eng) - 1024:
                pa = 0
            # segment may start mid-character if p was mid-character: skip continuation bytes
            k = 0
            while k < len(seg) and (seg[k] & 0xC0) == 0x80:
                k += 1
            seg = seg[k:]
            segs.append(seg)
            got += len(seg)
        docs.append(b"".join(segs))
    del parts, kind
    return pack(docs)


# C5-NFC: C5 with NFC-active text in a fraction of the docs (the GPU NFC path's workload, verdict
# round 1 item 8): decomposed Latin (e + U+0301 -> U+00E9, A + U+030A + U+0301), Hangul conjoining
# jamo (composed to syllables), Devanagari with nukta / virama and Arabic harakat (non-zero
# combining classes, reordered by canonical order), and combining marks stacked out of order.
_NFC_SNIPPETS = [s.encode() for s in [
    "caf\u0065\u0301 ", "A\u030a\u0301ngstr\u00f6m ", "\u1100\u1161\u11a8\u1100\u1161 ", "\u0915\u093c\u094d\u0937 ",
    "\u0928\u092e\u0938\u094d\u0924\u0947 ", "\u0628\u0650\u0633\u0652\u0645\u0650 ", "a\u0323\u0302b\u0302\u0323 ",
    "o\u0308\u0304 ", "\u212b \u2126 ", "n\u0303o\u0303 ", "\u05e9\u05c1\u05b8 ", "\u0e01\u0e48\u0e32 "]]


def corpus_c5nfc(n_docs: int = 1_000_000, seed: int = 5, frac: float = 0.03, base=None):
    """C5's docs with one NFC-active snippet spliced (at a char boundary) into `frac` of them.
    `base`: corpus_c5(n_docs, seed) when the caller already has it."""
    text, off = base if base is not None else corpus_c5(n_docs, seed)
    docs = unpack(text, off)
    rng = np.random.default_rng([seed, 0x4E4643])
    pick = rng.choice(n_docs, size=max(1, int(n_docs * frac)), replace=False)
    for j, d in enumerate(pick):
        sn = _NFC_SNIPPETS[j % len(_NFC_SNIPPETS)]
        doc = docs[d]
        cut = int(rng.integers(0, len(doc) + 1))
        while 0 < cut < len(doc) and (doc[cut] & 0xC0) == 0x80:
            cut -= 1
        docs[d] = doc[:cut] + sn + doc[cut:]
    return pack(docs)


# ----------------------------------------------------------------------------- helpers

def pack(docs: list[bytes]):
    lens = np.fromiter((len(d) for d in docs), dtype=np.int64, count=len(docs))
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    text = np.frombuffer(b"".join(docs), dtype=np.uint8).copy()
    return text, off


def unpack(text: np.ndarray, off: np.ndarray) -> list[bytes]:
    t = text.tobytes()
    o = off.astype(np.int64)
    return [t[o[i]:o[i + 1]] for i in range(len(o) - 1)]


CONFIGS = {"C1": corpus_c1, "C2": corpus_c2, "C3": corpus_c3, "C4": corpus_c4, "C5": corpus_c5,
           "C5NFC": corpus_c5nfc}
