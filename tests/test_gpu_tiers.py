"""Every length tier of the BPE kernels against the C oracle, at and around its boundaries:
the whole-piece probe (<= 8 B), the register passes (9..16, 17..32, 33..64 B: k_bpe_short,
k_bpe_c2, k_bpe_c3), the dense wave tiers (65..256, 257..2048, 2049..4096 B: k_bpe_wave) and
the global-memory linked-list tier beyond 4096 B (k_bpe_long).  Each length is tried with
letters drawn from a small alphabet (many merges), with (x, x) chains ("aaaa", "====", whose
rounds take every other site), with two-token periods, with multi-byte letters (CJK, 3 bytes
each) and with a table that is not rank-monotone (one site per round)."""
import json
import os
import random

import pytest

from complexity_tokenizer import Tokenizer
from datagen import corpus
from oracle import ref_c
from tests import toys
from tests.test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu

LENGTHS = [8, 9, 16, 17, 31, 32, 33, 40, 63, 64, 65, 100, 255, 256, 257, 1000, 2047, 2048, 2049, 3000, 4095,
           4096, 4097, 6000]


def tier_docs(seed):
    rng = random.Random(seed)
    docs = []
    for n in LENGTHS:
        docs.append("".join(rng.choice("etaoinshr") for _ in range(n)))        # letters, many merges
        docs.append("a" * n)                                                   # (x, x) chain
        docs.append("=" * n)                                                   # punctuation chain
        docs.append(("th" * n)[:n])                                            # two-token period
        docs.append("".join(rng.choice("一二三四五六七八九十") for _ in range(max(1, n // 3))))  # 3-byte letters
        docs.append(" " + "".join(rng.choice("0123456789") for _ in range(n - 1)))  # attached space + digits
    rng.shuffle(docs)
    return docs


@pytest.fixture(scope="module")
def gpt2(gpt2_path):
    with open(gpt2_path) as f:
        obj = json.load(f)
    return obj, Tokenizer.from_file(gpt2_path), ref_c.RefC(obj)


def check(tok, rc, docs):
    text, off = corpus.pack([d.encode() for d in docs])
    assert_same(*tok.encode_packed(text, off, timing=True), *rc.encode_packed(text, off))
    return tok.last_stats


def test_tiers_gpt2(gpt2):
    _, tok, rc = gpt2
    st = check(tok, rc, tier_docs(1))
    assert st["long_pieces"] > 0 and st["class_ids"][3] > 0


def test_tiers_multilingual(multi_path):
    with open(multi_path) as f:
        obj = json.load(f)
    check(Tokenizer.from_file(multi_path), ref_c.RefC(obj), tier_docs(2))


def test_tiers_improper_table(gpt2):
    obj, _, _ = gpt2
    sh = toys.shuffled_merges(obj, seed=5)
    check(Tokenizer.from_str(json.dumps(sh)), ref_c.RefC(sh), tier_docs(3))


def test_tiers_many_docs_interleaved(gpt2):
    """Tiers running side by side in one call (merge passes on the main stream, long tiers on the
    side stream) over a C2 sample with long docs spliced in."""
    _, tok, rc = gpt2
    text, off = corpus.corpus_c2(20_000, seed=31)
    docs = [d.decode() for d in corpus.unpack(text, off)]
    extra = tier_docs(4)
    for i, d in enumerate(extra):
        docs.insert((i * 7919) % len(docs), d)
    check(tok, rc, docs)


def test_pieces_across_tile_ends(gpt2, multi_path):
    """Pieces that start in the last bytes of a 3968-byte pre-tokenizer tile and end in the next
    one: past the tile's look-ahead they go to the long list even when shorter than 64 bytes."""
    tile = 3968
    rng = random.Random(9)
    docs, pos = [], 0
    for delta in range(1, 80):
        for n in (33, 60, 62, 63, 64, 65, 70, 130):
            target = ((pos + 200) // tile + 1) * tile
            filler = target - delta - pos
            docs.append(("ab " * filler)[:filler])
            alpha = "一二三四五" if n % 2 else "etaoinshr"
            piece = "".join(rng.choice(alpha) for _ in range(n))
            piece = piece.encode()[:n].decode("utf-8", "ignore")
            docs.append(piece)
            pos = target - delta + len(piece.encode())
    _, tok, rc = gpt2
    check(tok, rc, docs)
    with open(multi_path) as f:
        obj = json.load(f)
    check(Tokenizer.from_file(multi_path), ref_c.RefC(obj), docs)


class _env:
    """Set an environment variable for the duration of a block (the library reads CTOK_C3_SPARSE
    on every call)."""

    def __init__(self, k, v):
        self.k, self.v = k, v

    def __enter__(self):
        self.old = os.environ.get(self.k)
        os.environ[self.k] = self.v

    def __exit__(self, *a):
        if self.old is None:
            del os.environ[self.k]
        else:
            os.environ[self.k] = self.old


@pytest.mark.parametrize("bound", ["0", "1", "100000000"])
def test_c3_register_and_sparse_paths(gpt2, multi_path, bound):
    """The 33..64 B class by either implementation, against the C oracle: the register pass
    (k_bpe_mid<3>; CTOK_C3_SPARSE=0 or a bound below the class's size) and the sparse path
    (k_bpe_sparse over k_segment's class-3 queue: a wavefront per piece, taken when the class holds at most the
    bound's pieces; 100000000 forces it on the multilingual sample's dense class 3)."""
    _, tok, rc = gpt2
    with open(multi_path) as f:
        mobj = json.load(f)
    mtok, mrc = Tokenizer.from_file(multi_path), ref_c.RefC(mobj)
    text, off = corpus.corpus_c5(20_000, seed=77)
    c5 = [d.decode() for d in corpus.unpack(text, off)]
    with _env("CTOK_C3_SPARSE", bound):
        st = check(tok, rc, tier_docs(5))
        assert st["class_ids"][3] > 0
        st5 = check(mtok, mrc, c5 + tier_docs(6))
        assert st5["class_ids"][3] > 1000  # (a dense class 3: CJK runs)
    with _env("CTOK_C3_SPARSE", "0"):
        ref5 = check(mtok, mrc, c5 + tier_docs(6))
    # both implementations merge the same pieces into the same number of ids
    assert st5["class_bytes"][3] == ref5["class_bytes"][3] and st5["class_ids"][3] == ref5["class_ids"][3]


@pytest.mark.parametrize("bound", ["default", "100000000"])
def test_c3_sparse_queue_shards(gpt2, bound):
    """k_segment's 64-shard class-3 queue (shard = tile % 64), against the C oracle.  Packed: 40
    pieces of 33..64 B in one tile of a ~200 KB batch; under the default bound (one piece per 16
    tiles, at least 64: capacity one piece per shard) that shard overflows and the report steers
    the call to the register pass; at 10^8 the sparse pass takes them.  Spread: one such piece in
    each of 12 tiles, taken by the sparse pass under either bound."""
    _, tok, rc = gpt2
    rng = random.Random(5)

    def word(n):
        return "".join(rng.choice("etaoinshrdlu") for _ in range(n))

    # (~4.6 KB documents with no class-3 piece: one piece at each one's end lands in a tile of its
    # own, 12 tiles, so in a shard of its own)
    filler = [" ".join(word(rng.randint(2, 9)) for _ in range(700)) for _ in range(12)]
    packed = [" ".join(word(rng.randint(33, 48)) for _ in range(40))] + filler
    spread = [f + " " + word(rng.randint(33, 60)) for f in filler]
    env = _env("CTOK_C3_SPARSE", bound) if bound != "default" else _env("CTOK_C3_SPARSE_UNUSED", "1")
    with env:
        assert check(tok, rc, packed)["class_ids"][3] > 0
        assert check(tok, rc, spread)["class_ids"][3] > 0


def test_c3_sparse_improper_and_wide_tables(gpt2, llama3_path):
    """The sparse path on a table that is not rank-monotone (serial rounds, no window merges) and
    on a wide (128k-vocabulary) table, against the C oracle."""
    obj, _, _ = gpt2
    sh = toys.shuffled_merges(obj, seed=9)
    with open(llama3_path) as f:
        lobj = json.load(f)
    with _env("CTOK_C3_SPARSE", "100000000"):
        check(Tokenizer.from_str(json.dumps(sh)), ref_c.RefC(sh), tier_docs(7))
        st = check(Tokenizer.from_file(llama3_path), ref_c.RefC(lobj), tier_docs(8))
        assert st["class_ids"][3] > 0
