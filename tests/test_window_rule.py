"""The window rounds of the segmented long-piece tier (kernels.hip bpe_wave_seg) restated in
Python (tests/window_model.py) against the reference's sequential merge loop (oracle/ref_py.py,
src/bpe.rs:88-153): random rank-monotone tables with long tokens (wide windows), the Llama-3-shaped
fixture on C3-like runs, and the round counts that make the rule worth it."""
import json

import numpy as np
import pytest

from oracle.ref_py import RefTokenizer
from tests import toys
from tests.window_model import eager_set, window_bpe, window_bpe_dense, window_meta


def _ids(tok, data: bytes):
    be = toys.byte_map()
    return [tok.vocab[be[b]] for b in data if be[b] in tok.vocab]


@pytest.mark.parametrize("seed", range(12))
def test_window_rounds_random_proper_tables(seed):
    tok = RefTokenizer(toys.random_proper(seed, alphabet="abc"[: 2 + seed % 2], max_len=8 + 3 * seed))
    assert window_meta(tok) is not None
    rng = np.random.default_rng(seed)
    for n in [2, 5, 17, 64, 130, 300, 700]:
        for _ in range(3):
            data = bytes(rng.choice(list(b"abc"[: 2 + seed % 2]), size=n).astype(np.uint8))
            ids = _ids(tok, data)
            want = tok.bpe("".join(toys.byte_map()[b] for b in data))
            for k in (16, 64):
                got, _ = window_bpe(tok, ids, k=k)
                assert got == want, (seed, n, k)
            assert window_bpe_dense(tok, ids)[0] == want, (seed, n, "dense")


MULTI = ["日本語", "かなカ", "한국어", "日a本", "\U0001F600\U0001F601", "éßø"]


@pytest.mark.parametrize("seed", range(len(MULTI)))
def test_window_rounds_multibyte_tables(seed):
    """The same on tables over the UTF-8 bytes of multi-byte chars (CJK / kana / Hangul / emoji /
    Latin-1 runs: the dense tier's C5 workload), pieces of random chars."""
    alpha = MULTI[seed]
    rng = np.random.default_rng(seed)
    sample = "".join(rng.choice(list(alpha), size=2000)).encode()
    tok = RefTokenizer(toys.random_proper_from_text(seed, sample, n_merges=120, max_len=9 + 2 * seed))
    assert window_meta(tok) is not None
    for n in [1, 3, 9, 22, 40, 85]:
        for _ in range(3):
            data = "".join(rng.choice(list(alpha), size=n)).encode()
            ids = _ids(tok, data)
            want = tok.bpe("".join(toys.byte_map()[b] for b in data))
            for k in (16, 64):
                assert window_bpe(tok, ids, k=k)[0] == want, (seed, n, k)
            assert window_bpe_dense(tok, ids)[0] == want, (seed, n, "dense")


def _non_monotone(seed):
    """Two tables that are not rank-monotone, from one random proper table: its merges shuffled,
    and re-laid out as the tiktoken conversion does (every split of every token, by the token's id:
    datagen/build_tokenizers.py tiktoken_style_merges)."""
    from datagen.build_tokenizers import tiktoken_style_merges
    alpha = ["abc", "ab", "abcd", "日本", "xyz"][seed % 5]
    rng = np.random.default_rng(seed)
    base = toys.random_proper_from_text(seed, "".join(rng.choice(list(alpha), size=2000)).encode(),
                                        n_merges=60 + seed % 80, max_len=6 + seed % 12)
    tt = json.loads(json.dumps(base))
    tt["model"]["merges"] = ["%s %s" % m for m in tiktoken_style_merges(tt["model"]["vocab"])]
    return alpha, rng, [toys.shuffled_merges(base, seed), tt]


@pytest.mark.parametrize("seed", range(16))
def test_window_rounds_non_monotone_tables(seed):
    """Window rounds on tables that are not rank-monotone (round 4): a candidate whose merge is
    eager also needs its new pairs with today's neighbours to rank above it and a window that covers
    the neighbours' windows (kernels.hip bpe_wave_seg / bpe_wave_dense).  Against the reference loop."""
    alpha, rng, objs = _non_monotone(seed)
    for o in objs:
        tok = RefTokenizer(o)
        assert window_meta(tok) is not None
        eg = eager_set(tok)
        assert eg  # (the table really is not rank-monotone)
        for n in [3, 10, 40, 100, 300]:
            data = "".join(rng.choice(list(alpha), size=n)).encode()
            ids = _ids(tok, data)
            want = tok.bpe("".join(toys.byte_map()[b] for b in data))
            for k in (16, 64):
                assert window_bpe(tok, ids, k=k, eager=eg)[0] == want, (seed, n, k)
            assert window_bpe_dense(tok, ids, eager=eg)[0] == want, (seed, n, "dense")


def test_window_rounds_tiktoken_layout_llama3(llama3_tt_path):
    """The 304k-merge tiktoken-layout Llama-3 fixture (C3TT): exact, and the eager-candidate rule
    cuts the rounds of C3-like runs several-fold (rank rounds alone: ~350-1200)."""
    with open(llama3_tt_path) as f:
        tok = RefTokenizer(json.load(f))
    eg = eager_set(tok)
    rng = np.random.default_rng(3)
    words = [w for w in (tok.id_to_token_map[i] for i in range(300, 8000)) if w.isalpha()][:3000]
    runs = [bytes(rng.integers(ord("a"), ord("z") + 1, size=1200).astype(np.uint8)),
            "".join(words[int(i)] for i in rng.integers(len(words), size=400)).encode()[:1200], b"q" * 1200]
    for data in runs:
        got, rounds = window_bpe(tok, _ids(tok, data), k=64, eager=eg)
        assert got == tok.bpe("".join(toys.byte_map()[b] for b in data))
        assert rounds < 60


def test_window_meta_refuses_shifted_ranks():
    """An invalid merge before valid ones shifts the new ids (src/bpe.rs:60-69): a merged token
    need not spell its two sides, so the window bound does not hold and the rule is off."""
    obj = toys.with_invalid_merges(toys.random_proper(1), seed=3, n_bad=5)
    assert window_meta(RefTokenizer(obj)) is None


def test_window_rounds_llama3_runs(llama3_path):
    with open(llama3_path) as f:
        tok = RefTokenizer(json.load(f))
    rng = np.random.default_rng(3)
    words = [w for w in (tok.id_to_token_map[i] for i in range(300, 8000)) if w.isalpha()][:3000]
    runs = [bytes(rng.integers(ord("a"), ord("z") + 1, size=1200).astype(np.uint8)),
            bytes(rng.integers(ord("0"), ord("9") + 1, size=1200).astype(np.uint8)),
            "".join(words[int(i)] for i in rng.integers(len(words), size=400)).encode()[:1200],
            b"q" * 1200]
    for data in runs:
        ids = _ids(tok, data)
        got, rounds = window_bpe(tok, ids, k=64)
        assert got == tok.bpe("".join(toys.byte_map()[b] for b in data))
        assert rounds < 60  # (rank rounds alone: ~300-400 on the first three)
