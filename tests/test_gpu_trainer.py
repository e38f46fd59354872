"""GPU parity of the trainer: the GPU pair histogram
(compute_initial_pairs, src/trainer.rs:341-367) and the GPU merge passes with their pair-count
deltas (apply_merge_incremental, :522-590) against oracle/trainer_ref.py, whole trainings
compared merge by merge, the saved tokenizer.json byte for byte, and the reference's own trainer
tests (src/trainer.rs:669-706) through the product."""
import json
import random

import numpy as np
import pytest

from complexity_tokenizer import Tokenizer, Trainer
from datagen import corpus
from oracle import ref_py, trainer_ref

pytestmark = pytest.mark.gpu


def _texts(seed, n, alpha, lo=1, hi=40):
    rng = random.Random(seed)
    return ["".join(rng.choice(alpha) for _ in range(rng.randint(lo, hi))) for _ in range(n)]


def _c1_texts(n=400):
    text, off = corpus.corpus_c1()
    return [d.decode() for d in corpus.unpack(text, off)][:n]


def _both(texts, **kw):
    gpu = Trainer(**kw)
    gpu.train_from_iterator(texts)
    ref = trainer_ref.RefTrainer(**kw)
    ref.train_from_texts(texts)
    return gpu, ref


def _same(gpu, ref):
    want = json.dumps(ref.to_json(), indent=2, sort_keys=True, ensure_ascii=False)
    got = gpu.to_str()
    if got != want:
        g, w = json.loads(got), json.loads(want)
        gm, wm = g["model"]["merges"], w["model"]["merges"]
        k = next((i for i in range(min(len(gm), len(wm))) if gm[i] != wm[i]), min(len(gm), len(wm)))
        raise AssertionError("first differing merge %d: gpu %r, oracle %r (of %d / %d)"
                             % (k, gm[k:k + 1], wm[k:k + 1], len(gm), len(wm)))
    assert gpu.vocab_size == len(ref.vocab) and gpu.num_merges == len(ref.merges)


def test_initial_pair_histogram_c1():
    texts = _c1_texts(1000)
    gpu, ref = _both(texts, vocab_size=300, min_frequency=1)
    a, b, c = gpu.initial_pairs()
    got = {(int(x), int(y)): int(z) for x, y, z in zip(a, b, c)}
    assert got == ref.initial_pairs
    assert len(got) > 100


def test_training_matches_oracle_c1():
    gpu, ref = _both(_c1_texts(600), vocab_size=400, min_frequency=2)
    assert gpu.num_merges > 50
    _same(gpu, ref)


def test_training_matches_oracle_small_alphabet():
    """Two letters and a space: long (x, x) runs, overlapping occurrences in one word, and merged
    strings that are already in the vocab (the reference's insert-overwrite quirk)."""
    gpu, ref = _both(_texts(3, 500, "aab "), vocab_size=120, min_frequency=1)
    _same(gpu, ref)


def test_training_matches_oracle_unicode_and_nfc():
    """Multi-byte chars (2..4 byte UTF-8) and decomposed sequences that NFC composes on the GPU."""
    alpha = ["é", "é", "中", "文", "😀", "a", " ", "ñ", "ß"]
    gpu, ref = _both(_texts(4, 400, alpha, 1, 12), vocab_size=200, min_frequency=1)
    _same(gpu, ref)


@pytest.mark.parametrize("alpha,beta,gate", [(0.9, 0.3, 0.5), (0.0, 0.0, 0.0), (0.5, 1.5, 2.0)])
def test_inl_parameters(alpha, beta, gate):
    gpu, ref = _both(_c1_texts(300), vocab_size=250, min_frequency=1, inl_alpha=alpha, inl_beta=beta, inl_gate=gate)
    _same(gpu, ref)


def test_count_batch_finish_equals_train_from_iterator():
    texts = _c1_texts(500)
    one = Trainer(vocab_size=300, min_frequency=2)
    one.train_from_iterator(texts)
    two = Trainer(vocab_size=300, min_frequency=2)
    for i in range(0, len(texts), 128):
        two.count_batch(texts[i:i + 128])
    two.finish_training()
    assert one.to_str() == two.to_str()


def test_train_files_crlf_and_min_word_length(tmp_path):
    p = tmp_path / "a.txt"
    p.write_bytes("hello world hello world\r\nhello hello hello\nwörld wörld\n".encode())
    gpu = Trainer(vocab_size=60, min_frequency=1, min_word_length=3)
    gpu.train([str(p)])
    ref = trainer_ref.RefTrainer(vocab_size=60, min_frequency=1, min_word_length=3)
    ref.train_files([str(p)])
    _same(gpu, ref)


def test_reference_trainer_tests_through_the_product(tmp_path):
    """src/trainer.rs:669-706 (basic training, heap correctness)."""
    p = tmp_path / "t.txt"
    p.write_text("hello world hello world\nhello hello hello\n")
    t = Trainer(vocab_size=50, min_frequency=1)
    t.train([str(p)])
    assert t.vocab_size > 10 and t.num_merges > 0
    q = tmp_path / "h.txt"
    q.write_text("aaa bbb aaa bbb ccc\n")
    t = Trainer(vocab_size=30, min_frequency=1, inl_alpha=0.0, inl_beta=0.0, inl_gate=0.0)
    t.train([str(q)])
    assert t.num_merges > 0


def test_saved_tokenizer_encodes_like_the_oracle(tmp_path):
    texts = _c1_texts(800)
    t = Trainer(vocab_size=500, min_frequency=2)
    t.train_from_iterator(texts)
    path = tmp_path / "tok.json"
    t.save(str(path))
    tok = Tokenizer.from_file(str(path))
    tok.device = 0
    with open(path) as f:
        ref = ref_py.RefTokenizer(json.load(f))
    docs = texts[:200]
    assert tok.encode_batch(docs) == ref.encode_batch(docs)


def test_larger_training_and_timing():
    """A 20k-doc C2 sample (~2.5 MB): a few thousand merges, the GPU pair passes timed."""
    text, off = corpus.corpus_c2(20_000, seed=7)
    texts = [d.decode() for d in corpus.unpack(text, off)]
    gpu = Trainer(vocab_size=2000, min_frequency=2)
    gpu.train_from_iterator(texts)
    tm = gpu.timing()
    print("trainer timing", tm, "merges", gpu.num_merges)
    ref = trainer_ref.RefTrainer(vocab_size=2000, min_frequency=2)
    wf = {}
    ref._count_into(wf, texts)
    wf = {w: c for w, c in wf.items() if c >= 2}
    words = ref.init_vocab_bytelevel(wf)
    ref.compute_initial_pairs(words)
    a, b, c = gpu.initial_pairs()
    assert {(int(x), int(y)): int(z) for x, y, z in zip(a, b, c)} == ref.initial_pairs
    assert gpu.num_merges >= 2000 - len(ref.vocab)


def test_merge_order_pinned_without_ties():
    """The product against the independent Counter recount of tests/test_trainer_cpu.py on counts
    with no equal live scores (the order does not depend on the tie-break choice)."""
    from tests.test_trainer_cpu import naive_merges, tie_free_word_freqs
    wf = tie_free_word_freqs()
    target = 4 + 7 + 70
    want = naive_merges(wf, target, 4 + 7)
    t = Trainer(vocab_size=target, min_frequency=1, inl_gate=0.0)
    t.train_from_word_freqs({w.encode(): f for w, f in wf.items()})
    got = [tuple(m.split(" ")) for m in json.loads(t.to_str())["model"]["merges"]]
    assert got == want


def test_word_counting_in_chunks_equals_one_call(monkeypatch):
    """count() hands the texts to the GPU pre-tokenizer in doc-aligned chunks
    (CTOK_TRAIN_CHUNK_BYTES, default 256 MB); the counts, hence the training, must not depend on
    the chunking (chunks of a few docs here, and a doc longer than a chunk)."""
    texts = _c1_texts(600) + ["x" * 5000 + " tail"]
    one = Trainer(vocab_size=300, min_frequency=2)
    one.train_from_iterator(texts)
    monkeypatch.setenv("CTOK_TRAIN_CHUNK_BYTES", "700")
    many = Trainer(vocab_size=300, min_frequency=2)
    many.train_from_iterator(texts)
    assert one.to_str() == many.to_str()


def test_train_files_streamed_in_blocks(tmp_path):
    """train(files) reads and counts each file in blocks (lines cut by a block edge carried
    over); small blocks and several files give the one-block result, and the oracle's."""
    texts = _c1_texts(400)
    paths = []
    for k in range(3):
        p = tmp_path / ("f%d.txt" % k)
        p.write_bytes(("\r\n".join(texts[k::3]) + ("\n" if k != 1 else "")).encode())
        paths.append(str(p))
    big = Trainer(vocab_size=300, min_frequency=2)
    big.train(paths)
    small = Trainer(vocab_size=300, min_frequency=2)
    small.train(paths, block_bytes=97)
    assert big.to_str() == small.to_str()
    ref = trainer_ref.RefTrainer(vocab_size=300, min_frequency=2)
    ref.train_files(paths)
    _same(small, ref)


def test_train_files_bad_utf8_drops_partial_counts(tmp_path):
    """A line that is not UTF-8 after blocks were counted: IOError, and the counts made so far are
    dropped (the reference returns the error before keeping anything, src/trainer.rs:265-285), so a
    later training sees only its own texts."""
    good = tmp_path / "good.txt"
    good.write_bytes(("hello world\n" * 200).encode())
    bad = tmp_path / "bad.txt"
    bad.write_bytes(b"fine line\n" * 50 + b"\xff\xfe\n")
    t = Trainer(vocab_size=60, min_frequency=1)
    with pytest.raises(IOError):
        t.train([str(good), str(bad)], block_bytes=64)
    t2 = Trainer(vocab_size=60, min_frequency=1)
    other = ["abc abd abe"] * 5
    t.train_from_iterator(other)
    t2.train_from_iterator(other)
    assert t.to_str() == t2.to_str()
