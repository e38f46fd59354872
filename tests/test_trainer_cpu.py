"""CPU tests of the trainer: the oracle restatement (oracle/trainer_ref.py)
against the reference's own trainer tests (src/trainer.rs:659-707) and a direct pair count; the
Trainer's argument handling and its save() JSON before training; no GPU needed."""
import collections
import json
import random

import pytest

from complexity_tokenizer import DeviceError, Trainer
from oracle import trainer_ref
from oracle.ref_py import bytes_to_unicode


def test_kat_byte_level_encoding():
    """src/trainer.rs:659-667."""
    enc = bytes_to_unicode()
    assert len(enc) == 256
    assert enc[ord("a")] == "a" and enc[ord("Z")] == "Z"


def test_kat_basic_training(tmp_path):
    """src/trainer.rs:669-686."""
    p = tmp_path / "t.txt"
    p.write_text("hello world hello world\nhello hello hello\n")
    tr = trainer_ref.RefTrainer(vocab_size=50, min_frequency=1)
    tr.train_files([str(p)])
    assert len(tr.vocab) > 10
    assert tr.merges


def test_kat_heap_correctness(tmp_path):
    """src/trainer.rs:688-706."""
    p = tmp_path / "t.txt"
    p.write_text("aaa bbb aaa bbb ccc\n")
    tr = trainer_ref.RefTrainer(vocab_size=30, min_frequency=1, inl_alpha=0.0, inl_beta=0.0, inl_gate=0.0)
    tr.train_files([str(p)])
    assert tr.merges


def _random_texts(seed, n, alpha="ab c", lo=1, hi=30):
    rng = random.Random(seed)
    return ["".join(rng.choice(alpha) for _ in range(rng.randint(lo, hi))) for _ in range(n)]


def test_initial_pairs_are_a_pair_histogram():
    tr = trainer_ref.RefTrainer(vocab_size=10, min_frequency=1)
    texts = _random_texts(1, 300, "abcd éü\n")
    tr.train_from_texts(texts)
    wf = collections.Counter(w for t in texts for w in tr.pretokenize(t))
    want = collections.Counter()
    for w, f in wf.items():
        ids = [tr.vocab[c] for c in w]
        for x, y in zip(ids, ids[1:]):
            want[(x, y)] += f
    assert tr.initial_pairs == dict(want)


def test_merge_strings_concatenate_and_vocab_grows():
    tr = trainer_ref.RefTrainer(vocab_size=80, min_frequency=1)
    tr.train_from_texts(_random_texts(2, 400, "ab c"))
    assert tr.merges
    for a, b in tr.merges:
        assert a + b in tr.vocab
    # specials first, then the alphabet in code point order
    assert [tr.vocab_r[i] for i in range(4)] == trainer_ref.DEFAULT_SPECIALS
    alpha = [tr.vocab_r[i] for i in range(4, 4 + len({c for t in tr.vocab for c in t if len(t) == 1}) - 4)]
    assert alpha == sorted(alpha)


def test_rust_lines():
    assert trainer_ref.rust_lines(b"a\r\nb\n\nc") == ["a", "b", "", "c"]
    assert trainer_ref.rust_lines(b"") == []
    assert trainer_ref.rust_lines(b"x\n") == ["x"]
    with pytest.raises(UnicodeDecodeError):
        trainer_ref.rust_lines(b"\xff\n")


def test_trainer_json_before_training_matches_oracle():
    t = Trainer(vocab_size=100, min_frequency=1, special_tokens=["<s>", 'q"\\\n'])
    want = trainer_ref.RefTrainer(vocab_size=100, special_tokens=["<s>", 'q"\\\n']).to_json()
    s = t.to_str()
    assert json.loads(s) == want
    assert s == json.dumps(want, indent=2, sort_keys=True, ensure_ascii=False)
    assert t.vocab_size == 0 and t.num_merges == 0


def test_trainer_argument_errors():
    with pytest.raises(TypeError):
        Trainer(vocab_size="10")
    with pytest.raises(OverflowError):
        Trainer(min_frequency=-1)
    with pytest.raises(TypeError):
        Trainer(special_tokens="<s>")
    with pytest.raises(TypeError):
        Trainer().train("file.txt")


def test_trainer_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(DeviceError):
        Trainer(vocab_size=50, min_frequency=1).train_from_iterator(["hello world"])
    with pytest.raises(DeviceError):
        Trainer(vocab_size=50, min_frequency=1).train_from_word_freqs({b"ab": 2})


def test_trainer_missing_file_is_ioerror(tmp_path):
    with pytest.raises(IOError):
        Trainer().train([str(tmp_path / "missing.txt")])
    p = tmp_path / "bad.txt"
    p.write_bytes(b"ok\n\xff\xfe\n")
    with pytest.raises(IOError):
        Trainer().train([str(p)])
