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
    # BufRead::lines drops '\r' only as part of "\r\n": an unterminated last line keeps it
    assert trainer_ref.rust_lines(b"a\r\nb\r") == ["a", "b\r"]
    assert trainer_ref.rust_lines(b"\r") == ["\r"]
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


@pytest.mark.parametrize("block", [1, 2, 3, 5, 64, 1 << 20])
def test_file_lines_streamed_in_blocks(tmp_path, block):
    """train(files) reads files in blocks: the lines must be BufRead::lines' for any block size
    (src/trainer.rs:272), including CRLF pairs and multi-byte chars cut by a block edge."""
    from complexity_tokenizer.trainer import _file_line_blocks
    for data in (b"", b"\n", b"a\r\nb\n\nc", b"x\n", "héllo wörld\r\n日本語\n\nend".encode(), b"\r\n\r\n", b"last",
                 b"end\r", b"a\r\nb\r", b"\r"):
        p = tmp_path / "f.txt"
        p.write_bytes(data)
        got = [ln for blk in _file_line_blocks(str(p), block) for ln in blk]
        assert got == trainer_ref.rust_lines(data), (data, block)


def naive_merges(word_freqs, n_vocab_target, n_base):
    """An independent restatement of learn_merges_heap's merge ORDER with inl_gate = 0 (score =
    pair count): string tokens, pair counts recounted from scratch with collections.Counter
    (no incremental deltas, no ids), the heap rebuilt every 100 merges from the true counts and
    popped in count order while stale entries are skipped (src/trainer.rs:407-520).  It asserts
    that no pop meets a live entry of the same score, so the result does not depend on how equal
    scores are ordered (the reference leaves that to hash order)."""
    import collections
    words = [[list(w), f] for w, f in word_freqs.items()]

    def counts():
        c = collections.Counter()
        for toks, f in words:
            for i in range(len(toks) - 1):
                c[(toks[i], toks[i + 1])] += f
        return c

    merges, vocab = [], n_base
    while vocab < n_vocab_target:
        heap = sorted(counts().items(), key=lambda kv: -kv[1])
        hi, progressed = 0, False
        for _ in range(100):
            if vocab >= n_vocab_target:
                break
            cur = counts()
            while hi < len(heap) and cur.get(heap[hi][0], 0) <= 0:
                hi += 1
            if hi == len(heap):
                break
            (a, b), score = heap[hi]
            ties = [p for p, s in heap[hi + 1:] if s == score and cur.get(p, 0) > 0]
            assert not ties, "tie at merge %d: %r and %r (score %d)" % (len(merges), (a, b), ties[0], score)
            hi += 1
            merges.append((a, b))
            vocab += 1
            progressed = True
            for w in words:  # apply_merge_incremental's left-to-right loop (:537-577)
                toks, i = w[0], 0
                while i < len(toks) - 1:
                    if toks[i] == a and toks[i + 1] == b:
                        toks[i:i + 2] = [a + b]
                    else:
                        i += 1
        if not progressed or not any(v > 0 for v in counts().values()):
            break
    return merges


def tie_free_word_freqs(seed=11, n_words=300):
    rng = random.Random(seed)
    wf = {}
    while len(wf) < n_words:
        w = "".join(rng.choice("abcdefg") for _ in range(rng.randint(2, 9)))
        wf.setdefault(w, rng.randint(1, 10 ** 7))
    return wf


def test_trainer_oracle_merge_order_pinned_without_ties():
    """the oracle's merge sequence against an independent Counter recount on counts
    with no equal live scores, so the tie-break choice cannot hide a mistake.  Two heap builds
    (more merges than the 49 initial pairs of a 7-letter alphabet)."""
    wf = tie_free_word_freqs()
    n_base = 4 + 7  # the default specials + the alphabet
    target = n_base + 70
    want = naive_merges(wf, target, n_base)
    assert len(want) == 70
    ref = trainer_ref.RefTrainer(vocab_size=target, min_frequency=1, inl_gate=0.0)
    ref.train_from_word_freqs(dict(wf))
    assert ref.merges == want


@pytest.mark.parametrize("threads", [1, 4])
def test_trainer_c_restatement_matches_oracle(threads):
    """oracle/trainer_ref.c (the CPU timing baseline of the trainer, tools/trainer_timing.py) applies
    a training run's merges with the reference's bookkeeping: its final words and live pair count
    must equal oracle/trainer_ref.py's after the same training."""
    import copy
    from oracle import trainer_c
    from datagen import corpus
    text, off = corpus.corpus_c1()
    texts = [d.decode() for d in corpus.unpack(text, off)][:400]
    ref = trainer_ref.RefTrainer(vocab_size=350, min_frequency=1)
    wf = {}
    ref._count_into(wf, texts)
    words = ref.init_vocab_bytelevel(wf)
    start = copy.deepcopy(words)
    tf0 = dict(ref.token_freqs)
    ref.compute_initial_pairs(words)
    ref.learn_merges_heap(words)
    merges = [(ref.vocab[a], ref.vocab[b], ref.vocab[a + b]) for a, b in ref.merges]
    assert len(merges) > 30
    got, _, _, live = trainer_c.run([(t, f) for t, f in start], merges, tf0, len(ref.vocab) + 1, threads)
    assert got == [t for t, _ in words]
    assert live == len(ref.pair_freqs)
