"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the INL-BPE trainer.

Line-by-line Python restatement of `InlBpeTrainer` (reference src/trainer.rs), the checker for the
GPU pair counting / merge application behind `complexity_tokenizer.Trainer`.  The product never
imports it.

What the reference leaves unspecified, and the choice made here (the product makes the same one):
  * init_vocab_bytelevel (src/trainer.rs:296-339) numbers the alphabet in the iteration order of a
    hashbrown HashSet (randomly seeded): here the chars get ids in ascending code point order.
  * learn_merges_heap pops a std BinaryHeap ordered by the f32 score alone (src/trainer.rs:131-136);
    among equal scores the pop order follows the heap's internal layout, i.e. the HashMap
    iteration order it was built from (randomly seeded).  Here equal scores pop in ascending
    (vocab_r[a], vocab_r[b]) UTF-8 byte order, then ascending (a, b).
Every other step is deterministic in the reference and restated exactly, including the f32
arithmetic of build_heap (numpy.float32, one rounding per operation, no fused multiply-add) and the
vocab-size quirk of a merged string that is already in the vocab (insert overwrites its id, the
vocab does not grow, the next merge reuses the same new id).

Pinning: the reference's own trainer tests (src/trainer.rs:659-707: byte map, basic training,
heap correctness) are re-run against this module in tests/test_trainer_cpu.py; the pair counts
of compute_initial_pairs are checked against a direct collections.Counter of the words' pairs.
"""
from __future__ import annotations

import unicodedata

import numpy as np

from oracle.ref_py import GPT2_PATTERN, bytes_to_unicode

F32 = np.float32
DEFAULT_SPECIALS = ["</s>", "<pad>", "<s>", "<unk>"]


def rust_lines(data: bytes):
    """BufRead::lines (Rust std): split on b'\\n'; a line that ended in b'\\n' also drops one b'\\r'
    before it, an unterminated last line keeps its b'\\r'; UTF-8 or error."""
    if not data:
        return []
    parts = data.split(b"\n")
    last = parts.pop()
    out = []
    for p in parts:
        if p.endswith(b"\r"):
            p = p[:-1]
        out.append(p.decode("utf-8"))  # UnicodeDecodeError ~ io::ErrorKind::InvalidData
    if last:
        out.append(last.decode("utf-8"))
    return out


class RefTrainer:
    """src/trainer.rs:66-149 (TrainerConfig defaults) and :165-632."""

    def __init__(self, vocab_size=32000, min_frequency=2, special_tokens=None, min_word_length=1, inl_alpha=0.9,
                 inl_beta=0.3, inl_gate=0.5, inl_mu_target=0.01, inl_velocity_max=10.0, inl_beta_max=2.0):
        self.vocab_size = vocab_size
        self.min_frequency = min_frequency
        self.special_tokens = list(DEFAULT_SPECIALS if special_tokens is None else special_tokens)
        self.min_word_length = min_word_length
        self.alpha, self.beta, self.gate = F32(inl_alpha), F32(inl_beta), F32(inl_gate)
        self.mu_target, self.vmax, self.beta_max = F32(inl_mu_target), F32(inl_velocity_max), F32(inl_beta_max)
        self.vocab: dict[str, int] = {}
        self.vocab_r: dict[int, str] = {}
        self.merges: list[tuple[str, str]] = []
        self.token_freqs: dict[int, int] = {}
        self.velocity: dict[int, np.float32] = {}
        self.pair_freqs: dict[tuple[int, int], int] = {}
        self.acc: dict[str, int] = {}
        self.byte_encoder = bytes_to_unicode()
        self.initial_pairs = None  # compute_initial_pairs result, kept for the parity tests

    # src/trainer.rs:171-185 (normalizer NFC, pre-tokenizer ByteLevel{add_prefix_space: false})
    def pretokenize(self, text):
        text = unicodedata.normalize("NFC", text)
        words = []
        for m in GPT2_PATTERN.finditer(text):
            enc = "".join(self.byte_encoder[b] for b in m.group(0).encode("utf-8"))
            if enc:
                words.append(enc)
        return words

    def _count_into(self, freqs, texts):
        for text in texts:
            for w in self.pretokenize(text):
                if len(w) >= self.min_word_length:  # word.chars().count()
                    freqs[w] = freqs.get(w, 0) + 1

    def train_files(self, paths):  # src/trainer.rs:187-193, count_words :265-285
        wf = {}
        for p in paths:
            with open(p, "rb") as f:
                self._count_into(wf, rust_lines(f.read()))
        wf = {w: c for w, c in wf.items() if c >= self.min_frequency}
        self.train_from_word_freqs(wf)

    def train_from_texts(self, texts):  # :195-204, :245-263
        wf = {}
        self._count_into(wf, texts)
        wf = {w: c for w, c in wf.items() if c >= self.min_frequency}
        self.train_from_word_freqs(wf)

    def count_batch(self, texts):  # :207-220
        self._count_into(self.acc, texts)

    def finish_training(self):  # :223-229
        wf, self.acc = self.acc, {}
        wf = {w: c for w, c in wf.items() if c >= self.min_frequency}
        self.train_from_word_freqs(wf)

    def train_from_word_freqs(self, word_freqs):  # :231-243
        words = self.init_vocab_bytelevel(word_freqs)
        self.compute_initial_pairs(words)
        self.learn_merges_heap(words)

    def init_vocab_bytelevel(self, word_freqs):  # :288-339
        next_id = 0
        for tok in self.special_tokens:
            self.vocab[tok] = next_id
            self.vocab_r[next_id] = tok
            next_id += 1
        chars = sorted({c for w in word_freqs for c in w})  # (HashSet order in the reference)
        for c in chars:
            if c not in self.vocab:
                self.vocab[c] = next_id
                self.vocab_r[next_id] = c
                next_id += 1
        words = [[[self.vocab[c] for c in w if c in self.vocab], f] for w, f in word_freqs.items()]
        for toks, f in words:
            for t in toks:
                self.token_freqs[t] = self.token_freqs.get(t, 0) + f
        for i in self.vocab.values():
            self.velocity[i] = F32(0.0)
        return words

    def compute_initial_pairs(self, words):  # :341-367
        pc = {}
        for toks, f in words:
            for i in range(len(toks) - 1):
                k = (toks[i], toks[i + 1])
                pc[k] = pc.get(k, 0) + f
        self.pair_freqs = pc
        self.initial_pairs = dict(pc)

    def scores(self):  # build_heap :369-405, as a list in pop order
        total = sum(self.token_freqs.values())
        mu = self.mu_target * F32(total)
        beta_c = max(min(self.beta, self.beta_max), F32(0.0))
        out = []
        for (a, b), f in self.pair_freqs.items():
            if f <= 0:
                continue
            base = F32(f)
            fa, fb = F32(self.token_freqs.get(a, 0)), F32(self.token_freqs.get(b, 0))
            ea, eb = fa - mu, fb - mu
            va, vb = self.velocity.get(a, F32(0.0)), self.velocity.get(b, F32(0.0))
            van = min(max(self.alpha * va - beta_c * ea, -self.vmax), self.vmax)
            vbn = min(max(self.alpha * vb - beta_c * eb, -self.vmax), self.vmax)
            score = base - self.gate * (van + vbn)
            out.append((score, a, b))
        key = lambda e: (-float(e[0]), self.vocab_r[e[1]].encode(), self.vocab_r[e[2]].encode(), e[1], e[2])
        out.sort(key=key)
        return out

    def learn_merges_heap(self, words):  # :407-520
        target = self.vocab_size
        while len(self.vocab) < target:
            heap = self.scores()
            hi = 0
            for _ in range(100):
                if len(self.vocab) >= target:
                    break
                best = None
                while hi < len(heap):
                    s, a, b = heap[hi]
                    hi += 1
                    if self.pair_freqs.get((a, b), 0) > 0:
                        best = (a, b)
                        break
                if best is None:
                    break
                a, b = best
                ta, tb = self.vocab_r[a], self.vocab_r[b]
                merged = ta + tb
                new_id = len(self.vocab)
                self.vocab[merged] = new_id
                self.vocab_r[new_id] = merged
                self.merges.append((ta, tb))
                self.apply_merge_incremental(words, best, new_id)
                self.velocity[new_id] = (self.velocity.get(a, F32(0.0)) + self.velocity.get(b, F32(0.0))) / F32(2.0)
            if not any(v > 0 for v in self.pair_freqs.values()):
                break

    def apply_merge_incremental(self, words, pair, new_id):  # :522-590
        self.pair_freqs.pop(pair, None)
        a, b = pair
        deltas = {}
        new_tf = 0
        for w in words:
            toks, f = w
            i = 0
            while i < len(toks) - 1:
                if toks[i] == a and toks[i + 1] == b:
                    if i > 0:
                        k = (toks[i - 1], a)
                        deltas[k] = deltas.get(k, 0) - f
                    if i + 2 < len(toks):
                        k = (b, toks[i + 2])
                        deltas[k] = deltas.get(k, 0) - f
                    toks[i] = new_id
                    del toks[i + 1]
                    if i > 0:
                        k = (toks[i - 1], new_id)
                        deltas[k] = deltas.get(k, 0) + f
                    if i + 1 < len(toks):
                        k = (new_id, toks[i + 1])
                        deltas[k] = deltas.get(k, 0) + f
                    new_tf += f
                else:
                    i += 1
        for k, d in deltas.items():
            self.pair_freqs[k] = self.pair_freqs.get(k, 0) + d
        if a in self.token_freqs:
            self.token_freqs[a] = max(0, self.token_freqs[a] - new_tf)
        if b in self.token_freqs:
            self.token_freqs[b] = max(0, self.token_freqs[b] - new_tf)
        self.token_freqs[new_id] = new_tf
        self.pair_freqs = {k: v for k, v in self.pair_freqs.items() if v > 0}

    def to_json(self):  # save(), src/trainer.rs:600-645 (serde_json::Value maps are key-sorted)
        return {
            "version": "1.0",
            "model": {"type": "BPE", "vocab": dict(self.vocab), "merges": ["%s %s" % m for m in self.merges]},
            "added_tokens": [{"id": i, "content": t, "special": True, "single_word": False, "lstrip": False,
                              "rstrip": False, "normalized": False} for i, t in enumerate(self.special_tokens)],
            "pre_tokenizer": {"type": "ByteLevel", "add_prefix_space": False, "use_regex": True},
            "decoder": {"type": "ByteLevel"},
        }
