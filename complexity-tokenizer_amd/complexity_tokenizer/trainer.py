"""`complexity_tokenizer.Trainer`: the INL-BPE trainer (reference src/bindings/trainers.rs:10-92 over
src/trainer.rs) with its pair counting on the GPU, through include/ctok_trainer.h.

Word counting pre-tokenizes on the GPU (NFC + ByteLevel, the encode path's k_segment); the pair
histogram and each merge's pass over the words run on the GPU; the INL-scored heap runs in the
native host runtime.  There is no CPU fallback: without a HIP device the calls raise DeviceError.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as _n


def _raise(code):
    from . import _raise as r
    r(code)


def _rust_lines(data: bytes, path: str):
    """BufRead::lines (src/trainer.rs:272): split on '\\n', the '\\r' of a "\\r\\n" ending dropped (a
    last line without '\\n' keeps its '\\r'), UTF-8 or an InvalidData io::Error (-> IOError)."""
    if not data:
        return []
    parts = data.split(b"\n")
    last = parts.pop()  # b"" after a trailing newline, else the unterminated last line
    out = [_line(p, path) for p in parts]
    if last:
        out.append(_line(last, path, False))
    return out


def _line(p: bytes, path: str, newline: bool = True) -> str:
    if newline and p.endswith(b"\r"):
        p = p[:-1]
    try:
        return p.decode("utf-8")
    except UnicodeDecodeError:
        raise IOError("stream did not contain valid UTF-8 (%s)" % path) from None


def _file_line_blocks(path: str, block: int):
    """The lines of a file as BufRead::lines yields them, in lists of about `block` bytes (the file
    is streamed, never held whole)."""
    with open(path, "rb") as f:  # IOError as the reference's File::open / read
        carry = b""
        while True:
            data = f.read(block)
            if not data:
                break
            parts = (carry + data).split(b"\n")
            carry = parts.pop()  # the unfinished last line (b"" after a trailing newline)
            if parts:
                yield [_line(p, path) for p in parts]
        if carry:  # a last line without '\n' keeps a trailing '\r'
            yield [_line(carry, path, False)]


class Trainer:
    """Trainer(vocab_size=32000, min_frequency=2, special_tokens=None, min_word_length=1,
    inl_alpha=0.9, inl_beta=0.3, inl_gate=0.5) -- src/bindings/trainers.rs:18-55."""

    def __init__(self, vocab_size=32000, min_frequency=2, special_tokens=None, min_word_length=1, inl_alpha=0.9,
                 inl_beta=0.3, inl_gate=0.5, device=0):
        for name, v in (("vocab_size", vocab_size), ("min_frequency", min_frequency),
                        ("min_word_length", min_word_length)):
            if not isinstance(v, (int, np.integer)) or isinstance(v, bool):
                raise TypeError("argument '%s': '%s' object cannot be interpreted as an integer" % (name, type(v).__name__))
            if v < 0:
                raise OverflowError("argument '%s': can't convert negative int to unsigned" % name)
        if min_frequency > 0xFFFFFFFF:
            raise OverflowError("argument 'min_frequency': out of range for u32")
        if special_tokens is None:
            special_tokens = ["</s>", "<pad>", "<s>", "<unk>"]
        if isinstance(special_tokens, (str, bytes)):
            raise TypeError("argument 'special_tokens': Can't extract `str` to `Vec`")
        sp = [s.encode("utf-8") if isinstance(s, str) else None for s in special_tokens]
        if any(s is None for s in sp):
            raise TypeError("argument 'special_tokens': 'list' items must be str")
        self._special_tokens = list(special_tokens)
        off = np.zeros(len(sp) + 1, dtype=np.uint64)
        np.cumsum([len(s) for s in sp], out=off[1:])
        blob = b"".join(sp)
        cfg = _n.TrainerConfig(vocab_size=vocab_size, min_frequency=min_frequency, min_word_length=min_word_length,
                               inl_alpha=inl_alpha, inl_beta=inl_beta, inl_gate=inl_gate, inl_mu_target=0.01,
                               inl_velocity_max=10.0, inl_beta_max=2.0, special=blob,
                               special_off=off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n_special=len(sp),
                               device=device)
        h = ctypes.c_void_p()
        rc = _n.lib.ctok_trainer_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc:
            _raise(rc)
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            _n.lib.ctok_trainer_destroy(h)
            self._h = None

    def _count(self, texts, into_acc):
        from . import pack_texts
        buf, off = pack_texts(texts)
        rc = _n.lib.ctok_trainer_count(self._h, buf.ctypes.data, off.ctypes.data, len(off) - 1, 1 if into_acc else 0)
        if rc:
            _raise(rc)

    def _train(self, from_acc):
        rc = _n.lib.ctok_trainer_train(self._h, 1 if from_acc else 0)
        if rc:
            _raise(rc)

    def train(self, files, block_bytes: int = 64 << 20):
        """Train on text files, one text per line (src/trainer.rs:187-193, count_words :265-285).
        Files are read and counted in blocks of about `block_bytes`; on an unreadable file or a
        line that is not UTF-8 the counts made so far are dropped and IOError is raised, as the
        reference returns the error before anything is trained."""
        if isinstance(files, (str, bytes)):
            raise TypeError("Can't extract `str` to `Vec`")
        try:
            for p in list(files):
                for lines in _file_line_blocks(p, block_bytes):
                    self._count(lines, False)
        except BaseException:
            _n.lib.ctok_trainer_clear_counts(self._h, 0)
            raise
        self._train(False)

    def train_from_iterator(self, texts):
        """src/trainer.rs:195-204 (count_words_from_iter_bytelevel, then train_from_word_freqs)."""
        self._count(texts, False)
        self._train(False)

    def count_batch(self, texts):
        """src/trainer.rs:207-220: add the texts' words to the accumulator."""
        self._count(texts, True)

    def finish_training(self):
        """src/trainer.rs:223-229: train on the accumulated counts."""
        self._train(True)

    def train_from_word_freqs(self, word_freqs):
        """train_from_word_freqs (src/trainer.rs:231-243) on a {raw-bytes word: freq} dict (the words as
        pre-tokenized pieces before the byte-to-char map); extension for callers that count words
        themselves."""
        words = [bytes(w) for w in word_freqs]
        freqs = np.asarray([int(word_freqs[w]) for w in word_freqs], dtype=np.uint32)
        off = np.zeros(len(words) + 1, dtype=np.uint64)
        np.cumsum([len(w) for w in words], out=off[1:])
        blob = np.frombuffer(b"".join(words) + b"\0", dtype=np.uint8)
        rc = _n.lib.ctok_trainer_train_words(self._h, blob.ctypes.data, off.ctypes.data, freqs.ctypes.data, len(words))
        if rc:
            _raise(rc)

    def to_str(self) -> str:
        """The tokenizer.json `save` writes (src/trainer.rs:600-645)."""
        n = ctypes.c_size_t()
        rc = _n.lib.ctok_trainer_json(self._h, None, 0, ctypes.byref(n))
        if rc:
            _raise(rc)
        buf = ctypes.create_string_buffer(n.value)
        rc = _n.lib.ctok_trainer_json(self._h, buf, n.value, ctypes.byref(n))
        if rc:
            _raise(rc)
        return buf.raw[:n.value].decode("utf-8")

    def save(self, path):
        """src/bindings/trainers.rs:78-81 -> src/trainer.rs:600-645 (IOError on failure)."""
        if not isinstance(path, str):
            raise TypeError("argument 'path': '%s' object cannot be converted to 'PyString'" % type(path).__name__)
        rc = _n.lib.ctok_trainer_save(self._h, path.encode())
        if rc:
            _raise(rc)

    @property
    def vocab_size(self) -> int:
        return int(_n.lib.ctok_trainer_vocab_size(self._h))

    @property
    def num_merges(self) -> int:
        return int(_n.lib.ctok_trainer_num_merges(self._h))

    def initial_pairs(self):
        """(a, b, count) arrays of the last training's compute_initial_pairs, sorted by (a, b)."""
        n = ctypes.c_uint64()
        rc = _n.lib.ctok_trainer_initial_pairs(self._h, None, None, None, 0, ctypes.byref(n))
        if rc:
            _raise(rc)
        a = np.zeros(n.value, dtype=np.uint32)
        b = np.zeros(n.value, dtype=np.uint32)
        c = np.zeros(n.value, dtype=np.int64)
        rc = _n.lib.ctok_trainer_initial_pairs(self._h, a.ctypes.data, b.ctypes.data, c.ctypes.data, n.value,
                                               ctypes.byref(n))
        if rc:
            _raise(rc)
        return a, b, c

    def timing(self) -> dict:
        v = [ctypes.c_double() for _ in range(3)]
        rc = _n.lib.ctok_trainer_timing(self._h, *[ctypes.byref(x) for x in v])
        if rc:
            _raise(rc)
        return {"ms_pairs": v[0].value, "ms_merges": v[1].value, "ms_heap": v[2].value}
