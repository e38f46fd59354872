"""complexity_tokenizer -- MI355X-native batch ByteLevel-BPE encode path.

Drop-in for the encode surface of Complexity-ML/complexity-tokenizer's `Tokenizer`
(python/complexity_tokenizer/__init__.py:16-18 re-exporting the PyO3 class of
src/bindings/tokenizer.rs:11-14): `from_file`, `from_pretrained`, `encode`, `encode_batch`,
`vocab_size`, `token_to_id`, `id_to_token`, `special_tokens`.  The work runs in hand-written
HIP kernels on an MI355X (gfx950) behind the C ABI of include/ctok.h; there is no CPU path.

Example:
    >>> from complexity_tokenizer import Tokenizer
    >>> tok = Tokenizer.from_file("tokenizer.json")
    >>> tok.encode_batch(["Hello world!", "second doc"])
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _native as _n

__version__ = "0.3.3"
__all__ = ["Tokenizer", "PanicException", "UnsupportedConfigError", "DeviceError", "__version__"]


class PanicException(BaseException):
    """Raised where the reference raises pyo3_runtime.PanicException (a Rust panic), e.g. a
    merge rank that indexes past the list of valid merges (reference src/bpe.rs:141)."""


class UnsupportedConfigError(NotImplementedError):
    """tokenizer.json selects a component outside the ByteLevel-BPE encode path."""


class DeviceError(RuntimeError):
    """HIP runtime failure, or no MI355X visible (the encode path has no CPU fallback)."""


def _raise(code: int, what: str = ""):
    msg = _n.last_error() or what
    if code in (_n.CTOK_E_IO, _n.CTOK_E_PARSE):
        raise IOError(msg)
    if code == _n.CTOK_E_UNSUPPORTED:
        raise UnsupportedConfigError(msg)
    if code == _n.CTOK_E_PANIC:
        raise PanicException(msg)
    if code == _n.CTOK_E_DEVICE:
        raise DeviceError(msg)
    if code == _n.CTOK_E_ARG:
        raise ValueError(msg)
    raise RuntimeError("ctok error %d: %s" % (code, msg))


def _hub_cache_dir() -> str:
    """dirs::cache_dir()/huggingface/hub (reference src/hub.rs:22-35) on Linux."""
    base = os.environ.get("XDG_CACHE_HOME") or os.path.join(os.path.expanduser("~"), ".cache")
    return os.path.join(base, "huggingface", "hub")


def pack_texts(texts) -> tuple[np.ndarray, np.ndarray]:
    """list[str] -> (utf-8 bytes as uint8 array, uint64 offsets[D+1]).  Mirrors the PyO3
    `Vec<String>` extraction: a bare str is refused and every element must be a str."""
    if isinstance(texts, (str, bytes)):
        raise TypeError("Can't extract `str` to `Vec`")
    enc = []
    for t in texts:
        if not isinstance(t, str):
            raise TypeError("'%s' object cannot be converted to 'PyString'" % type(t).__name__)
        enc.append(t.encode("utf-8"))
    lens = np.fromiter((len(e) for e in enc), dtype=np.uint64, count=len(enc))
    off = np.zeros(len(enc) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    # 16 bytes of padding keep the device-side 16-byte loads inside the allocation
    buf = np.frombuffer(b"".join(enc) + b"\0" * 16, dtype=np.uint8)
    return buf, off


class Tokenizer:
    """HuggingFace-format ByteLevel-BPE tokenizer whose encode path runs on an MI355X."""

    def __init__(self, handle):
        self._h = ctypes.c_void_p(handle)
        self.device = int(os.environ.get("CTOK_DEVICE", "0"))
        self.last_stats = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _n.lib.ctok_destroy(h)
            self._h = None

    # ------------------------------------------------------------------ constructors
    @staticmethod
    def from_file(path: str) -> "Tokenizer":
        """src/bindings/tokenizer.rs:18-23 -> src/huggingface/mod.rs:159-166."""
        h = ctypes.c_void_p()
        rc = _n.lib.ctok_create_from_file(os.fsencode(path), ctypes.byref(h))
        if rc != _n.CTOK_OK:
            _raise(rc)
        return Tokenizer(h.value)

    @staticmethod
    def from_str(json_text: str) -> "Tokenizer":
        """HuggingFaceTokenizer::from_str (src/huggingface/mod.rs:168-173)."""
        b = json_text.encode("utf-8")
        h = ctypes.c_void_p()
        rc = _n.lib.ctok_create_from_buffer(b, len(b), ctypes.byref(h))
        if rc != _n.CTOK_OK:
            _raise(rc)
        return Tokenizer(h.value)

    @staticmethod
    def from_pretrained(repo_id: str, revision: str | None = None, local_files_only: bool = False) -> "Tokenizer":
        """src/bindings/tokenizer.rs:25-31 -> src/huggingface/mod.rs:188-241.  With
        local_files_only the reference reads <cache>/huggingface/hub/<org--name>/tokenizer.json;
        otherwise it downloads from the Hub, which needs a network this build never uses."""
        if local_files_only:
            path = os.path.join(_hub_cache_dir(), repo_id.replace("/", "--"), "tokenizer.json")
            if os.path.exists(path):
                return Tokenizer.from_file(path)
            raise IOError("Model '%s' not found in cache and local_files_only=true" % repo_id)
        raise IOError("https://huggingface.co/%s/resolve/%s/tokenizer.json: network access is not available; "
                      "use local_files_only=True or from_file()" % (repo_id, revision or "main"))

    # ------------------------------------------------------------------ getters
    @property
    def vocab_size(self) -> int:
        return int(_n.lib.ctok_vocab_size(self._h))

    def token_to_id(self, token: str):
        b = token.encode("utf-8")
        out = ctypes.c_uint32()
        rc = _n.lib.ctok_token_to_id(self._h, b, len(b), ctypes.byref(out))
        if rc == _n.CTOK_E_NOTFOUND:
            return None
        if rc != _n.CTOK_OK:
            _raise(rc)
        return int(out.value)

    def id_to_token(self, id: int):
        n = ctypes.c_size_t()
        buf = ctypes.create_string_buffer(256)
        rc = _n.lib.ctok_id_to_token(self._h, int(id), buf, 256, ctypes.byref(n))
        if rc == _n.CTOK_E_NOTFOUND:
            return None
        if rc != _n.CTOK_OK:
            _raise(rc)
        if n.value > 256:
            buf = ctypes.create_string_buffer(n.value)
            _n.lib.ctok_id_to_token(self._h, int(id), buf, n.value, ctypes.byref(n))
        return buf.raw[:n.value].decode("utf-8")

    @property
    def special_tokens(self) -> dict:
        out = {}
        for i in range(int(_n.lib.ctok_num_special_tokens(self._h))):
            n = ctypes.c_size_t()
            tid = ctypes.c_uint32()
            buf = ctypes.create_string_buffer(1024)
            rc = _n.lib.ctok_special_token(self._h, i, buf, 1024, ctypes.byref(n), ctypes.byref(tid))
            if rc != _n.CTOK_OK:
                _raise(rc)
            if n.value > 1024:
                buf = ctypes.create_string_buffer(n.value)
                _n.lib.ctok_special_token(self._h, i, buf, n.value, ctypes.byref(n), ctypes.byref(tid))
            out[buf.raw[:n.value].decode("utf-8")] = int(tid.value)
        return out

    # ------------------------------------------------------------------ encode
    def encode_packed(self, text: np.ndarray, off: np.ndarray, timing: bool = False):
        """Extension: encode a packed batch (uint8 UTF-8 buffer, uint64 offsets[D+1]) and return
        (ids uint32[T], tok_off uint64[D+1]) without building Python lists."""
        text = np.ascontiguousarray(text, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        n_docs = len(off) - 1
        if n_docs < 0:
            raise ValueError("offsets must hold n_docs + 1 entries")
        n_bytes = int(off[-1]) if n_docs >= 0 else 0
        if len(text) < n_bytes:
            raise ValueError("text shorter than offsets[-1]")
        cap = int(n_bytes + n_docs + 16)
        while True:
            ids = np.empty(max(cap, 1), dtype=np.uint32)
            tok_off = np.empty(n_docs + 1, dtype=np.uint64)
            ex = _n.Exec(self.device, None, _n.CTOK_F_TIMING if timing else 0)
            st = _n.Stats()
            rc = _n.lib.ctok_encode_batch(self._h, text.ctypes.data, off.ctypes.data, n_docs, ids.ctypes.data, cap,
                                          tok_off.ctypes.data, ctypes.byref(ex), ctypes.byref(st))
            if rc == _n.CTOK_E_CAPACITY:
                cap = int(tok_off[-1])
                continue
            if rc != _n.CTOK_OK:
                _raise(rc)
            self.last_stats = st.as_dict()
            return ids[: int(tok_off[-1])], tok_off

    def encode_packed_device(self, d_text: int, d_off: int, n_docs: int, n_bytes: int, d_ids: int, ids_cap: int,
                             d_tok_off: int, stream: int = 0, timing: bool = False, device: int | None = None):
        """Extension: encode a batch already resident in HBM (raw device pointers, e.g. from
        torch tensors' data_ptr()).  Work is ordered on `stream` (a hipStream_t as int, 0 = the
        library's own stream).  Returns the total number of ids written; stats in last_stats."""
        ex = _n.Exec(self.device if device is None else device, stream or None, _n.CTOK_F_TIMING if timing else 0)
        st = _n.Stats()
        ntok = ctypes.c_uint64()
        rc = _n.lib.ctok_encode_batch_device(self._h, d_text, d_off, n_docs, n_bytes, d_ids, ids_cap, d_tok_off,
                                             ctypes.byref(ntok), ctypes.byref(ex), ctypes.byref(st))
        if rc != _n.CTOK_OK:
            _raise(rc)
        self.last_stats = st.as_dict()
        return int(ntok.value)

    def encode_batch_flat(self, texts):
        """Extension: list[str] -> (ids uint32[T], tok_off uint64[D+1])."""
        text, off = pack_texts(texts)
        return self.encode_packed(text, off)

    def encode_batch(self, texts) -> list:
        """src/bindings/tokenizer.rs:207-210 -> src/huggingface/mod.rs:694-696."""
        ids, tok_off = self.encode_batch_flat(texts)
        flat = ids.tolist()
        o = tok_off.tolist()
        return [flat[o[i]:o[i + 1]] for i in range(len(o) - 1)]

    def encode(self, text: str) -> list:
        """src/bindings/tokenizer.rs:203-205 -> src/huggingface/mod.rs:551-613."""
        if not isinstance(text, str):
            raise TypeError("'%s' object cannot be converted to 'PyString'" % type(text).__name__)
        return self.encode_batch([text])[0]

    def __repr__(self):
        return "Tokenizer(vocab_size=%d, device=%d)" % (self.vocab_size, self.device)


def device_count() -> int:
    return int(_n.lib.ctok_device_count())
