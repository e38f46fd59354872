"""complexity_tokenizer -- MI355X-native batch ByteLevel-BPE encode path.

Drop-in for the encode / decode surface of Complexity-ML/complexity-tokenizer's `Tokenizer`
(python/complexity_tokenizer/__init__.py:16-18 re-exporting the PyO3 class of
src/bindings/tokenizer.rs:11-14): `from_file`, `from_pretrained`, `encode`, `encode_batch`,
`decode`, `decode_with_options`, `decode_batch`, `decode_batch_with_options`, `batch_decode`,
`vocab_size`, `token_to_id`, `id_to_token`, `special_tokens`.  The work runs in hand-written
HIP kernels on an MI355X (gfx950) behind the C ABI of include/ctok.h; there is no CPU path.

Example:
    >>> from complexity_tokenizer import Tokenizer
    >>> tok = Tokenizer.from_file("tokenizer.json")
    >>> tok.encode_batch(["Hello world!", "second doc"])
"""
from __future__ import annotations

import ctypes
import gc
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


def pack_ids(batch) -> tuple[np.ndarray, np.ndarray]:
    """list[list[int]] -> (uint32 ids, uint64 offsets[D+1]).  Mirrors the PyO3 `Vec<Vec<u32>>`
    extraction: a bare str is refused, elements must be ints in [0, 2**32)."""
    if isinstance(batch, (str, bytes)):
        raise TypeError("Can't extract `str` to `Vec`")
    lens = []
    flat = []
    for seq in batch:
        if isinstance(seq, (str, bytes)):
            raise TypeError("Can't extract `str` to `Vec`")
        seq = list(seq)
        for x in seq:
            if not isinstance(x, (int, np.integer)):
                raise TypeError("'%s' object cannot be interpreted as an integer" % type(x).__name__)
            if x < 0 or x > 0xFFFFFFFF:
                raise OverflowError("can't convert %d to u32" % x)
        lens.append(len(seq))
        flat.extend(seq)
    off = np.zeros(len(lens) + 1, dtype=np.uint64)
    np.cumsum(np.asarray(lens, dtype=np.uint64), out=off[1:])
    return np.asarray(flat, dtype=np.uint64).astype(np.uint32), off


def _split_lists(flat: np.ndarray, off: np.ndarray) -> list:
    """(flat uint array, offsets[D+1]) -> D Python lists.  The cyclic garbage collector is paused
    while the lists are built: creating ~1e5 container objects otherwise triggers collections
    that rescan every list built so far (3x the cost of the conversion itself)."""
    was = gc.isenabled()
    gc.disable()
    try:
        f = flat.tolist()
        o = off.tolist()
        return [f[o[i]:o[i + 1]] for i in range(len(o) - 1)]
    finally:
        if was:
            gc.enable()


class Tokenizer:
    """HuggingFace-format ByteLevel-BPE tokenizer whose encode path runs on an MI355X."""

    def __init__(self, handle):
        self._h = ctypes.c_void_p(handle)
        self.device = int(os.environ.get("CTOK_DEVICE", "0"))
        # host-buffer encode over several GPUs of this process (byte-balanced doc shards, one
        # host thread per device): e.g. tok.devices = list(range(device_count()))
        env = os.environ.get("CTOK_DEVICES", "")
        self.devices = [int(x) for x in env.split(",") if x.strip()] or None
        self.chunk_mb = 0  # pipeline chunk of the host-buffer path (0 = library default)
        self.last_stats = None
        self.last_decode_stats = None

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
            ex = self._host_exec(timing)
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

    def _host_exec(self, timing: bool):
        ex = _n.Exec(self.device, None, _n.CTOK_F_TIMING if timing else 0)
        if self.devices:
            arr = (ctypes.c_int * len(self.devices))(*[int(d) for d in self.devices])
            ex.devices = ctypes.cast(arr, ctypes.POINTER(ctypes.c_int))
            ex.n_devices = len(self.devices)
            ex._keep = arr  # keeps the array alive as long as the struct
        ex.chunk_mb = int(self.chunk_mb)
        return ex

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
        return _split_lists(ids, tok_off)

    def encode(self, text: str) -> list:
        """src/bindings/tokenizer.rs:203-205 -> src/huggingface/mod.rs:551-613."""
        if not isinstance(text, str):
            raise TypeError("'%s' object cannot be converted to 'PyString'" % type(text).__name__)
        return self.encode_batch([text])[0]

    # ------------------------------------------------------------------ decode
    def decode_packed(self, ids: np.ndarray, tok_off: np.ndarray, skip_special_tokens: bool = False,
                      clean_up_tokenization_spaces: bool = True, timing: bool = False):
        """Extension: decode packed ids (uint32[T], uint64 offsets[D+1]) and return
        (utf-8 bytes uint8[N], out_off uint64[D+1]) without building Python strings."""
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        tok_off = np.ascontiguousarray(tok_off, dtype=np.uint64)
        n_docs = len(tok_off) - 1
        if n_docs < 0:
            raise ValueError("offsets must hold n_docs + 1 entries")
        if len(ids) < int(tok_off[-1]):
            raise ValueError("ids shorter than tok_off[-1]")
        opts = (_n.CTOK_D_SKIP_SPECIAL if skip_special_tokens else 0) | (
            _n.CTOK_D_CLEANUP if clean_up_tokenization_spaces else 0)
        cap = 4 * len(ids) + 64
        while True:
            out = np.empty(cap, dtype=np.uint8)
            out_off = np.empty(n_docs + 1, dtype=np.uint64)
            ex = _n.Exec(self.device, None, _n.CTOK_F_TIMING if timing else 0)
            st = _n.DecodeStats()
            rc = _n.lib.ctok_decode_batch(self._h, ids.ctypes.data if len(ids) else None, tok_off.ctypes.data, n_docs,
                                          opts, out.ctypes.data, cap, out_off.ctypes.data, ctypes.byref(ex),
                                          ctypes.byref(st))
            if rc == _n.CTOK_E_CAPACITY:
                cap = int(out_off[-1]) + 64
                continue
            if rc != _n.CTOK_OK:
                _raise(rc)
            self.last_decode_stats = st.as_dict()
            return out[: int(out_off[-1])], out_off

    def decode_packed_device(self, d_ids: int, d_tok_off: int, n_docs: int, n_ids: int, d_out: int, out_cap: int,
                             d_out_off: int, skip_special_tokens: bool = False,
                             clean_up_tokenization_spaces: bool = True, stream: int = 0, timing: bool = False,
                             device: int | None = None):
        """Extension: decode ids already resident in HBM (raw device pointers).  Returns the
        number of output bytes; raises ValueError when out_cap is smaller (the size is in the
        message and in last_decode_needed)."""
        opts = (_n.CTOK_D_SKIP_SPECIAL if skip_special_tokens else 0) | (
            _n.CTOK_D_CLEANUP if clean_up_tokenization_spaces else 0)
        ex = _n.Exec(self.device if device is None else device, stream or None, _n.CTOK_F_TIMING if timing else 0)
        st = _n.DecodeStats()
        nb = ctypes.c_uint64()
        rc = _n.lib.ctok_decode_batch_device(self._h, d_ids, d_tok_off, n_docs, n_ids, opts, d_out, out_cap, d_out_off,
                                             ctypes.byref(nb), ctypes.byref(ex), ctypes.byref(st))
        self.last_decode_needed = int(nb.value)
        if rc == _n.CTOK_E_CAPACITY:
            raise ValueError("out_cap too small: %d bytes needed" % nb.value)
        if rc != _n.CTOK_OK:
            _raise(rc)
        self.last_decode_stats = st.as_dict()
        return int(nb.value)

    def decode_batch_with_options(self, batch, skip_special_tokens: bool = False,
                                  clean_up_tokenization_spaces: bool = True) -> list:
        """src/bindings/tokenizer.rs:231-238 -> src/huggingface/mod.rs:777-785."""
        ids, off = pack_ids(batch)
        out, out_off = self.decode_packed(ids, off, skip_special_tokens, clean_up_tokenization_spaces)
        raw = out.tobytes()
        o = out_off.tolist()
        return [raw[o[i]:o[i + 1]].decode("utf-8") for i in range(len(o) - 1)]

    def decode_batch(self, batch) -> list:
        """src/bindings/tokenizer.rs:226-228 -> src/huggingface/mod.rs:771-773."""
        return self.decode_batch_with_options(batch, False, True)

    def batch_decode(self, sequences, skip_special_tokens: bool = False,
                     clean_up_tokenization_spaces: bool = True) -> list:
        """HF-compatible alias, src/bindings/tokenizer.rs:655-663."""
        return self.decode_batch_with_options(sequences, skip_special_tokens, clean_up_tokenization_spaces)

    def decode_with_options(self, ids, skip_special_tokens: bool = False,
                            clean_up_tokenization_spaces: bool = True) -> str:
        """src/bindings/tokenizer.rs:216-224 -> src/huggingface/mod.rs:702-709."""
        if isinstance(ids, (str, bytes)):
            raise TypeError("Can't extract `str` to `Vec`")
        return self.decode_batch_with_options([ids], skip_special_tokens, clean_up_tokenization_spaces)[0]

    def decode(self, ids) -> str:
        """src/bindings/tokenizer.rs:212-214 -> src/huggingface/mod.rs:698-700."""
        return self.decode_with_options(ids, False, True)

    def __repr__(self):
        return "Tokenizer(vocab_size=%d, device=%d)" % (self.vocab_size, self.device)


def device_count() -> int:
    return int(_n.lib.ctok_device_count())
