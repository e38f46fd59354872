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
from . import _fast  # the Python-object edges of encode_batch (csrc/pyfast.c); built with libctok.so

__version__ = "0.3.3"
__all__ = ["Tokenizer", "Trainer", "Encoding", "BatchEncoding", "PanicException", "UnsupportedConfigError",
           "DeviceError", "__version__"]


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
    `Vec<String>` extraction: a bare str is refused and every element must be a str.  One C pass
    (complexity_tokenizer._fast.pack, csrc/pyfast.c); 16 bytes of padding keep the device-side
    16-byte loads inside the allocation."""
    buf, offs = _fast.pack(texts)
    return np.frombuffer(buf, dtype=np.uint8), np.frombuffer(offs, dtype=np.uint64)


def _as_str(t):
    if not isinstance(t, str):
        raise TypeError("'%s' object cannot be converted to 'PyString'" % type(t).__name__)
    return t


def _as_str_list(texts):
    if isinstance(texts, (str, bytes)):
        raise TypeError("Can't extract `str` to `Vec`")
    return [_as_str(t) for t in texts]


def _extract_str_list(v):
    """PyO3 `extract::<Vec<String>>()` as a test: a non-str sequence of str, else None."""
    if isinstance(v, (str, bytes)):
        return None
    try:
        items = list(v)
    except TypeError:
        return None
    return items if all(isinstance(x, str) for x in items) else None


def _split_pairs(pairs):
    a, b = [], []
    for p in pairs:
        x, y = p
        a.append(_as_str(x))
        b.append(_as_str(y))
    return a, b


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


_ID_CACHE: list = []


# threads filling the rows of _split_lists (the CPUs this process may use, at most 16)
_SPLIT_THREADS = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)))


def _split_lists(flat: np.ndarray, off: np.ndarray) -> list:
    """(flat uint32 ids, uint64 offsets[D+1]) -> D Python lists, built in C (csrc/pyfast.c) from a
    shared cache of the int objects 0 .. 2^17 - 1 (ids past it are created per use).  The cyclic
    garbage collector is paused while the lists are built: creating ~1e5 container objects
    otherwise triggers collections that rescan every list built so far."""
    global _ID_CACHE
    if not _ID_CACHE:
        _ID_CACHE = list(range(1 << 17))
    flat = np.ascontiguousarray(flat, dtype=np.uint32)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    was = gc.isenabled()
    gc.disable()
    try:
        return _fast.split(flat.ctypes.data, off.ctypes.data, len(off) - 1, _ID_CACHE, _SPLIT_THREADS)
    finally:
        if was:
            gc.enable()


from .encoding import BatchEncoding, Encoding  # noqa: E402
from .trainer import Trainer  # noqa: E402


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
        lib = getattr(_n, "lib", None) if _n is not None else None  # (None at interpreter teardown)
        if h is not None and h.value and lib is not None:
            lib.ctok_destroy(h)
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
    def from_tables(vocab: dict, merges, added_tokens=(), nfc: bool = True, add_prefix_space: bool = False) -> "Tokenizer":
        """Extension (ctok_create_from_tables): a ByteLevel BPE tokenizer from in-memory tables --
        vocab {byte-level token string: id}, merges as (left id, right id) in rank order,
        added_tokens as dicts with the tokenizer.json fields (id, content, special, single_word,
        lstrip, rstrip, normalized) -- through the same loader as from_file."""
        toks = [k.encode("utf-8") for k in vocab]
        voff = np.zeros(len(toks) + 1, dtype=np.uint64)
        np.cumsum([len(k) for k in toks], out=voff[1:])
        vid = np.asarray([int(vocab[k]) for k in vocab], dtype=np.uint32)
        ml = np.asarray([int(a) for a, _ in merges], dtype=np.uint32)
        mr = np.asarray([int(b) for _, b in merges], dtype=np.uint32)
        added_tokens = list(added_tokens)
        ab = [a["content"].encode("utf-8") for a in added_tokens]
        aoff = np.zeros(len(ab) + 1, dtype=np.uint64)
        np.cumsum([len(x) for x in ab], out=aoff[1:])
        aid = np.asarray([int(a["id"]) for a in added_tokens], dtype=np.uint32)
        bits = {"special": 1, "single_word": 2, "lstrip": 4, "rstrip": 8, "normalized": 16}
        afl = np.asarray([sum(v for k, v in bits.items() if a.get(k, False)) for a in added_tokens], dtype=np.uint8)
        vb, abl = b"".join(toks), b"".join(ab)
        ptr = lambda a: a.ctypes.data if len(a) else None  # noqa: E731
        tb = _n.Tables(vb, ptr(voff), ptr(vid), len(toks), ptr(ml), ptr(mr), len(ml), abl, ptr(aoff), ptr(aid), ptr(afl),
                       len(ab), 1 if nfc else 0, 1 if add_prefix_space else 0)
        h = ctypes.c_void_p()
        rc = _n.lib.ctok_create_from_tables(ctypes.byref(tb), ctypes.byref(h))
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

    def num_piece_added_tokens(self) -> int:
        """Extension (diagnostic): added tokens the GPU split runs on (include/ctok.h)."""
        return int(_n.lib.ctok_num_piece_added_tokens(self._h))

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

    # ------------------------------------------------------------------ padded encode / Encodings
    # __call__, encode_to_encoding, encode_batch_with_padding, ...
    # (src/bindings/tokenizer.rs:46-201, :256-371 -> src/huggingface/mod.rs:340-545).  The ids,
    # post-processor, truncation, padding and the three masks come from the GPU
    # (ctok_encode_padded); Encoding objects are assembled on the host from its rows.

    @property
    def model_max_length(self) -> int:
        return int(_n.lib.ctok_model_max_length(self._h))

    @property
    def padding_side(self) -> str:
        return "right"  # from_file / from_str (src/huggingface/mod.rs:325); setters are out of scope

    @property
    def is_fast(self) -> bool:
        return True

    def num_special_tokens_to_add(self, is_pair: bool = False) -> int:
        """src/bindings/tokenizer.rs:248-251 -> src/huggingface/mod.rs:915-932."""
        return int(_n.lib.ctok_num_special_tokens_to_add(self._h, 1 if is_pair else 0))

    def _pad_id_token(self):
        """(pad id, pad token) as chosen by the reference (src/huggingface/mod.rs:500-505)."""
        pid = int(_n.lib.ctok_pad_id(self._h))
        tok = self._tok_str(pid)
        return pid, (tok if tok is not None else "<pad>")

    def _tok_str(self, i):
        """Vocab::get_token (model.vocab only), cached per id."""
        cache = self.__dict__.setdefault("_tok_cache", {})
        if i not in cache:
            cache[i] = self.id_to_token(i)
        return cache[i]

    def get_special_tokens_mask(self, ids, already_has_special_tokens: bool = True) -> list:
        """src/bindings/tokenizer.rs:243-246 -> src/huggingface/mod.rs:899-913."""
        if not already_has_special_tokens:
            return [0] * len(ids)
        sp = self.special_tokens
        return [1 if (self._tok_str(int(i)) is not None and self._tok_str(int(i)) in sp) else 0 for i in ids]

    def encode_padded(self, texts, pairs=None, *, add_special_tokens: bool = True, truncation: bool = False,
                      max_length: int | None = None, padding: str | None = None, pad_left: bool = False,
                      pad_id: int | None = None, timing: bool = False, no_postprocess: bool = False) -> dict:
        """Extension: the batch as [rows, width] uint32 arrays straight from the GPU --
        input_ids, attention_mask, token_type_ids, special_tokens_mask, plus row_len (content +
        padding).  padding: None, "longest" or "max_length"; pairs: a list of second texts (row r
        = texts[r] + pairs[r]).  Semantics as encode_batch_with_padding / __call__ (include/ctok.h,
        CTOK_P_*), without overflowing windows."""
        if pairs is not None:
            if len(pairs) != len(texts):
                raise ValueError("pairs must have one entry per text")
            docs = [x for ab in zip(texts, pairs) for x in ab]
        else:
            docs = list(texts)
        text, off = pack_texts(docs)
        rows = len(texts)
        f = 0
        if add_special_tokens:
            f |= _n.CTOK_P_ADD_SPECIAL
        if pairs is not None:
            f |= _n.CTOK_P_PAIRS
        if truncation:
            f |= _n.CTOK_P_TRUNCATE
        if padding == "longest":
            f |= _n.CTOK_P_PAD_LONGEST
        elif padding == "max_length":
            f |= _n.CTOK_P_PAD_TO_MAX
        elif padding is not None:
            raise ValueError("padding must be None, 'longest' or 'max_length'")
        if pad_left:
            f |= _n.CTOK_P_PAD_LEFT
        if pad_id is not None:
            f |= _n.CTOK_P_PAD_ID
        if no_postprocess:
            f |= _n.CTOK_P_NO_POSTPROCESS
        ml = int(max_length) if max_length is not None else self.model_max_length
        opts = _n.PadOpts(f, int(pad_id or 0), ml)
        # first guess of the width: ids <= bytes unless NFC grows the text (then the call reports
        # the width it needs and runs again)
        lens = np.diff(off.astype(np.int64))
        if pairs is not None:
            lens = lens.reshape(-1, 2).sum(axis=1) if rows else lens[:0]
        items = self._pp_items() if (add_special_tokens and not no_postprocess) else None
        n_a = items.count(_n.CTOK_PP_SEQUENCE) if items is not None else 1
        n_s = len(items) - n_a if items is not None else 0
        width = (int(lens.max()) * max(n_a, 1) + n_s + 1) if rows else 0
        if truncation:
            width = min(width, ml)
        if padding == "max_length":
            width = max(width, ml)
        while True:
            cap = max(rows * width, 1)
            arrs = [np.empty(cap, dtype=np.uint32) for _ in range(4)]
            row_len = np.empty(max(rows, 1), dtype=np.uint64)
            wout = ctypes.c_uint64()
            st = _n.Stats()
            ex = _n.Exec(self.device, None, _n.CTOK_F_TIMING if timing else 0)
            rc = _n.lib.ctok_encode_padded(self._h, text.ctypes.data, off.ctypes.data, len(docs), ctypes.byref(opts),
                                           arrs[0].ctypes.data, arrs[1].ctypes.data, arrs[2].ctypes.data,
                                           arrs[3].ctypes.data, cap, row_len.ctypes.data, ctypes.byref(wout),
                                           ctypes.byref(ex), ctypes.byref(st))
            if rc == _n.CTOK_E_CAPACITY and int(wout.value) > width:
                width = int(wout.value)
                continue
            if rc != _n.CTOK_OK:
                _raise(rc)
            break
        self.last_stats = st.as_dict()
        w = int(wout.value)
        shape = (rows, w)
        out = {k: a[: rows * w].reshape(shape) for k, a in
               zip(("input_ids", "attention_mask", "token_type_ids", "special_tokens_mask"), arrs)}
        out["row_len"] = row_len[:rows].astype(np.int64)
        return out

    def encode_offsets(self, texts):
        """Per text: (ids, offsets, word_ids) of encode_single_to_encoding
        (src/huggingface/mod.rs:395-480) -- ids from the GPU encode without the added-token
        split, each token's approximate (start, end) byte range in its text and its word index,
        placed by the C ABI's host walk (ctok_encode_offsets).  Raises PanicException where the
        reference's text slicing panics."""
        docs = _as_str_list(texts)
        text, off = pack_texts(docs)
        n = len(docs)
        cap = max(int(off[-1]) + n, 1)
        while True:
            ids = np.empty(cap, dtype=np.uint32)
            offs = np.empty(2 * cap, dtype=np.uint64)
            wids = np.empty(cap, dtype=np.uint32)
            tok_off = np.empty(n + 1, dtype=np.uint64)
            ex = _n.Exec(self.device, None, 0)
            rc = _n.lib.ctok_encode_offsets(self._h, text.ctypes.data, off.ctypes.data, n, ids.ctypes.data,
                                            offs.ctypes.data, wids.ctypes.data, cap, tok_off.ctypes.data,
                                            ctypes.byref(ex))
            if rc == _n.CTOK_E_CAPACITY and int(tok_off[n]) > cap:
                cap = int(tok_off[n])
                continue
            if rc != _n.CTOK_OK:
                _raise(rc)
            break
        pairs = offs[: 2 * int(tok_off[n])].reshape(-1, 2).tolist()
        res = []
        for d in range(n):
            a, b = int(tok_off[d]), int(tok_off[d + 1])
            res.append((ids[a:b].tolist(), [tuple(x) for x in pairs[a:b]], wids[a:b].tolist()))
        return res

    def _pp_items(self):
        """The post-processor as items (CTOK_PP_SEQUENCE = the ids), None without one."""
        n = ctypes.c_int64()
        buf = (ctypes.c_uint32 * 64)()
        rc = _n.lib.ctok_post_processor(self._h, buf, 64, ctypes.byref(n))
        if rc != _n.CTOK_OK:
            _raise(rc)
        return None if n.value < 0 else list(buf[: n.value])

    def _to_encodings(self, texts, pairs=None, add_special_tokens=True) -> list:
        """Encodings before truncation / padding, from one GPU call (rows unpadded):
        add_special_tokens -> encode_to_encoding / encode_pair_to_encoding
        (src/huggingface/mod.rs:340-392), else Encoding::from_ids over encode() (+ merge for a
        pair, src/bindings/tokenizer.rs:64-97)."""
        r = self.encode_padded(texts, pairs, add_special_tokens=add_special_tokens)
        items = self._pp_items() if add_special_tokens else None
        seq = _n.CTOK_PP_SEQUENCE
        orig_rows = None
        if items is not None and seq not in items:  # the ids are not in the rows: fetch them apart
            orig_rows = self.encode_padded(texts, pairs, add_special_tokens=True, no_postprocess=True)
        n_a = items.count(seq) if items is not None else 0
        n_s = len(items) - n_a if items is not None else 0
        first_a = items.index(seq) if (items is not None and n_a) else 0
        ids2d, att, typ, spc, rl = (r["input_ids"], r["attention_mask"], r["token_type_ids"],
                                    r["special_tokens_mask"], r["row_len"])
        offs_a = offs_b = None
        if add_special_tokens:  # offsets / word ids of encode_single_to_encoding, per sequence
            offs_a = self.encode_offsets(texts)
            offs_b = self.encode_offsets(pairs) if pairs is not None else None
        encs = []
        was = gc.isenabled()
        gc.disable()
        try:
            for i in range(len(texts)):
                L = int(rl[i])
                ids = ids2d[i, :L].tolist()
                types = typ[i, :L].tolist()
                if add_special_tokens:
                    if items is None:
                        n, orig = L, ids
                    elif n_a:
                        n = (L - n_s) // n_a
                        orig = ids[first_a: first_a + n]
                    else:
                        n = int(orig_rows["row_len"][i])
                        orig = orig_rows["input_ids"][i, :n].tolist()
                    # one token string per original id, "" outside model.vocab (mod.rs:410); the
                    # post-processor adds no tokens (mod.rs:378-386)
                    toks = [(self._tok_str(t) or "") for t in orig]
                    na = types[:n].count(0)
                    # offsets / word ids: the sequences' own, merged (encoding.rs:240-255); the
                    # post-processor does not extend them (mod.rs:378-386)
                    offs, wids = list(offs_a[i][1]), list(offs_a[i][2])
                    if offs_b is not None:
                        offs += offs_b[i][1]
                        wids += offs_b[i][2]
                    if len(offs) != n:
                        raise RuntimeError("offsets: %d tokens for %d ids" % (len(offs), n))
                    encs.append(Encoding(ids, types, toks, att[i, :L].tolist(), spc[i, :L].tolist(), offs, wids,
                                         [0] * na + [1] * (n - na)))
                else:
                    toks = [t for t in (self._tok_str(x) for x in ids) if t is not None]
                    na = types.count(0)
                    encs.append(Encoding(ids, types, toks, att[i, :L].tolist(), spc[i, :L].tolist(), [], [],
                                         [0] * na + [1] * (L - na)))
        finally:
            if was:
                gc.enable()
        return encs

    def encode_to_encoding(self, text: str) -> Encoding:
        """src/bindings/tokenizer.rs:298-300 -> src/huggingface/mod.rs:340-342."""
        return self._to_encodings([_as_str(text)])[0]

    def encode_plus(self, text: str) -> Encoding:
        """src/bindings/tokenizer.rs:258-260."""
        return self.encode_to_encoding(text)

    def encode_pair_to_encoding(self, text: str, text_pair: str) -> Encoding:
        """src/bindings/tokenizer.rs:302-304 -> src/huggingface/mod.rs:344-346."""
        return self._to_encodings([_as_str(text)], [_as_str(text_pair)])[0]

    def encode_with_truncation(self, text: str, text_pair: str | None = None, max_length: int = 512,
                               stride: int = 0) -> Encoding:
        """src/bindings/tokenizer.rs:306-318 -> src/huggingface/mod.rs:348-392: truncation
        with stride (0 = plain windows) when longer than max_length."""
        enc = (self.encode_pair_to_encoding(text, text_pair) if text_pair is not None
               else self.encode_to_encoding(text))
        if len(enc) > max_length:
            enc.truncate_with_stride(max_length, stride)
        return enc

    def encode_batch_to_encoding(self, texts) -> list:
        """src/bindings/tokenizer.rs:320-326 -> src/huggingface/mod.rs:483-485."""
        return self._to_encodings(_as_str_list(texts))

    def batch_encode_plus(self, texts) -> list:
        """src/bindings/tokenizer.rs:262-269."""
        return self.encode_batch_to_encoding(texts)

    def encode_batch_pairs_to_encoding(self, pairs) -> list:
        """src/bindings/tokenizer.rs:328-336 -> src/huggingface/mod.rs:487-491."""
        a, b = _split_pairs(pairs)
        return self._to_encodings(a, b)

    def _pad_all(self, encs, max_length, pad_left):
        target = max_length if max_length is not None else max((len(e) for e in encs), default=0)
        pid, ptok = self._pad_id_token()
        for e in encs:
            e.pad(target, pid, ptok, pad_left)
        return encs

    def encode_batch_with_padding(self, texts, max_length: int | None = None, pad_left: bool = False) -> list:
        """src/bindings/tokenizer.rs:338-350 -> src/huggingface/mod.rs:493-517 (no truncation:
        a row longer than max_length stays longer)."""
        return self._pad_all(self.encode_batch_to_encoding(texts), max_length, pad_left)

    def encode_batch_pairs_with_padding(self, pairs, max_length: int | None = None, pad_left: bool = False) -> list:
        """src/bindings/tokenizer.rs:352-367 -> src/huggingface/mod.rs:519-543."""
        return self._pad_all(self.encode_batch_pairs_to_encoding(pairs), max_length, pad_left)

    def __call__(self, text, text_pair=None, add_special_tokens: bool = True, padding: str | None = None,
                 truncation: bool = False, max_length: int | None = None, stride: int = 0,
                 return_attention_mask: bool = True, return_token_type_ids: bool = True,
                 return_offsets_mapping: bool = False, return_special_tokens_mask: bool = False) -> BatchEncoding:
        """src/bindings/tokenizer.rs:33-201."""
        flags = (return_attention_mask, return_token_type_ids, return_offsets_mapping, return_special_tokens_mask)
        max_len = max_length if max_length is not None else self.model_max_length
        batch = _extract_str_list(text)
        if batch is not None:
            pairs = _extract_str_list(text_pair) if text_pair is not None else None
            if pairs is not None:
                m = min(len(batch), len(pairs))  # Iterator::zip
                encs = self._to_encodings(batch[:m], pairs[:m], add_special_tokens)
            else:
                encs = self._to_encodings(batch, None, add_special_tokens)
            longest = max((len(e) for e in encs), default=0)
        elif isinstance(text, str):
            pair = text_pair if isinstance(text_pair, str) else None
            encs = self._to_encodings([text], [pair] if pair is not None else None, add_special_tokens)
            longest = len(encs[0])
        else:
            raise TypeError("Expected str or List[str]")
        if truncation:
            for e in encs:
                if len(e) > max_len:
                    if stride > 0:
                        e.truncate_with_stride(max_len, stride)
                    else:
                        e.truncate(max_len)
            if batch is None:
                longest = len(encs[0])
        if padding is not None:
            if batch is not None:
                target = max_len if padding == "max_length" else max((len(e) for e in encs), default=0)
            else:
                target = max_len if padding == "max_length" else len(encs[0])
            pid, ptok = self._pad_id_token()
            left = padding == "left" or self.padding_side == "left"
            for e in encs:
                e.pad(target, pid, ptok, left)
        del longest
        return BatchEncoding(encs, *flags)

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
