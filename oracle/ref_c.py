"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of the C oracle (oracle/ctok_ref.c).

Builds the reference tokenizer state from a tokenizer.json (parsed with Python's json module,
whose duplicate-key rule -- last wins -- matches the reference's HashMap) and encodes packed
batches on the host CPU with N threads.  Used by tests/ as a fast checker and by bench.py as
the `cpu_baseline` (kind "port": a faithful C restatement; the Rust reference cannot be built
in this image).
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess

import numpy as np

from . import ref_py

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libctok_ref.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        P = ctypes.c_void_p
        L.ref_create.restype = P
        L.ref_create.argtypes = [P, P, P, ctypes.c_int64, P, P, ctypes.c_int64, P, P, P, P, ctypes.c_int64,
                                 ctypes.c_int, ctypes.c_int]
        L.ref_destroy.argtypes = [P]
        L.ref_encode_batch.restype = ctypes.c_int
        L.ref_encode_batch.argtypes = [P, P, P, ctypes.c_int64, P, ctypes.c_uint64, P, ctypes.c_int]
        L.ref_nfc.restype = ctypes.c_int64
        L.ref_nfc.argtypes = [P, ctypes.c_uint64, P]
        L.ref_pieces.restype = ctypes.c_int64
        L.ref_pieces.argtypes = [P, ctypes.c_uint64, P]
        L.ref_dec_create.restype = P
        L.ref_dec_create.argtypes = [P, P, P, ctypes.c_uint64, P, P, ctypes.c_int64, ctypes.c_int]
        L.ref_dec_destroy.argtypes = [P]
        L.ref_decode_batch.restype = ctypes.c_int
        L.ref_decode_batch.argtypes = [P, P, P, ctypes.c_int64, ctypes.c_int, ctypes.c_int, P, ctypes.c_uint64, P,
                                       ctypes.c_int]
        _lib = L
    return _lib


def _strarr(items: list[bytes]):
    arr = (ctypes.c_char_p * max(1, len(items)))(*items)
    lens = np.array([len(x) for x in items] or [0], dtype=np.uint32)
    return arr, lens


class RefC:
    """The reference encode path as a faithful C port (cost model included)."""

    def __init__(self, obj: dict):
        py = ref_py.RefTokenizer(obj)  # same loader decisions (normaliser, pre-tokenizer, merges)
        self.py = py
        L = lib()
        vt = [k.encode("utf-8") for k in py.vocab]
        vid = np.array(list(py.vocab.values()) or [0], dtype=np.uint32)
        merges = [m.encode("utf-8") for m in ref_py.deserialize_merges(obj["model"].get("merges", []))]
        at = obj.get("added_tokens", [])
        ac = [a["content"].encode("utf-8") for a in at]
        aid = np.array([a["id"] for a in at] or [0], dtype=np.uint32)
        af = np.array([(1 if a.get("single_word") else 0) | (2 if a.get("lstrip") else 0) |
                       (4 if a.get("rstrip") else 0) for a in at] or [0], dtype=np.uint8)
        self._keep = []
        va, vl = _strarr(vt)
        ma, ml = _strarr(merges)
        aa, al = _strarr(ac)
        self._keep += [va, vl, vid, ma, ml, aa, al, aid, af]
        nfc = 1 if py.normalizer is not None else 0
        aps = 0
        pt = py.pre_tokenizer
        for p in (pt[1] if pt[0] == "Sequence" else [pt]):
            if p[0] == "ByteLevel":
                aps = 1 if p[1] else 0
        self.h = L.ref_create(ctypes.cast(va, ctypes.c_void_p), vl.ctypes.data, vid.ctypes.data, len(vt),
                              ctypes.cast(ma, ctypes.c_void_p), ml.ctypes.data, len(merges),
                              ctypes.cast(aa, ctypes.c_void_p), al.ctypes.data, aid.ctypes.data, af.ctypes.data,
                              len(ac), nfc, aps)

    @classmethod
    def from_file(cls, path):
        with open(path, "r", encoding="utf-8") as f:
            return cls(json.load(f))

    def __del__(self):
        if getattr(self, "h", None):
            lib().ref_destroy(self.h)
            self.h = None
        if getattr(self, "hd", None):
            lib().ref_dec_destroy(self.hd)
            self.hd = None

    def _decoder(self):
        """The decode-side state: Vocab::id_to_token (model.vocab only), the special added
        tokens by content, and the decoder kind (ByteLevel or raw concatenation)."""
        if getattr(self, "hd", None):
            return self.hd
        py = self.py
        if py.decoder[0] == "unsupported":
            raise ref_py.UnsupportedConfig("decoder " + py.decoder[1])
        n = max(py.id_to_token_map, default=-1) + 1
        toks = [py.id_to_token_map.get(i, "").encode("utf-8") for i in range(n)]
        has = np.array([1 if i in py.id_to_token_map else 0 for i in range(n)] or [0], dtype=np.uint8)
        ta, tl = _strarr(toks)
        sp = [k.encode("utf-8") for k in py.special_tokens]
        sa, sl = _strarr(sp)
        self._keep += [ta, tl, has, sa, sl]
        self.hd = lib().ref_dec_create(ctypes.cast(ta, ctypes.c_void_p), tl.ctypes.data, has.ctypes.data, n,
                                       ctypes.cast(sa, ctypes.c_void_p), sl.ctypes.data, len(sp),
                                       1 if py.decoder[0] == "ByteLevel" else 0)
        return self.hd

    def decode_packed(self, ids: np.ndarray, tok_off: np.ndarray, skip_special_tokens=False,
                      clean_up_tokenization_spaces=True, threads: int = 0):
        """decode_batch_with_options on packed ids -> (utf-8 bytes uint8[N], out_off uint64[D+1])."""
        hd = self._decoder()
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        tok_off = np.ascontiguousarray(tok_off, dtype=np.uint64)
        nd = len(tok_off) - 1
        threads = threads or os.cpu_count() or 1
        cap = 64
        while True:
            out = np.empty(cap, dtype=np.uint8)
            out_off = np.empty(nd + 1, dtype=np.uint64)
            rc = lib().ref_decode_batch(hd, ids.ctypes.data if len(ids) else None, tok_off.ctypes.data, nd,
                                        int(bool(skip_special_tokens)), int(bool(clean_up_tokenization_spaces)),
                                        out.ctypes.data, cap, out_off.ctypes.data, threads)
            if rc == -2:
                cap = int(out_off[-1]) + 64
                continue
            if rc != 0:
                raise RuntimeError("ref_decode_batch rc=%d" % rc)
            return out[: int(out_off[-1])].copy(), out_off

    def decode_batch(self, batch, skip_special_tokens=False, clean_up_tokenization_spaces=True, threads: int = 0):
        off = np.zeros(len(batch) + 1, dtype=np.uint64)
        np.cumsum([len(b) for b in batch], out=off[1:])
        ids = np.array([i for b in batch for i in b] or [0], dtype=np.uint32)
        out, out_off = self.decode_packed(ids, off, skip_special_tokens, clean_up_tokenization_spaces, threads)
        o = out_off.tolist()
        raw = out.tobytes()
        return [raw[o[k]:o[k + 1]].decode("utf-8") for k in range(len(batch))]

    def encode_packed(self, text: np.ndarray, off: np.ndarray, threads: int = 0):
        text = np.ascontiguousarray(text, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        nd = len(off) - 1
        threads = threads or os.cpu_count() or 1
        cap = int(off[-1]) * 3 + nd + 16
        ids = np.empty(max(cap, 1), dtype=np.uint32)
        tok_off = np.empty(nd + 1, dtype=np.uint64)
        rc = lib().ref_encode_batch(self.h, text.ctypes.data if len(text) else None, off.ctypes.data, nd,
                                    ids.ctypes.data, cap, tok_off.ctypes.data, threads)
        if rc == -3:
            raise ref_py.PanicException("reference panics (src/bpe.rs:141)")
        if rc != 0:
            raise RuntimeError("ref_encode_batch rc=%d" % rc)
        return ids[: int(tok_off[-1])].copy(), tok_off

    def encode_batch(self, texts: list[str], threads: int = 0):
        enc = [t.encode("utf-8") for t in texts]
        off = np.zeros(len(enc) + 1, dtype=np.uint64)
        np.cumsum([len(e) for e in enc], out=off[1:])
        text = np.frombuffer(b"".join(enc) + b"\0", dtype=np.uint8)
        ids, tok_off = self.encode_packed(text, off, threads)
        o = tok_off.tolist()
        f = ids.tolist()
        return [f[o[i]:o[i + 1]] for i in range(len(texts))]


def nfc_bytes(b: bytes) -> bytes:
    out = ctypes.create_string_buffer(3 * len(b) + 8)
    n = lib().ref_nfc(b, len(b), out)
    return out.raw[:n]


def pieces(b: bytes) -> list[bytes]:
    ends = np.zeros(len(b) + 2, dtype=np.uint64)
    k = lib().ref_pieces(b, len(b), ends.ctypes.data)
    out, s = [], 0
    for e in ends[:k].tolist():
        out.append(b[s:e])
        s = e
    return out
