"""ctypes binding of libctok.so (the C ABI declared in include/ctok.h).

No CPU fallback: if the shared library is missing the import fails loudly, and encode calls on
a machine without a HIP device raise DeviceError.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CTOK_LIB", os.path.join(_HERE, "libctok.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        "complexity_tokenizer: native library not found at %s -- build it with "
        "`make -C complexity-tokenizer_amd/csrc` (or `python -c 'import __graft_entry__ as g; g.build()'`)" % LIB_PATH)

lib = ctypes.CDLL(LIB_PATH)

CTOK_OK = 0
CTOK_E_IO = -1
CTOK_E_PARSE = -2
CTOK_E_UNSUPPORTED = -3
CTOK_E_ARG = -4
CTOK_E_CAPACITY = -5
CTOK_E_PANIC = -6
CTOK_E_DEVICE = -7
CTOK_E_NOTFOUND = -8
CTOK_F_TIMING = 1


class Exec(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("stream", ctypes.c_void_p), ("flags", ctypes.c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [("ms_total", ctypes.c_double), ("ms_device", ctypes.c_double), ("ms_pretok", ctypes.c_double),
                ("ms_bpe_short", ctypes.c_double), ("ms_bpe_long", ctypes.c_double),
                ("ms_emit", ctypes.c_double), ("ms_h2d", ctypes.c_double),
                ("ms_d2h", ctypes.c_double), ("bytes_in", ctypes.c_uint64), ("bytes_norm", ctypes.c_uint64),
                ("docs", ctypes.c_uint64), ("pieces", ctypes.c_uint64), ("long_pieces", ctypes.c_uint64),
                ("tokens", ctypes.c_uint64), ("nfc_docs", ctypes.c_uint64), ("ms_segment", ctypes.c_double),
                ("ms_bpe_lo", ctypes.c_double), ("ms_bpe_hi", ctypes.c_double),
                ("class_bytes", ctypes.c_uint64 * 3), ("class_ids", ctypes.c_uint64 * 3)]

    def as_dict(self):
        d = {}
        for k, _ in self._fields_:
            v = getattr(self, k)
            d[k] = list(v) if isinstance(v, ctypes.Array) else v
        return d


_p = ctypes.c_void_p
_u64 = ctypes.c_uint64
_u64p = ctypes.POINTER(ctypes.c_uint64)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_sz = ctypes.c_size_t

SIGS = {
    "ctok_last_error": (ctypes.c_char_p, []),
    "ctok_version": (ctypes.c_char_p, []),
    "ctok_create_from_file": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(_p)]),
    "ctok_create_from_buffer": (ctypes.c_int, [ctypes.c_char_p, _sz, ctypes.POINTER(_p)]),
    "ctok_destroy": (None, [_p]),
    "ctok_vocab_size": (_u64, [_p]),
    "ctok_token_to_id": (ctypes.c_int, [_p, ctypes.c_char_p, _sz, _u32p]),
    "ctok_id_to_token": (ctypes.c_int, [_p, ctypes.c_uint32, ctypes.c_char_p, _sz, ctypes.POINTER(_sz)]),
    "ctok_num_special_tokens": (_u64, [_p]),
    "ctok_special_token": (ctypes.c_int, [_p, _u64, ctypes.c_char_p, _sz, ctypes.POINTER(_sz), _u32p]),
    "ctok_ids_bound": (_u64, [_p, _u64, _u64]),
    "ctok_encode_batch": (ctypes.c_int, [_p, _p, _p, _u64, _p, _u64, _p, ctypes.POINTER(Exec), ctypes.POINTER(Stats)]),
    "ctok_encode_batch_device": (ctypes.c_int, [_p, _p, _p, _u64, _u64, _p, _u64, _p, _u64p, ctypes.POINTER(Exec),
                                                ctypes.POINTER(Stats)]),
    "ctok_device_count": (ctypes.c_int, []),
}

for _name, (_res, _args) in SIGS.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args


def last_error() -> str:
    return lib.ctok_last_error().decode("utf-8", "replace")
