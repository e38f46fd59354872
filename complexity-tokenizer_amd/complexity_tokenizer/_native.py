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


def _share_torch_hip_runtime():
    """torch wheels bundle their own HIP runtime with the same SONAME (libamdhip64.so.7) as
    /opt/rocm's.  Whichever copy loads first serves libctok.so; if /opt/rocm's came first and torch
    were imported later, torch would load its copy next to it and two HIP runtimes in one process
    fail to share the device.  Preloading torch's copy (without importing torch) makes every HIP
    user in the process resolve to one runtime.  CTOK_NO_TORCH_HIP=1 disables this."""
    if os.environ.get("CTOK_NO_TORCH_HIP"):
        return
    try:
        import importlib.util
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return
    if spec is None or not spec.origin:
        return
    path = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(path):
        ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


_share_torch_hip_runtime()
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
    _fields_ = [("device", ctypes.c_int), ("stream", ctypes.c_void_p), ("flags", ctypes.c_uint32),
                ("devices", ctypes.POINTER(ctypes.c_int)), ("n_devices", ctypes.c_int),
                ("chunk_mb", ctypes.c_uint32), ("host_threads", ctypes.c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [("ms_total", ctypes.c_double), ("ms_device", ctypes.c_double), ("ms_pretok", ctypes.c_double),
                ("ms_bpe_short", ctypes.c_double), ("ms_bpe_long", ctypes.c_double),
                ("ms_emit", ctypes.c_double), ("ms_h2d", ctypes.c_double),
                ("ms_d2h", ctypes.c_double), ("bytes_in", ctypes.c_uint64), ("bytes_norm", ctypes.c_uint64),
                ("docs", ctypes.c_uint64), ("pieces", ctypes.c_uint64), ("long_pieces", ctypes.c_uint64),
                ("tokens", ctypes.c_uint64), ("nfc_docs", ctypes.c_uint64), ("ms_segment", ctypes.c_double),
                ("ms_bpe_lo", ctypes.c_double), ("ms_bpe_hi", ctypes.c_double),
                ("class_bytes", ctypes.c_uint64 * 4), ("class_ids", ctypes.c_uint64 * 4),
                ("ms_bpe_med", ctypes.c_double), ("workspace_bytes", ctypes.c_uint64),
                ("long_rounds", ctypes.c_uint64)]

    def as_dict(self):
        d = {}
        for k, _ in self._fields_:
            v = getattr(self, k)
            d[k] = list(v) if isinstance(v, ctypes.Array) else v
        return d


class DecodeStats(ctypes.Structure):
    _fields_ = [("ms_total", ctypes.c_double), ("ms_device", ctypes.c_double), ("ms_len", ctypes.c_double),
                ("ms_gather", ctypes.c_double), ("ms_clean", ctypes.c_double), ("ms_h2d", ctypes.c_double),
                ("ms_d2h", ctypes.c_double), ("ids", ctypes.c_uint64), ("docs", ctypes.c_uint64),
                ("bytes_raw", ctypes.c_uint64), ("bytes_out", ctypes.c_uint64), ("direct", ctypes.c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


CTOK_D_SKIP_SPECIAL = 1
CTOK_D_CLEANUP = 2

CTOK_P_ADD_SPECIAL = 1
CTOK_P_PAIRS = 2
CTOK_P_TRUNCATE = 4
CTOK_P_PAD_LONGEST = 8
CTOK_P_PAD_TO_MAX = 16
CTOK_P_PAD_LEFT = 32
CTOK_P_PAD_ID = 64
CTOK_P_NO_POSTPROCESS = 128
CTOK_PP_SEQUENCE = 0xFFFFFFFF


class PadOpts(ctypes.Structure):
    _fields_ = [("flags", ctypes.c_uint32), ("pad_id", ctypes.c_uint32), ("max_length", ctypes.c_uint64)]


class Tables(ctypes.Structure):  # include/ctok.h ctok_tables
    _fields_ = [("vocab", ctypes.c_char_p), ("vocab_off", ctypes.c_void_p), ("vocab_id", ctypes.c_void_p),
                ("n_vocab", ctypes.c_uint64), ("merge_left", ctypes.c_void_p), ("merge_right", ctypes.c_void_p),
                ("n_merges", ctypes.c_uint64), ("added", ctypes.c_char_p), ("added_off", ctypes.c_void_p),
                ("added_id", ctypes.c_void_p), ("added_flags", ctypes.c_void_p), ("n_added", ctypes.c_uint64),
                ("nfc", ctypes.c_int), ("add_prefix_space", ctypes.c_int)]


class TrainerConfig(ctypes.Structure):  # include/ctok_trainer.h
    _fields_ = [("vocab_size", ctypes.c_uint64), ("min_frequency", ctypes.c_uint32),
                ("min_word_length", ctypes.c_uint64), ("inl_alpha", ctypes.c_float), ("inl_beta", ctypes.c_float),
                ("inl_gate", ctypes.c_float), ("inl_mu_target", ctypes.c_float),
                ("inl_velocity_max", ctypes.c_float), ("inl_beta_max", ctypes.c_float),
                ("special", ctypes.c_char_p), ("special_off", ctypes.POINTER(ctypes.c_uint64)),
                ("n_special", ctypes.c_uint64), ("device", ctypes.c_int)]


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
    "ctok_create_from_tables": (ctypes.c_int, [ctypes.POINTER(Tables), ctypes.POINTER(_p)]),
    "ctok_destroy": (None, [_p]),
    "ctok_vocab_size": (_u64, [_p]),
    "ctok_token_to_id": (ctypes.c_int, [_p, ctypes.c_char_p, _sz, _u32p]),
    "ctok_id_to_token": (ctypes.c_int, [_p, ctypes.c_uint32, ctypes.c_char_p, _sz, ctypes.POINTER(_sz)]),
    "ctok_num_special_tokens": (_u64, [_p]),
    "ctok_special_token": (ctypes.c_int, [_p, _u64, ctypes.c_char_p, _sz, ctypes.POINTER(_sz), _u32p]),
    "ctok_ids_bound": (_u64, [_p, _u64, _u64]),
    "ctok_num_piece_added_tokens": (_u64, [_p]),
    "ctok_piece_can_contain": (ctypes.c_int, [ctypes.c_char_p, _sz]),
    "ctok_encode_batch": (ctypes.c_int, [_p, _p, _p, _u64, _p, _u64, _p, ctypes.POINTER(Exec), ctypes.POINTER(Stats)]),
    "ctok_encode_batch_device": (ctypes.c_int, [_p, _p, _p, _u64, _u64, _p, _u64, _p, _u64p, ctypes.POINTER(Exec),
                                                ctypes.POINTER(Stats)]),
    "ctok_device_count": (ctypes.c_int, []),
    "ctok_encode_padded": (ctypes.c_int, [_p, _p, _p, _u64, ctypes.POINTER(PadOpts), _p, _p, _p, _p, _u64, _p, _u64p,
                                          ctypes.POINTER(Exec), ctypes.POINTER(Stats)]),
    "ctok_encode_padded_device": (ctypes.c_int, [_p, _p, _p, _u64, _u64, ctypes.POINTER(PadOpts), _p, _p, _p, _p, _u64, _p,
                                                 _u64p, ctypes.POINTER(Exec), ctypes.POINTER(Stats)]),
    "ctok_model_max_length": (_u64, [_p]),
    "ctok_pad_id": (ctypes.c_uint32, [_p]),
    "ctok_num_special_tokens_to_add": (_u64, [_p, ctypes.c_int]),
    "ctok_post_processor": (ctypes.c_int, [_p, _u32p, _u64, ctypes.POINTER(ctypes.c_int64)]),
    "ctok_encode_offsets": (ctypes.c_int, [_p, _p, _p, _u64, _p, _p, _p, _u64, _p, ctypes.POINTER(Exec)]),
    "ctok_decode_batch": (ctypes.c_int, [_p, _p, _p, _u64, ctypes.c_uint32, _p, _u64, _p, ctypes.POINTER(Exec),
                                         ctypes.POINTER(DecodeStats)]),
    "ctok_decode_batch_device": (ctypes.c_int, [_p, _p, _p, _u64, _u64, ctypes.c_uint32, _p, _u64, _p, _u64p,
                                                ctypes.POINTER(Exec), ctypes.POINTER(DecodeStats)]),
    # include/ctok_trainer.h
    "ctok_trainer_create": (ctypes.c_int, [ctypes.POINTER(TrainerConfig), ctypes.POINTER(_p)]),
    "ctok_trainer_destroy": (None, [_p]),
    "ctok_trainer_count": (ctypes.c_int, [_p, _p, _p, _u64, ctypes.c_int]),
    "ctok_trainer_clear_counts": (ctypes.c_int, [_p, ctypes.c_int]),
    "ctok_trainer_train": (ctypes.c_int, [_p, ctypes.c_int]),
    "ctok_trainer_train_words": (ctypes.c_int, [_p, _p, _p, _p, _u64]),
    "ctok_trainer_vocab_size": (_u64, [_p]),
    "ctok_trainer_num_merges": (_u64, [_p]),
    "ctok_trainer_json": (ctypes.c_int, [_p, ctypes.c_char_p, _sz, ctypes.POINTER(_sz)]),
    "ctok_trainer_save": (ctypes.c_int, [_p, ctypes.c_char_p]),
    "ctok_trainer_initial_pairs": (ctypes.c_int, [_p, _p, _p, _p, _u64, _u64p]),
    "ctok_trainer_timing": (ctypes.c_int, [_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double)]),
}

for _name, (_res, _args) in SIGS.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args


def last_error() -> str:
    return lib.ctok_last_error().decode("utf-8", "replace")
