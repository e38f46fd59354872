"""TEST / MEASUREMENT INFRASTRUCTURE ONLY -- ctypes wrapper of oracle/trainer_ref.c, the C
restatement of the reference trainer's per-merge work (apply_merge_incremental +
build_heap every 100 merges, /root/reference/src/trainer.rs:369-405, :519-588), used as the CPU
baseline of the trainer timing (tools/trainer_timing.py).  The merge sequence is an input."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libtrainer_ref.so")


def _lib():
    if not os.path.exists(_LIB):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    L = ctypes.CDLL(_LIB)
    P, U32, I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    L.trm_run.restype = ctypes.c_uint64
    L.trm_run.argtypes = [U32, P, P, P, P, U32, P, P, P, P, U32, I, ctypes.POINTER(ctypes.c_double),
                          ctypes.POINTER(ctypes.c_double)]
    return L


def run(words, merges, token_freqs, n_ids, threads=1):
    """words: [(token ids, freq)]; merges: [(a, b, new_id)]; token_freqs: {id: freq}.  Applies the
    merges with the reference's bookkeeping; returns (final token lists, seconds in the merges,
    seconds in the heap rebuilds, live pairs left)."""
    lens = np.array([len(t) for t, _ in words], dtype=np.uint32)
    off = np.zeros(len(words) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    toks = np.array([x for t, _ in words for x in t], dtype=np.uint32)
    freq = np.array([f for _, f in words], dtype=np.uint64)
    m = np.array(merges, dtype=np.uint32).reshape(-1, 3)
    ma, mb, mn = (np.ascontiguousarray(m[:, i]) for i in range(3))
    tf = np.zeros(n_ids, dtype=np.uint64)
    for k, v in token_freqs.items():
        if k < n_ids:
            tf[k] = v
    sm, sh = ctypes.c_double(), ctypes.c_double()
    live = _lib().trm_run(len(words), off.ctypes.data, toks.ctypes.data, lens.ctypes.data, freq.ctypes.data, len(m),
                          ma.ctypes.data, mb.ctypes.data, mn.ctypes.data, tf.ctypes.data, n_ids, threads,
                          ctypes.byref(sm), ctypes.byref(sh))
    out = [toks[int(off[i]):int(off[i]) + int(lens[i])].tolist() for i in range(len(words))]
    return out, sm.value, sh.value, int(live)
