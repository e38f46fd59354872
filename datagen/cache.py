"""Build full-size corpora into .npz files in the background (tests/conftest.py starts this at the
start of a GPU test session, so that the 1M-doc digest tests of tests/test_gpu_z_full_configs.py
find C2 / C5 / C5-NFC built while the other GPU tests run; building C5 takes about a minute of
one core).

  python -m datagen.cache OUTDIR C2          -> OUTDIR/C2.npz
  python -m datagen.cache OUTDIR C5 C5NFC    -> OUTDIR/C5.npz, OUTDIR/C5NFC.npz (C5-NFC from C5)

Each file is written to a temporary name and renamed when complete.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np


def _generator_key() -> str:
    """Short hash of the corpus generator's source: a cached corpus is reused only by the
    generator that wrote it (a changed generator writes new files instead of reading stale ones)."""
    import hashlib
    src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "corpus.py")
    with open(src, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:12]


def path_of(outdir: str, name: str) -> str:
    return os.path.join(outdir, "%s.%s.npz" % (name, _generator_key()))


def _save(outdir, name, text, off):
    p = path_of(outdir, name)
    tmp = "%s.%d.tmp.npz" % (p, os.getpid())  # (per writer: concurrent builders never share a temp file)
    np.savez(tmp, text=text, off=off)
    os.replace(tmp, p)


def build(outdir: str, names) -> None:
    from datagen import corpus
    os.makedirs(outdir, exist_ok=True)
    c5 = None
    for name in names:
        if os.path.exists(path_of(outdir, name)):
            continue
        t = time.time()
        if name == "C5":
            c5 = corpus.corpus_c5()
            text, off = c5
        elif name == "C5NFC":
            text, off = corpus.corpus_c5nfc(base=c5)
        elif name == "C4":  # 10M docs: independent 1M-doc blocks on worker processes
            text, off = corpus.corpus_c4(workers=min(16, len(os.sched_getaffinity(0))))
        elif name.startswith("C4S"):  # C4S<N>: rank 0's shard of the N-way split (bench.py --gpus N)
            text, off = c4_shard(int(name[3:]), 0)
        elif name == "C2L":  # C2's text cut into 100 documents of ~1.28 MB (long documents: tiles deep
            # inside a document, whose first document k_segment finds by bisecting the offsets)
            text, off = corpus.corpus_c2()
            off = np.linspace(0, len(text), 101).astype(np.uint64)
        else:
            text, off = corpus.CONFIGS[name]()
        _save(outdir, name, text, off)
        print("datagen.cache: %s built in %.1f s" % (name, time.time() - t), file=sys.stderr, flush=True)


def c4_shard(world: int, rank: int):
    """(text, off) of rank `rank`'s byte-balanced shard of C4 cut `world` ways -- the per-GPU work
    of bench.py --gpus `world` (complexity_tokenizer.parallel.shard_bounds)."""
    from datagen import corpus
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pkg = os.path.join(root, "complexity-tokenizer_amd")
    if pkg not in sys.path:
        sys.path.insert(0, pkg)
    from complexity_tokenizer.parallel import shard_bounds
    d0, d1 = shard_bounds(corpus.c4_offsets(corpus.C4_DOCS), world, rank)
    return corpus.corpus_c4_range(d0, d1, corpus.C4_DOCS, workers=min(8, len(os.sched_getaffinity(0))))


_PROCS: dict = {}  # corpus name -> the background process building it


def default_dir() -> str:
    return os.path.join(os.environ.get("TMPDIR", "/tmp"), "ctok_corpus", "full")


def start_background(outdir: str, groups) -> None:
    """One child interpreter per group of names (a fresh process: it never shares the parent's
    GPU state); call before anything touches the GPU."""
    import subprocess
    os.makedirs(outdir, exist_ok=True)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for names in groups:
        todo = [n for n in names if not os.path.exists(path_of(outdir, n))]
        if not todo:
            continue
        proc = subprocess.Popen([sys.executable, "-m", "datagen.cache", outdir] + list(names), cwd=root,
                                stdout=subprocess.DEVNULL)
        for n in names:
            _PROCS[n] = proc


def wait_load(outdir: str, name: str, timeout_s: float = 900.0):
    """(text, off) of a corpus being built by a background `datagen.cache` process; builds it in
    this process when none is (or it failed)."""
    p = path_of(outdir, name)
    proc = _PROCS.get(name)
    t0 = time.time()
    while proc is not None and proc.poll() is None and not os.path.exists(p) and time.time() - t0 < timeout_s:
        time.sleep(0.5)
    if not os.path.exists(p):
        build(outdir, [name])
    with np.load(p) as z:
        return z["text"], z["off"]


if __name__ == "__main__":
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if here not in sys.path:
        sys.path.insert(0, here)
    build(sys.argv[1], sys.argv[2:])
