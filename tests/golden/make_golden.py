#!/usr/bin/env python3
"""Generate the committed golden vectors (run in the dev container; the outputs are data).

  c1_gpt2_50k.npz     C1 corpus (1,000 docs) + ids from the Python oracle (ref_py), which is a
                      line-by-line restatement of the reference; cross-checked with the C oracle.
  edge_gpt2_50k.json  tests/edge_cases.py documents + their ids (ref_py).
  digests.json        sha256 over (tok_off u64 LE, ids u32 LE) for the full benchmark configs,
                      computed with the C oracle (ctok_ref.c), itself checked against ref_py on a
                      sample of the same corpus first.  Also digests of the first 100k docs (CPU tests).

Usage: python tests/golden/make_golden.py [c1 edge c2 c3 c4 c5]
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "complexity-tokenizer_amd")]

from datagen import corpus  # noqa: E402
from datagen.build_tokenizers import fixture_path  # noqa: E402
from oracle import ref_c, ref_py  # noqa: E402
from tests import edge_cases  # noqa: E402

TMP = "/tmp/ctok_golden"


def digest(ids, tok_off):
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(tok_off, dtype="<u8").tobytes())
    h.update(np.ascontiguousarray(ids, dtype="<u4").tobytes())
    return h.hexdigest()


def load(name):
    p = fixture_path(name, TMP)
    with open(p) as f:
        return json.load(f)


def c1():
    obj = load("gpt2_50k")
    py = ref_py.RefTokenizer(obj)
    text, off = corpus.corpus_c1()
    docs = [d.decode() for d in corpus.unpack(text, off)]
    res = py.encode_batch(docs)
    ids = np.array([i for r in res for i in r], dtype=np.uint32)
    tok_off = np.zeros(len(res) + 1, dtype=np.uint64)
    np.cumsum([len(r) for r in res], out=tok_off[1:])
    cids, coff = ref_c.RefC(obj).encode_packed(text, off)
    assert np.array_equal(cids, ids) and np.array_equal(coff, tok_off)
    np.savez_compressed(os.path.join(HERE, "c1_gpt2_50k.npz"), text=text, off=off, ids=ids, tok_off=tok_off)
    print("c1:", len(docs), "docs", len(ids), "ids")


def edge():
    obj = load("gpt2_50k")
    py = ref_py.RefTokenizer(obj)
    docs = edge_cases.EDGE + edge_cases.long_docs()
    out = [[d, py.encode(d)] for d in docs]
    with open(os.path.join(HERE, "edge_gpt2_50k.json"), "w") as f:
        json.dump(out, f, ensure_ascii=True)
    print("edge:", len(out), "docs")


CONFIGS = {  # name -> (tokenizer fixture, corpus fn)
    "C2": ("gpt2_50k", corpus.corpus_c2),
    "C3": ("llama3_128k", corpus.corpus_c3),
    "C5": ("multi_32k", corpus.corpus_c5),
    "C5NFC": ("multi_32k", corpus.corpus_c5nfc),
    "C3TT": ("llama3_tt_128k", corpus.corpus_c3),  # C3 with the tiktoken-style 304k-merge list
}


_PIN = {}


def _pin_init(obj):
    _PIN["py"] = ref_py.RefTokenizer(obj)


def _pin_chunk(docs):
    return _PIN["py"].encode_batch(docs)


def ref_py_packed(obj, docs, workers=7):
    """ref_py over `docs` on a pool of worker processes (the Python restatement is slow: ~1.5 ms per
    C5 document); (ids, tok_off) packed like the C oracle's."""
    import multiprocessing as mp
    step = max(1, len(docs) // (workers * 8))
    chunks = [docs[i:i + step] for i in range(0, len(docs), step)]
    with mp.get_context("fork").Pool(workers, initializer=_pin_init, initargs=(obj,)) as pool:
        res = [r for part in pool.map(_pin_chunk, chunks) for r in part]
    ids = np.array([i for r in res for i in r], dtype=np.uint32)
    tok_off = np.zeros(len(res) + 1, dtype=np.uint64)
    np.cumsum([len(r) for r in res], out=tok_off[1:])
    return ids, tok_off


# The C oracle (which produces every full-config digest) pinned against the Python restatement on
# the first PIN_DOCS documents of each config (>= 100k): ref_py uses the `regex`
# module and `unicodedata` directly, the C oracle the generated tables of csrc/gen/unicode_data.h,
# so the pin also covers the tables on the config's text.  Recorded as pin_ref_py in digests.json.
PIN_DOCS = {"C2": 100_000, "C5": 100_000, "C5NFC": 100_000, "C3": 20_000, "C3TT": 20_000}


def big(name):
    tok, fn = CONFIGS[name]
    obj = load(tok)
    t = time.time()
    text, off = fn()
    print(name, "corpus", len(off) - 1, "docs", len(text), "bytes in %.1fs" % (time.time() - t))
    rc = ref_c.RefC(obj)
    py = ref_py.RefTokenizer(obj)
    # pin the C oracle against the Python restatement on the config's first PIN_DOCS documents
    ns = PIN_DOCS[name]
    sample_docs = [d.decode() for d in corpus.unpack(text[: int(off[ns])], off[: ns + 1])]
    t = time.time()
    pid, poff = ref_py_packed(obj, sample_docs)
    cid, coff = rc.encode_packed(text[: int(off[ns])], off[: ns + 1])
    assert np.array_equal(pid, cid) and np.array_equal(poff, coff), name + ": C oracle disagrees with ref_py"
    print(name, "ref_py == C oracle on the first %d docs (%.0f s)" % (ns, time.time() - t), flush=True)
    del py
    t = time.time()
    ids, tok_off = rc.encode_packed(text, off)
    print(name, "C oracle %.1fs" % (time.time() - t), len(ids), "ids")
    n1 = min(100_000, len(off) - 1)
    ids1, off1 = ids[: int(tok_off[n1])], tok_off[: n1 + 1]
    path = os.path.join(HERE, "digests.json")
    d = json.load(open(path)) if os.path.exists(path) else {}
    d[name] = {"tokenizer": tok, "docs": len(off) - 1, "bytes": int(len(text)), "tokens": int(len(ids)),
               "sha256": digest(ids, tok_off), "first_docs": n1, "first_tokens": int(len(ids1)),
               "first_sha256": digest(ids1, off1),
               "pin_ref_py": {"docs": ns, "tokens": int(len(pid)), "sha256": digest(pid, poff)}}
    with open(path, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)


def c4_shard_digests(counts, ids_blocks, worlds=(1, 2, 4, 8)):
    """sha256 of (tok_off, ids) of every rank's shard (parallel.shard_bounds over C4's byte
    offsets) for each world size: what bench.py checks per rank."""
    from complexity_tokenizer.parallel import shard_bounds
    off = corpus.c4_offsets()
    tok_off = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    ids = np.concatenate(ids_blocks)
    out = {}
    for w in worlds:
        for r in range(w):
            d0, d1 = shard_bounds(off, w, r)
            t0, t1 = int(tok_off[d0]), int(tok_off[d1])
            out["%d/%d" % (r, w)] = {"docs": [d0, d1], "bytes": int(off[d1] - off[d0]), "tokens": t1 - t0,
                                     "sha256": digest(ids[t0:t1], tok_off[d0:d1 + 1] - np.uint64(t0))}
    return out


def c4():
    """C4 (10M docs, 1.28 GB) block by block through the C oracle; digests per shard."""
    obj = load("gpt2_50k")
    rc = ref_c.RefC(obj)
    py = ref_py.RefTokenizer(obj)
    n = corpus.C4_DOCS
    counts = np.zeros(n, dtype=np.int64)
    blocks = []
    t = time.time()
    for b in range(0, n, corpus.C4_BLOCK):
        e = min(n, b + corpus.C4_BLOCK)
        text, off = corpus.corpus_c4_range(b, e)
        if b == 0:  # pin the C oracle against ref_py on a sample of this corpus
            ns = 2000
            docs = [d.decode() for d in corpus.unpack(text[: int(off[ns])], off[: ns + 1])]
            assert py.encode_batch(docs) == rc.encode_batch(docs), "C4: C oracle disagrees with ref_py"
        ids, tok_off = rc.encode_packed(text, off)
        counts[b:e] = np.diff(tok_off.astype(np.int64))
        blocks.append(ids)
        print("C4 block %d: %d ids, %.1fs" % (b // corpus.C4_BLOCK, len(ids), time.time() - t), flush=True)
    path = os.path.join(HERE, "digests.json")
    d = json.load(open(path)) if os.path.exists(path) else {}
    d["C4"] = {"tokenizer": "gpt2_50k", "docs": n, "bytes": int(corpus.c4_offsets()[-1]),
               "tokens": int(counts.sum()), "shards": c4_shard_digests(counts, blocks)}
    with open(path, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)


def main(args):
    os.makedirs(TMP, exist_ok=True)
    for a in args or ["c1", "edge", "c2", "c3", "c5"]:
        if a == "c1":
            c1()
        elif a == "edge":
            edge()
        elif a == "c4":
            c4()
        else:
            big(a.upper())


if __name__ == "__main__":
    main(sys.argv[1:])
