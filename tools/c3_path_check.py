#!/usr/bin/env python3
"""Diagnostic (not product code): which class-3 path the scenarios of
tests/test_gpu_tiers.py::test_c3_sparse_queue_shards take -- run with CTOK_WGREC=1, the library
prints a k_bpe_sparse line when the sparse pass ran."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "complexity-tokenizer_amd"))
from complexity_tokenizer import Tokenizer  # noqa: E402
from datagen import corpus  # noqa: E402
from datagen.build_tokenizers import fixture_path  # noqa: E402

tok = Tokenizer.from_file(fixture_path("gpt2_50k", "/tmp"))
rng = random.Random(5)


def word(n):
    return "".join(rng.choice("etaoinshrdlu") for _ in range(n))


filler = [" ".join(word(rng.randint(2, 9)) for _ in range(700)) for _ in range(12)]
packed = [" ".join(word(rng.randint(33, 48)) for _ in range(40))] + filler
spread = [f + " " + word(rng.randint(33, 60)) for f in filler]
for name, docs in (("packed", packed), ("spread", spread)):
    text, off = corpus.pack([d.encode() for d in docs])
    print("== %s (CTOK_C3_SPARSE=%s)" % (name, os.environ.get("CTOK_C3_SPARSE", "default")), flush=True)
    tok.encode_packed(text, off, timing=True)
    print("class-3 ids", tok.last_stats["class_ids"][3], flush=True)
