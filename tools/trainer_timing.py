#!/usr/bin/env python3
"""Trainer timing: the GPU trainer (complexity_tokenizer.Trainer, pair histogram and
merge passes on the GPU, csrc/trainer.hip) against the C restatement of the reference's per-merge
work (oracle/trainer_ref.c: apply_merge_incremental + build_heap every 100 merges,
/root/reference/src/trainer.rs:369-405, :519-588) on the same words and the same merge sequence.
Prints one JSON line.   usage: python tools/trainer_timing.py [n_docs] [vocab_size]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "complexity-tokenizer_amd")]

from complexity_tokenizer import Trainer  # noqa: E402
from datagen import corpus  # noqa: E402
from oracle import trainer_c, trainer_ref  # noqa: E402

n_docs = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000
vocab_size = int(sys.argv[2]) if len(sys.argv) > 2 else 2_200
text, off = corpus.corpus_c2(n_docs, seed=31)
texts = [d.decode() for d in corpus.unpack(text, off)]

gpu = Trainer(vocab_size=vocab_size, min_frequency=2)
t = time.perf_counter()
gpu.train_from_iterator(texts)
wall = time.perf_counter() - t
tm = gpu.timing()
obj = json.loads(gpu.to_str())
vocab = obj["model"]["vocab"]
merges = [(vocab[a], vocab[b], vocab[a + b]) for a, b in (m.split(" ") for m in obj["model"]["merges"])]

ref = trainer_ref.RefTrainer(vocab_size=vocab_size, min_frequency=2)
wf = {}
ref._count_into(wf, texts)
wf = {w: c for w, c in wf.items() if c >= 2}
words = ref.init_vocab_bytelevel(wf)
assert all(ref.vocab.get(k) == v for k, v in vocab.items() if k in ref.vocab)
n_ids = max(vocab.values()) + 1
threads = len(os.sched_getaffinity(0))
try:
    q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
    if q != "max":
        threads = max(1, min(threads, int(int(q) / int(p))))
except (OSError, ValueError):
    pass
res = {}
for th in sorted({1, threads}):
    _, sm, sh, _ = trainer_c.run([(list(tk), f) for tk, f in words], merges, dict(ref.token_freqs), n_ids, th)
    res[th] = {"ms_per_merge": round(1e3 * (sm + sh) / len(merges), 4), "ms_merges": round(1e3 * sm, 1),
               "ms_heap": round(1e3 * sh, 1)}
print(json.dumps({
    "what": "trainer per-merge cost on %d C2 docs (%d words, %d merges)" % (n_docs, len(words), len(merges)),
    "gpu": {"ms_per_merge": round((tm["ms_merges"] + tm["ms_heap"]) / len(merges), 4), "ms_pairs": round(tm["ms_pairs"], 2),
            "ms_merges": round(tm["ms_merges"], 1), "ms_heap": round(tm["ms_heap"], 1), "wall_s": round(wall, 2)},
    "cpu_c_restatement": {"threads": res, "note": "oracle/trainer_ref.c: apply_merge_incremental (words split over "
                          "threads, per-thread delta maps aggregated, retain) + build_heap every 100 merges, fed the GPU "
                          "run's merge sequence"},
}), flush=True)
