"""Debug helper: encode edge-case docs one by one on the GPU with per-kernel sync logging."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "complexity-tokenizer_amd")]
from complexity_tokenizer import Tokenizer  # noqa: E402
from datagen.build_tokenizers import fixture_path  # noqa: E402
from oracle import ref_py  # noqa: E402
from tests import edge_cases  # noqa: E402

p = fixture_path("gpt2_50k", "/tmp")
tok = Tokenizer.from_file(p)
py = ref_py.RefTokenizer(json.load(open(p)))
docs = edge_cases.EDGE + edge_cases.long_docs()
bad = 0
for i, d in enumerate(docs):
    print("doc", i, repr(d[:40]), len(d), flush=True)
    t = time.time()
    g = tok.encode(d)
    r = py.encode(d)
    if g != r:
        bad += 1
        print("  MISMATCH gpu", g[:20], "ref", r[:20], flush=True)
    print("  ok %.3fs" % (time.time() - t), flush=True)
print("bad", bad)
