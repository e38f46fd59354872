#!/usr/bin/env python3
"""Device-path probe for one matrix config (profiling helper for rocprofv3, not product code):
usage probe.py CONFIG [fixture] [reps] -- e.g. probe.py c5 multi_32k 5."""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "complexity-tokenizer_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from complexity_tokenizer import Tokenizer  # noqa: E402
from datagen import corpus  # noqa: E402
from datagen.build_tokenizers import fixture_path  # noqa: E402

cfg = sys.argv[1].upper() if len(sys.argv) > 1 else "C3"
fx = sys.argv[2] if len(sys.argv) > 2 else {"C3": "llama3_128k", "C5": "multi_32k", "C5NFC": "multi_32k"}.get(cfg, "gpt2_50k")
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
tok = Tokenizer.from_file(fixture_path(fx, "/tmp"))
print("building %s" % cfg, flush=True)  # (cached per box under $TMPDIR: A/B runs reuse it)
from datagen import cache  # noqa: E402
cache.build(cache.default_dir(), [cfg])
text, off = cache.wait_load(cache.default_dir(), cfg)
nb, nd = int(off[-1]), len(off) - 1
d_text = torch.zeros(nb + 64, dtype=torch.uint8, device="cuda")
d_text[:nb] = torch.from_numpy(text).cuda()
d_off = torch.from_numpy(off.astype(np.int64)).cuda()
cap = 3 * nb + nd + 16
d_ids = torch.empty(cap, dtype=torch.int32, device="cuda")
d_tok = torch.empty(nd + 1, dtype=torch.int64, device="cuda")
args = (d_text.data_ptr(), d_off.data_ptr(), nd, nb, d_ids.data_ptr(), cap, d_tok.data_ptr())
tok.encode_packed_device(*args)
ts = []
timing = os.environ.get("PROBE_TIMING", "1") != "0"  # (0: calls without the per-kernel events)
for _ in range(reps):
    t = time.perf_counter()
    tok.encode_packed_device(*args, timing=timing)
    ts.append(time.perf_counter() - t)
if not timing:
    tok.encode_packed_device(*args, timing=True)
st = tok.last_stats
# the last call's output against the golden digest of the config (tests/golden/digests.json)
gold = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json"))).get(cfg)
if cfg.startswith("C4S"):  # C4S<N>: rank 0's shard of the N-way split
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))["C4"]
    gold = dict(gold, sha256=gold["shards"]["0/%d" % int(cfg[3:])]["sha256"])
elif gold is not None and "shards" in gold:  # C4: the digest of the 1-way shard is the whole corpus's
    gold = dict(gold, sha256=gold["shards"]["0/1"]["sha256"])
parity = "no golden digest"
if gold is not None and gold["tokenizer"] == fx:
    torch.cuda.synchronize()
    h = hashlib.sha256()
    h.update(d_tok.cpu().numpy().view(np.uint64).tobytes())
    h.update(d_ids[: int(d_tok[-1])].cpu().numpy().view(np.uint32).tobytes())
    parity = "digest ok" if h.hexdigest() == gold["sha256"] else "DIGEST MISMATCH"
print("%s%s %s: %d docs %d B, call %.3f ms (%.0f MB/s), device %.3f ms, long %.3f ms, long pieces %d, nfc docs %d, %s" % (
    "" if timing else "untimed ", cfg, fx, nd, nb, min(ts) * 1e3, nb / min(ts) / 1e6, st["ms_device"], st["ms_bpe_long"], st["long_pieces"],
    st.get("nfc_docs", -1), parity), flush=True)
print({k: v for k, v in st.items() if k.startswith("ms_")}, flush=True)
