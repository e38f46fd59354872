"""C4 (BASELINE.json configs[3]): 10M synthetic docs, 1.28 GB, GPT-2-shaped 50k BPE, the config
the 1/2/4/8-GPU curve is quoted on.  The reference's document parallelism (rayon `par_iter`,
src/huggingface/mod.rs:694-696) becomes one rank per GPU over byte-balanced doc shards
(complexity_tokenizer.parallel.shard_bounds); every shard's (tok_off, ids) must hash to the C
oracle's digest in tests/golden/digests.json.

* the whole corpus in one call (shard 0/1) and shards of the 8-way split, through
  encode_packed_device with the inputs resident in HBM (the bench's path);
* the multi-rank bench itself: `bench.py --gpus 2` spawned as a subprocess on the one-GPU box
  (the two ranks share device 0, each encodes its own shard and votes on its digest).
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from complexity_tokenizer import Tokenizer
from complexity_tokenizer.parallel import shard_bounds
from datagen import corpus

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))["C4"]


def digest(ids, tok_off):
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(tok_off, dtype="<u8").tobytes())
    h.update(np.ascontiguousarray(ids, dtype="<u4").tobytes())
    return h.hexdigest()


def _workers():
    return max(1, min(8, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))))


@pytest.fixture(scope="module")
def c4():
    assert GOLD["docs"] == corpus.C4_DOCS
    text, off = corpus.corpus_c4(corpus.C4_DOCS, workers=_workers())
    assert int(off[-1]) == GOLD["bytes"]
    return text, off


@pytest.fixture(scope="module")
def tok(gpt2_path):
    t = Tokenizer.from_file(gpt2_path)
    t.device = 0
    return t


def _encode_device(tok, text, off):
    import torch
    dev = torch.device("cuda", 0)
    n_docs, n_bytes = len(off) - 1, int(off[-1])
    d_text = torch.empty(n_bytes + 16, dtype=torch.uint8, device=dev)
    d_text[:n_bytes].copy_(torch.from_numpy(text[:n_bytes]))
    d_text[n_bytes:].zero_()
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    cap = n_bytes + n_docs + 16
    d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
    d_tok_off = torch.empty(n_docs + 1, dtype=torch.int64, device=dev)
    ntok = tok.encode_packed_device(d_text.data_ptr(), d_off.data_ptr(), n_docs, n_bytes, d_ids.data_ptr(), cap,
                                    d_tok_off.data_ptr(), device=0)
    torch.cuda.synchronize(dev)
    ids = d_ids[:ntok].cpu().numpy().view(np.uint32)
    toff = d_tok_off.cpu().numpy().view(np.uint64)
    del d_text, d_off, d_ids, d_tok_off
    torch.cuda.empty_cache()
    return ids, toff


def _check_shard(tok, c4, rank, world):
    text, off = c4
    key = "%d/%d" % (rank, world)
    want = GOLD["shards"][key]
    d0, d1 = shard_bounds(off, world, rank)
    assert [d0, d1] == want["docs"], key
    a, z = int(off[d0]), int(off[d1])
    ids, toff = _encode_device(tok, text[a:z], (off[d0:d1 + 1] - off[d0]).astype(np.uint64))
    assert len(ids) == want["tokens"], key
    assert int(toff[-1]) == want["tokens"], key
    assert digest(ids, toff) == want["sha256"], "C4 shard %s differs from the C-oracle digest" % key


def test_c4_whole_corpus_one_call(tok, c4):
    """1.28 GB, 10M docs, one ctok_encode_batch_device call (the bench's N = 1 step)."""
    _check_shard(tok, c4, 0, 1)
    assert tok.last_stats["tokens"] == GOLD["tokens"]


@pytest.mark.parametrize("rank", [0, 5, 7])
def test_c4_shards_of_eight(tok, c4, rank):
    """Shards of the 8-GPU split (the last one ends at the corpus end)."""
    _check_shard(tok, c4, rank, 8)


@pytest.mark.parametrize("rank", [1, 3])
def test_c4_shards_of_four(tok, c4, rank):
    _check_shard(tok, c4, rank, 4)


def _bench_ranks(c4, world, extra=()):
    """`bench.py --gpus world` with every rank on device 0 (RANK / LOCAL_RANK / WORLD_SIZE set by
    bench.py before any GPU call; gloo barrier, max-over-ranks timing, per-rank parity vote).  The
    ranks' shards are pre-built into bench.py's corpus cache from the module's corpus, so the ranks
    load them instead of rebuilding."""
    text, off = c4
    cache = os.path.join(os.environ.get("TMPDIR", "/tmp"), "ctok_corpus")
    os.makedirs(cache, exist_ok=True)
    n = corpus.C4_DOCS
    for r in range(world):
        d0, d1 = shard_bounds(off, world, r)
        p = os.path.join(cache, "c4_%d_%d_%d.npz" % (n, d0, d1))
        if not os.path.exists(p):
            a, z = int(off[d0]), int(off[d1])
            np.savez(p + ".%d.tmp.npz" % os.getpid(), text=text[a:z], off=(off[d0:d1 + 1] - off[d0]).astype(np.uint64))
            os.replace(p + ".%d.tmp.npz" % os.getpid(), p)
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    proc = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "2",
                           "--warmup", "1", "--no-cpu-baseline"] + list(extra), cwd=ROOT, env=env, capture_output=True,
                          text=True, timeout=540)
    sys.stderr.write(proc.stderr[-4000:])
    assert proc.returncode == 0, proc.stderr[-4000:]
    lines = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, proc.stdout
    out = json.loads(lines[0])
    if os.path.isdir(os.path.join(ROOT, "gpurun_out")):  # evidence for the GPU-box session log
        with open(os.path.join(ROOT, "gpurun_out", "bench_%drank_one_gpu.json" % world), "w") as f:
            f.write(lines[0] + "\n")
    assert out["n_gpus"] == world
    assert out["config"]["docs_total"] == n
    assert out["parity"].startswith("bit-exact"), out["parity"]
    assert "C4 shards of %d" % world in out["parity"]
    return out


@pytest.mark.timeout(600)
def test_bench_two_ranks_share_one_gpu(c4):
    out = _bench_ranks(c4, 2)
    assert out["value"] > 0 and out["config"]["tokens_per_gpu"] == GOLD["shards"]["0/2"]["tokens"]


@pytest.mark.timeout(600)
def test_bench_eight_ranks_share_one_gpu(c4):
    """Rehearsal of the driver's 8-GPU scaling run (bench.py --gpus 8) with the 8 ranks on device 0:
    every rank's shard of the 8-way split bit-exact against its golden digest (one vote per rank)."""
    out = _bench_ranks(c4, 8, ["--no-user-facing"])
    assert out["config"]["parallelism"] == "doc-sharded x8, no collectives"
    assert out["value"] > 0 and out["config"]["tokens_per_gpu"] == GOLD["shards"]["0/8"]["tokens"]
