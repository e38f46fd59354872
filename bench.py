#!/usr/bin/env python3
"""Benchmark: MB/s of raw UTF-8 encoded by the MI355X batch ByteLevel-BPE encode path.

Metric (BASELINE.json): "MB/s raw UTF-8 encoded (encode_batch), 50k ByteLevel BPE, 1/2/4/8 MI355X".
Workload per GPU = config C2 (BASELINE.json configs[1]): 1,000,000 synthetic English-like ASCII
docs of 96-160 bytes (~128 MB), GPT-2-shaped 50,257-token ByteLevel BPE (synthetic merges, no
network).  A step = one `ctok_encode_batch_device` call over the whole batch, inputs already
resident in HBM (pre-tokenize + routing, BPE merge passes, id emission + token offsets, ending
with the host reading the token count).  N > 1: one process per GPU (torch.distributed.run), every rank encodes its own
1M-doc shard (seed 2 + 1000*rank): weak scaling, no data-path collective (gloo only for the
barrier and the max-over-ranks timing).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--cpu-seconds S]
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "complexity-tokenizer_amd")]

METRIC = "MB/s raw UTF-8 encoded (encode_batch), 50k ByteLevel BPE, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def digest(ids, tok_off):
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(tok_off, dtype="<u8").tobytes())
    h.update(np.ascontiguousarray(ids, dtype="<u4").tobytes())
    return h.hexdigest()


def cpu_baseline(tok_path, text, off, seconds, threads):
    """The reference's algorithm as a faithful C port (oracle/ctok_ref.c) on the host cores,
    on a bounded sample (the first docs of this rank's batch)."""
    from oracle import ref_c
    rc = ref_c.RefC.from_file(tok_path)
    n_docs = len(off) - 1
    n0 = min(20_000, n_docs)
    t = time.perf_counter()
    rc.encode_packed(text[: int(off[n0])], off[: n0 + 1], threads)
    rate = int(off[n0]) / max(time.perf_counter() - t, 1e-9)  # bytes/s
    n = n_docs
    if int(off[-1]) / rate > seconds:
        n = int(np.searchsorted(off.astype(np.int64), int(rate * seconds)))
        n = max(n0, min(n, n_docs))
    t = time.perf_counter()
    rc.encode_packed(text[: int(off[n])], off[: n + 1], threads)
    dt = time.perf_counter() - t
    return {"value": round(int(off[n]) / dt / 1e6, 3), "unit": "MB/s", "cores": threads, "kind": "port",
            "sample": "first %d docs (%.1f MB) of the rank-0 C2 batch, %.1f s, oracle/ctok_ref.c (faithful C "
                      "restatement of the Rust reference: per-doc NFC + byte-map rebuild, O(n^2) merge rescans, "
                      "rayon-like doc threads)" % (n, int(off[n]) / 1e6, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    args = ap.parse_args()

    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="gloo")

    from complexity_tokenizer import Tokenizer
    from datagen import corpus
    from datagen.build_tokenizers import fixture_path

    tmp = os.path.join("/tmp", "ctok_bench_%d" % os.getpid())
    os.makedirs(tmp, exist_ok=True)
    tok_path = fixture_path("gpt2_50k", tmp)
    t0 = time.time()
    text, off = corpus.corpus_c2(args.docs, seed=2 + 1000 * rank)
    n_docs, n_bytes = len(off) - 1, int(off[-1])
    log("[bench] rank %d: corpus %d docs %.1f MB in %.1fs" % (rank, n_docs, n_bytes / 1e6, time.time() - t0))

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    tok = Tokenizer.from_file(tok_path)
    tok.device = local
    d_text = torch.from_numpy(np.concatenate([text, np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    cap = n_bytes + n_docs + 16
    d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
    d_tok_off = torch.empty(n_docs + 1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step(timing):
        return tok.encode_packed_device(d_text.data_ptr(), d_off.data_ptr(), n_docs, n_bytes, d_ids.data_ptr(), cap,
                                        d_tok_off.data_ptr(), stream=stream, timing=timing, device=local)

    for _ in range(args.warmup):
        ntok = step(False)

    parity = None
    if rank == 0 and not args.no_parity and args.docs == 1_000_000:
        gold = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json"))).get("C2")
        ids = d_ids[:ntok].cpu().numpy().view(np.uint32)
        toff = d_tok_off.cpu().numpy().view(np.uint64)
        ok = gold is not None and digest(ids, toff) == gold["sha256"]
        parity = ("bit-exact: sha256(tok_off, ids) of all %d docs == C-oracle golden (tests/golden/digests.json)"
                  % n_docs) if ok else "MISMATCH vs golden digest"
        log("[bench] parity:", parity)

    # timed region: K steps bracketed by barrier + synchronize
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    stats = []
    for _ in range(args.steps):
        ntok = step(True)
        stats.append(dict(tok.last_stats))
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    elapsed_t = torch.tensor([elapsed], dtype=torch.float64)
    bytes_t = torch.tensor([float(n_bytes)], dtype=torch.float64)
    if dist:
        dist.all_reduce(elapsed_t, op=dist.ReduceOp.MAX)
        dist.all_reduce(bytes_t, op=dist.ReduceOp.SUM)
    elapsed_max = float(elapsed_t.item())
    total_bytes = float(bytes_t.item())

    def avg(k):
        return float(np.mean([s[k] for s in stats]))

    st = stats[-1]
    P, T, B, D = st["pieces"], st["tokens"], st["bytes_norm"], st["docs"]
    # Per-kernel rooflines (HIP events on the encode stream, averaged over the timed steps).
    # Algorithmic bytes per launch (DESIGN.md "Measurement"):
    #   k_segment:      text read (B) + doc-start bitmap read (B/8) + piece-start bitmap written (B/8)
    #   merge passes:   text bytes of the pieces of their length classes + 4 B per id written
    #                   (k_bpe_short: <= 16 B, k_bpe_mid: 17..32 B; 33..64 B run on the side stream)
    cb, ci = st["class_bytes"], st["class_ids"]
    kernels = {
        "k_segment": (avg("ms_segment"), 1.25 * B),
        "k_bpe_short": (avg("ms_bpe_lo"), cb[0] + cb[1] + 4 * (ci[0] + ci[1])),
        "k_bpe_mid": (avg("ms_bpe_hi"), cb[2] + 4 * ci[2]),
    }
    dom = max(kernels, key=lambda k: kernels[k][0])
    ms_dom, alg_dom = kernels[dom]
    ach = alg_dom / (ms_dom * 1e-3) / 1e9
    # whole pipeline: B_alg = sum L + 4 sum T + 16 (D+1)
    b_alg = B + 4 * T + 16 * (D + 1)
    ms_dev = avg("ms_device")

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            threads = min(16, os.cpu_count() or 1)
            cpu = cpu_baseline(tok_path, text, off, args.cpu_seconds, threads)
        traffic = None  # HBM bytes per launch of the dominant kernel from the committed PMC passes
        tr_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(tr_path):
            per = json.load(open(tr_path)).get("hbm_bytes_per_launch", {})
            hits = [v for k, v in per.items() if k.split("<")[0] == dom]
            traffic = hits[0] if len(hits) == 1 else None
        ms_step = elapsed_max / args.steps * 1e3
        out = {
            "metric": METRIC,
            "value": round(total_bytes * args.steps / elapsed_max / 1e6, 2),
            "unit": "MB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (datagen/corpus.py C2 generator, seed 2+1000*rank; synthetic GPT-2-shaped tokenizer)",
            "config": {"workload": "C2: %d docs x 96-160 B ASCII per GPU (%.1f MB), GPT-2-shaped 50,257-token "
                                   "ByteLevel BPE" % (n_docs, n_bytes / 1e6),
                       "docs_per_gpu": n_docs, "bytes_per_gpu": n_bytes, "tokens_per_gpu": int(T),
                       "parallelism": "doc-sharded x%d, no collectives" % world},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(ach, 2), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 5), "traffic": traffic,
                         "alg_bytes_per_launch": int(alg_dom), "ms_per_launch": round(ms_dom, 4),
                         "kernels": {k: {"ms": round(v[0], 4), "alg_bytes": int(v[1]),
                                         "GBps": round(v[1] / (v[0] * 1e-3) / 1e9, 2)} for k, v in kernels.items()}},
            "pipeline": {"ms_device": round(ms_dev, 4), "ms_pretok": round(avg("ms_pretok"), 4),
                         "ms_bpe_short": round(avg("ms_bpe_short"), 4), "ms_bpe_long": round(avg("ms_bpe_long"), 4),
                         "ms_emit": round(avg("ms_emit"), 4), "ms_call": round(avg("ms_total"), 4),
                         "B_alg": int(b_alg), "achieved_GBps": round(b_alg / (ms_dev * 1e-3) / 1e9, 2),
                         "pieces": int(P), "long_pieces": int(st["long_pieces"]),
                         "kernel_MBps": round(n_bytes / (ms_dev * 1e-3) / 1e6, 1)},
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
