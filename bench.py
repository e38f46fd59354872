#!/usr/bin/env python3
"""Benchmark: MB/s of raw UTF-8 encoded by the MI355X batch ByteLevel-BPE encode path.

Metric (BASELINE.json): "MB/s raw UTF-8 encoded (encode_batch), 50k ByteLevel BPE, 1/2/4/8 MI355X".

Workload (default, --config c4): BASELINE.json configs[3], the config the 1/2/4/8 curve is quoted
on -- 10,000,000 synthetic English-like ASCII docs of 96-160 B (1.28 GB, the C2 generator in
independent 1M-doc blocks, datagen/corpus.py), GPT-2-shaped 50,257-token ByteLevel BPE
(synthetic merges, no network).  The batch is cut into N contiguous byte-balanced doc shards
(complexity_tokenizer.parallel.shard_bounds), one per GPU: strong scaling, no data-path
collective (gloo only for the barrier, the max-over-ranks time and the parity vote).  At N = 1
the whole 1.28 GB is one call on one GPU.  --config c2 runs configs[1] instead (1M docs per GPU,
weak scaling).

A step = one `ctok_encode_batch_device` call over the rank's shard with its inputs already
resident in HBM (pre-tokenize + routing, BPE merge passes, id emission + token offsets, ending
with the host reading the token count).  `value` = bytes of all shards x steps / max-over-ranks
wall time of the K timed steps.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c2] [--cpu-seconds S]

With --gpus N > 1 and no WORLD_SIZE in the environment, N child processes (one per GPU) are
started before anything touches the GPU; under torch.distributed.run the ranks come from
RANK / LOCAL_RANK / WORLD_SIZE.
"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
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


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_share():
    """CPUs the cgroup lets this process use (cpu.max quota), or None when unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(tok_path, text, off, seconds):
    """The reference's algorithm as a faithful C port (oracle/ctok_ref.c) on the host cores, on
    a bounded sample (the first docs of this rank's shard): rayon's default thread count (every
    CPU of the affinity mask, reference src/huggingface/mod.rs:695) and one thread."""
    from oracle import ref_c
    rc = ref_c.RefC.from_file(tok_path)
    # rayon's default pool size is std::thread::available_parallelism(): the affinity mask,
    # capped by the cgroup v2 CPU quota on Linux
    threads = len(os.sched_getaffinity(0))
    quota = cpu_share()
    if quota:
        threads = max(1, min(threads, int(quota)))
    n_docs = len(off) - 1

    def timed(n, th):
        t = time.perf_counter()
        rc.encode_packed(text[: int(off[n])], off[: n + 1], th)
        return int(off[n]) / max(time.perf_counter() - t, 1e-9)

    def sized(rate, secs):  # docs for about `secs` of work at `rate` bytes/s
        return max(1000, min(n_docs, int(np.searchsorted(off.astype(np.int64), int(rate * secs)))))

    r1 = timed(min(2000, n_docs), 1)
    n1 = sized(r1, 0.25 * seconds)
    r1 = timed(n1, 1)
    rn = timed(min(20_000, n_docs), threads)
    nn = sized(rn, 0.75 * seconds)
    t = time.perf_counter()
    rc.encode_packed(text[: int(off[nn])], off[: nn + 1], threads)
    dt = time.perf_counter() - t
    return {"value": round(int(off[nn]) / dt / 1e6, 3), "unit": "MB/s", "cores": threads, "kind": "port",
            "value_1thread": round(r1 / 1e6, 3), "cpu_model": cpu_model(), "cgroup_cpus": cpu_share(),
            "sample": "first %d docs (%.1f MB) of the rank-0 shard, %.1f s on %d threads (rayon default: every CPU "
                      "of the affinity mask, capped by the cgroup CPU quota); 1-thread figure on the first %d docs; oracle/ctok_ref.c (faithful C "
                      "restatement of the Rust reference: per-doc NFC + byte-map rebuild, O(n^2) merge rescans, "
                      "rayon-like doc threads)" % (nn, int(off[nn]) / 1e6, dt, threads, n1)}


def user_facing(tok, text, off, ids_dev, toff_dev, reps, py_docs):
    """The user-facing rates of SURVEY.md 8(d), outside the headline `value`, on this rank's shard:
    `e2e` -- ctok_encode_batch from host buffers (text up, ids and offsets down through the chunked
    pipeline, include/ctok.h) into a reused output buffer, its result checked against the
    device-resident run's (itself checked against the golden digest); `python` --
    Tokenizer.encode_batch(list[str]) -> list[list[int]] (the reference's API,
    src/bindings/tokenizer.rs:207-210) on the shard's first `py_docs` docs, checked the same way."""
    import ctypes
    from complexity_tokenizer import _native as _n
    n_docs, n_bytes = len(off) - 1, int(off[-1])
    T = int(toff_dev[-1])
    ids = np.empty(T + 16, dtype=np.uint32)
    toff = np.empty(n_docs + 1, dtype=np.uint64)
    text = np.ascontiguousarray(text)
    off = np.ascontiguousarray(off, dtype=np.uint64)

    def call():
        ex = tok._host_exec(False)
        t = time.perf_counter()
        rc = _n.lib.ctok_encode_batch(tok._h, text.ctypes.data, off.ctypes.data, n_docs, ids.ctypes.data, T + 16,
                                      toff.ctypes.data, ctypes.byref(ex), None)
        dt = time.perf_counter() - t
        if rc != _n.CTOK_OK:
            raise RuntimeError("ctok_encode_batch: %d %s" % (rc, _n.last_error()))
        return dt

    call()  # (first touch of the output pages)
    ts = sorted(call() for _ in range(reps))
    e2e_ok = np.array_equal(toff, toff_dev) and np.array_equal(ids[:T], ids_dev)
    m = min(py_docs, n_docs)
    docs = [bytes(text[int(off[i]):int(off[i + 1])]).decode() for i in range(m)]
    tp = []
    for _ in range(3):
        t = time.perf_counter()
        got = tok.encode_batch(docs)
        tp.append(time.perf_counter() - t)
    py_ok = all(got[i] == ids_dev[int(toff_dev[i]):int(toff_dev[i + 1])].tolist() for i in range(m))
    tp.sort()
    mb = int(off[m]) / 1e6
    return {
        "e2e": {"value": round(n_bytes / ts[len(ts) // 2] / 1e6, 1), "unit": "MB/s", "ms_per_call": round(ts[len(ts) // 2] * 1e3, 3),
                "calls": reps, "parity": "identical to the digest-checked device run" if e2e_ok else "MISMATCH",
                "what": "ctok_encode_batch on the rank's whole shard from host buffers (pageable numpy; text up, "
                        "ids + offsets down over PCIe, chunked pipeline), reused output buffer, median call"},
        "python": {"value": round(mb / tp[1], 1), "unit": "MB/s", "ms_per_call": round(tp[1] * 1e3, 2), "docs": m,
                   "parity": "identical to the digest-checked device run" if py_ok else "MISMATCH",
                   "what": "Tokenizer.encode_batch(list[str]) -> list[list[int]] on the shard's first %d docs "
                           "(%.1f MB), median of 3" % (m, mb)},
    }


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """One child per GPU (RANK / LOCAL_RANK / WORLD_SIZE set), started before any GPU call in
    this process; returns the worst exit status."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return next((c for c in rcs if c != 0), 0)


def workload(args, rank, world):
    """(text, off, description dict) of this rank's shard."""
    from datagen import corpus
    from complexity_tokenizer.parallel import shard_bounds
    if args.config == "c2":
        n = args.docs or 1_000_000
        text, off = corpus.corpus_c2(n, seed=2 + 1000 * rank)
        return text, off, {"workload": "C2: %d docs x 96-160 B ASCII per GPU, GPT-2-shaped 50,257-token ByteLevel "
                                       "BPE (weak scaling)" % n, "docs_total": n * world}, None
    n = args.docs or corpus.C4_DOCS
    full = corpus.c4_offsets(n)
    d0, d1 = shard_bounds(full, world, rank)
    cpus = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    # shards are cached under /tmp: a profiled rerun (rocprofv3 --pmc initialises the GPU before
    # main) must not fork a corpus pool, so it reads what the unprofiled run built
    cache = os.path.join(os.environ.get("TMPDIR", "/tmp"), "ctok_corpus", "c4_%d_%d_%d.npz" % (n, d0, d1))
    # under a profiler (rocprofv3 sets ROCPROF_* variables for the program) the corpus is
    # built without a process pool when no cached shard exists: the profiler would follow the
    # forked workers
    profiled = any(k.startswith("ROCPROF") for k in os.environ)
    if os.path.exists(cache):
        z = np.load(cache)
        text, off = z["text"], z["off"]
    else:
        text, off = corpus.corpus_c4_range(d0, d1, n, workers=1 if (args.corpus_workers == 1 or profiled) else
                                           max(1, min(8, cpus // world)))
        try:
            os.makedirs(os.path.dirname(cache), exist_ok=True)
            np.savez(cache + ".tmp.npz", text=text, off=off)
            os.replace(cache + ".tmp.npz", cache)
        except OSError:
            pass
    desc = {"workload": "C4: %d docs x 96-160 B ASCII (%.2f GB), GPT-2-shaped 50,257-token ByteLevel BPE, "
                        "byte-balanced doc shards over %d GPU(s)" % (n, int(full[-1]) / 1e9, world),
            "docs_total": n, "bytes_total": int(full[-1])}
    return text, off, desc, ("%d/%d" % (rank, world), d0, d1, n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=["c4", "c2"], default="c4")
    ap.add_argument("--docs", type=int, default=0, help="override the doc count (tests; parity needs the default)")
    ap.add_argument("--cpu-seconds", type=float, default=16.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--corpus-workers", type=int, default=0, help="1: build the corpus without a process pool")
    ap.add_argument("--no-user-facing", action="store_true", help="skip the e2e / python rates (rank 0, after timing)")
    ap.add_argument("--py-docs", type=int, default=100_000)
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log("[bench] --gpus %d but WORLD_SIZE=%d: run one process per GPU (torch.distributed.run "
            "--nproc-per-node %d) or let bench.py start them" % (args.gpus, world, args.gpus))
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    # torch only holds device buffers here: one intra-op CPU thread, so its spinning pool does not
    # take the cgroup's CPUs from the CPU baseline's threads (tools/bench_matrix.py, same reason)
    torch.set_num_threads(1)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="gloo")

    from complexity_tokenizer import Tokenizer
    from datagen.build_tokenizers import fixture_path

    tmp = os.path.join("/tmp", "ctok_bench_%d" % os.getpid())
    os.makedirs(tmp, exist_ok=True)
    tok_path = fixture_path("gpt2_50k", tmp)
    t0 = time.time()
    text, off, desc, shard = workload(args, rank, world)
    n_docs, n_bytes = len(off) - 1, int(off[-1])
    log("[bench] rank %d: shard %d docs %.1f MB built in %.1fs" % (rank, n_docs, n_bytes / 1e6, time.time() - t0))

    n_dev = max(1, torch.cuda.device_count())
    if local >= n_dev:  # a rehearsal of N ranks on fewer GPUs: ranks share devices
        log("[bench] rank %d: LOCAL_RANK %d >= %d visible GPU(s), sharing device %d" % (rank, local, n_dev, local % n_dev))
    local = local % n_dev
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

    # parity (outside the timed region): this rank's (tok_off, ids) against the C-oracle digest
    # of its shard (tests/golden/digests.json), one vote per rank
    parity, bad = None, 0
    if not args.no_parity:
        gold = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))
        want = None
        if args.config == "c4" and shard[3] == gold["C4"]["docs"]:
            want = gold["C4"]["shards"].get(shard[0], {}).get("sha256")
        elif args.config == "c2" and rank == 0 and n_docs == gold["C2"]["docs"]:
            want = gold["C2"]["sha256"]
        if want is not None:
            ids = d_ids[:ntok].cpu().numpy().view(np.uint32)
            toff = d_tok_off.cpu().numpy().view(np.uint64)
            bad = 0 if digest(ids, toff) == want else 1
            del ids, toff
        else:
            bad = -1  # no golden digest for this shape
    votes = torch.tensor([1.0 if bad == 0 else 0.0, 1.0 if bad == 1 else 0.0], dtype=torch.float64)
    if dist:
        dist.all_reduce(votes, op=dist.ReduceOp.SUM)
    if not args.no_parity:
        if votes[1] > 0:
            parity = "MISMATCH vs golden digest on %d of %d rank(s)" % (int(votes[1]), world)
        elif votes[0] == world:
            parity = ("bit-exact: sha256(tok_off, ids) of every rank's shard == C-oracle golden "
                      "(tests/golden/digests.json, %s)" % ("C4 shards of %d" % world if args.config == "c4" else "C2"))
        else:
            parity = "unchecked on %d rank(s): no golden digest for this shape" % (world - int(votes[0]))
        if rank == 0:
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
    # Algorithmic bytes per launch, SURVEY.md 8(d)'s terms only (implementation
    # traffic -- bitmaps, lists, records, scratch ids, tables -- is not counted):
    #   k_segment:      the text (B) + the input document offsets (8 B per offset)
    #   k_bpe_short:    the text bytes of the <= 16 B pieces left to merge + 4 B per id they become
    #   k_bpe_mid<2>:   the same for the 17..32 B pieces
    #   k_emit:         the output ids (4 B each) + the output offsets (8 B each; with the tile scan
    #                   and k_tokoff)
    cb, ci = st["class_bytes"], st["class_ids"]
    kernels = {
        "k_segment": (avg("ms_segment"), B + 8 * (D + 1)),
        "k_bpe_short": (avg("ms_bpe_lo"), cb[0] + cb[1] + 4 * (ci[0] + ci[1])),
        "k_bpe_mid": (avg("ms_bpe_hi"), cb[2] + 4 * ci[2]),
        "k_emit": (avg("ms_emit"), 4 * T + 8 * (D + 1)),
    }
    dom = max(kernels, key=lambda k: kernels[k][0])
    ms_dom, alg_dom = kernels[dom]
    ach = alg_dom / (ms_dom * 1e-3) / 1e9
    # whole pipeline: B_alg = sum L + 4 sum T + 16 (D+1)
    b_alg = B + 4 * T + 16 * (D + 1)
    ms_dev = avg("ms_device")

    uf = None
    if rank == 0 and not args.no_user_facing:
        ids_dev = d_ids[:ntok].cpu().numpy().view(np.uint32)
        toff_dev = d_tok_off.cpu().numpy().view(np.uint64)
        del d_ids
        torch.cuda.empty_cache()
        uf = user_facing(tok, text, off, ids_dev, toff_dev, 5, args.py_docs)
        log("[bench] e2e %.1f MB/s, python %.1f MB/s" % (uf["e2e"]["value"], uf["python"]["value"]))
        del ids_dev, toff_dev

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(tok_path, text, off, args.cpu_seconds)
        # HBM bytes per launch of the dominant kernel from the committed PMC passes -- only when
        # they profiled this very library build (sha256 of the loaded libctok.so) and workload
        traffic, traffic_src = None, "no PMC record for this workload"
        tr_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(tr_path):
            from complexity_tokenizer import _native
            with open(_native.LIB_PATH, "rb") as fh:
                lib_sha = hashlib.sha256(fh.read()).hexdigest()
            tr = json.load(open(tr_path))
            if tr.get("workload") != "%s/%d" % (args.config, n_docs):
                pass
            elif tr.get("lib_sha256") != lib_sha:
                traffic_src = "PMC record of another libctok.so build (%s), not this one (%s): unmeasured" % (
                    str(tr.get("lib_sha256"))[:12], lib_sha[:12])
            else:
                per = tr.get("hbm_bytes_per_launch", {})
                hits = [v for k, v in per.items() if k.split("<")[0] == dom]
                traffic = hits[0] if len(hits) == 1 else None
                traffic_src = ("profiles/pmc_traffic.json (FETCH_SIZE x %s + WRITE_SIZE x 1, libctok.so sha256 %s; factors "
                               "calibrated in %s: reads beyond L2, Infinity-Cache hits included)" % (
                                   tr.get("fetch_correction"), lib_sha[:12], tr.get("calibration", "uncalibrated")))
        ms_step = elapsed_max / args.steps * 1e3
        cfg = dict(desc)
        cfg.update({"docs_per_gpu": n_docs, "bytes_per_gpu": n_bytes, "tokens_per_gpu": int(T),
                    "parallelism": "doc-sharded x%d, no collectives" % world})
        out = {
            "metric": METRIC,
            "value": round(total_bytes * args.steps / elapsed_max / 1e6, 2),
            "unit": "MB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if args.config == "c4" else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (datagen/corpus.py %s generator; synthetic GPT-2-shaped tokenizer)" % args.config.upper(),
            "config": cfg,
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(ach, 2), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 5), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "alg_bytes_per_launch": int(alg_dom), "ms_per_launch": round(ms_dom, 4),
                         "kernels": {k: {"ms": round(v[0], 4), "alg_bytes": int(v[1]),
                                         # (k_bpe_mid's ms: the time it adds after k_bpe_short's end, 0 when none)
                                         "GBps": round(v[1] / (v[0] * 1e-3) / 1e9, 2) if v[0] > 0 else None}
                                     for k, v in kernels.items()}},
            "pipeline": {"ms_device": round(ms_dev, 4), "ms_pretok": round(avg("ms_pretok"), 4),
                         "ms_bpe_short": round(avg("ms_bpe_short"), 4), "ms_bpe_long": round(avg("ms_bpe_long"), 4),
                         "ms_emit": round(avg("ms_emit"), 4), "ms_call": round(avg("ms_total"), 4),
                         "B_alg": int(b_alg), "achieved_GBps": round(b_alg / (ms_dev * 1e-3) / 1e9, 2),
                         "pieces": int(P), "long_pieces": int(st["long_pieces"]),
                         "kernel_MBps": round(n_bytes / (ms_dev * 1e-3) / 1e6, 1),
                         "workspace_bytes": int(st["workspace_bytes"]),
                         "workspace_B_per_byte": round(st["workspace_bytes"] / max(1, n_bytes), 2)},
            "user_facing": uf,
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
