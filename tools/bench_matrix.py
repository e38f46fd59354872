#!/usr/bin/env python3
"""Measurement matrix of SURVEY.md section 8(d) on one MI355X (bench.py keeps the one-line
driver contract; this tool reports everything around it).

Per config (C1, C2, C3, C5 of BASELINE.json, C3 with the tiktoken-layout merge list (C3TT) and C5
with NFC-active text (C5-NFC); C4 is C2's generator sharded by the driver's 1/2/4/8-GPU bench runs):
  kernel    device-resident ctok_encode_batch_device, host clock around the call (median of
            >= 10 after 3 warm-ups) and HIP-event device time
  e2e       ctok_encode_batch from host numpy buffers: pinned-staging pipeline, H2D + kernels +
            D2H overlapped (median of 5 after 1 warm-up), also with 2 shards on one device
  python    Tokenizer.encode_batch(list[str]) -> list[list[int]] on the first <= 100k docs
  cpu       oracle/ctok_ref.c (faithful C restatement of the Rust reference, kind "port") on
            1 thread and on `threads` threads, bounded samples
  hf        HF `tokenizers` encode_batch on the same <= 100k docs if importable: an external
            native CPU datum with different pre-tokenizer semantics (not an oracle)
  parity    sha256(tok_off, ids) of the whole config vs tests/golden/digests.json
plus the device-to-device copy rate (a measured HBM stream peak) and the host CPU model.

    python tools/bench_matrix.py [--configs c1,c2,c3,c3tt,c5,c5nfc] [--out profiles/x.json] [--threads 16]
"""
import argparse
import hashlib
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "complexity-tokenizer_amd")]
# one OpenMP thread for torch / numpy (before they load): their pools spin after CPU work and take
# the cgroup's CPU share from the host-buffer pipeline's threads (see main)
os.environ["OMP_NUM_THREADS"] = "1"

import numpy as np  # noqa: E402


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def digest(ids, tok_off):
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(tok_off, dtype="<u8").tobytes())
    h.update(np.ascontiguousarray(ids, dtype="<u4").tobytes())
    return h.hexdigest()


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


CONFIGS = {  # name: (tokenizer fixture, datagen.corpus generator, description)
    "c1": ("gpt2_50k", "corpus_c1", "C1: 1k ASCII docs 1-64 B"),
    "c2": ("gpt2_50k", "corpus_c2", "C2: 1M ASCII docs 96-160 B"),
    "c3": ("llama3_128k", "corpus_c3", "C3: 100k docs 16 B-4 KiB, Llama-3-shaped 128k vocab"),
    "c3tt": ("llama3_tt_128k", "corpus_c3", "C3 with the tiktoken-style Llama-3 merge list (304k merges, several per "
             "token: rank-valued wide table, not rank-monotone)"),
    "c5": ("multi_32k", "corpus_c5", "C5: 1M multilingual docs 64-512 B (CJK + emoji + ASCII), 32k vocab"),
    "c5nfc": ("multi_32k", "corpus_c5nfc", "C5-NFC: C5 with NFC-active text in 3% of the docs (GPU NFC path)"),
}


def timed(fn, reps, warm):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return statistics.median(ts)


def cpu_rate(rc, text, off, threads, seconds):
    n_docs = len(off) - 1
    n0 = min(2000, n_docs)
    t = time.perf_counter()
    rc.encode_packed(text[: int(off[n0])], off[: n0 + 1], threads)
    rate = int(off[n0]) / max(time.perf_counter() - t, 1e-9)
    n = n_docs if int(off[-1]) / rate <= seconds else max(n0, int(np.searchsorted(off.astype(np.int64),
                                                                                   int(rate * seconds))))
    n = min(n, n_docs)
    t = time.perf_counter()
    rc.encode_packed(text[: int(off[n])], off[: n + 1], threads)
    dt = time.perf_counter() - t
    return {"MBps": round(int(off[n]) / dt / 1e6, 3), "threads": threads, "docs": int(n),
            "MB": round(int(off[n]) / 1e6, 2), "s": round(dt, 2)}


def run_config(name, args, torch, dev):
    from complexity_tokenizer import Tokenizer
    from datagen import corpus
    from datagen.build_tokenizers import fixture_path
    from oracle import ref_c

    tok_name, gen_name, desc = CONFIGS[name]
    gen = getattr(corpus, gen_name)
    tmp = "/tmp/ctok_matrix"
    os.makedirs(tmp, exist_ok=True)
    path = fixture_path(tok_name, tmp)
    t0 = time.time()
    if name == "c1":
        text, off = gen()
    else:  # the per-box corpus cache (tools/session.sh corpus:NAME builds it ahead)
        from datagen import cache
        key = {"c3tt": "C3"}.get(name, name.upper())
        text, off = cache.wait_load(cache.default_dir(), key)
    n_docs, n_bytes = len(off) - 1, int(off[-1])
    log("[matrix] %s: %d docs %.1f MB (corpus %.1fs)" % (name, n_docs, n_bytes / 1e6, time.time() - t0))
    tok = Tokenizer.from_file(path)
    tok.device = 0
    out = {"config": name, "workload": desc, "tokenizer": tok_name, "docs": n_docs, "bytes": n_bytes}

    # kernel: device-resident
    d_text = torch.from_numpy(np.concatenate([text, np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    cap = 3 * n_bytes + n_docs + 16
    d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
    d_tok = torch.empty(n_docs + 1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    box = {}

    def kstep():
        box["n"] = tok.encode_packed_device(d_text.data_ptr(), d_off.data_ptr(), n_docs, n_bytes, d_ids.data_ptr(), cap,
                                            d_tok.data_ptr(), stream=stream, timing=True)
        box["st"] = dict(tok.last_stats)

    reps = 10 if n_bytes > 1e6 else 50
    for _ in range(3):
        kstep()
    ts, devs = [], []
    for _ in range(reps):
        t = time.perf_counter()
        kstep()
        ts.append(time.perf_counter() - t)
        devs.append(box["st"]["ms_device"])
    ntok = box["n"]
    ids = d_ids[:ntok].cpu().numpy().view(np.uint32)
    toff = d_tok.cpu().numpy().view(np.uint64)
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json"))).get(name.upper())
    if name == "c1":
        g = np.load(os.path.join(ROOT, "tests", "golden", "c1_gpt2_50k.npz"))
        ok = np.array_equal(g["ids"], ids) and np.array_equal(g["tok_off"], toff)
        out["parity"] = "bit-exact vs ref_py golden ids (tests/golden/c1_gpt2_50k.npz)" if ok else "MISMATCH"
    elif gold and gold["docs"] == n_docs:
        ok = digest(ids, toff) == gold["sha256"]
        out["parity"] = ("bit-exact: sha256 of all %d docs == golden" % n_docs) if ok else "MISMATCH"
    else:
        out["parity"] = "no golden digest"
    st = box["st"]
    med = statistics.median(ts)
    out["tokens"] = int(ntok)
    out["kernel"] = {"MBps": round(n_bytes / med / 1e6, 1), "ms_call": round(med * 1e3, 3),
                     "ms_device": round(statistics.median(devs), 3),
                     "MBps_device": round(n_bytes / (statistics.median(devs) * 1e-3) / 1e6, 1),
                     "ms_segment": round(st["ms_segment"], 4), "ms_bpe_short": round(st["ms_bpe_short"], 4),
                     "ms_bpe_le16": round(st["ms_bpe_lo"], 4), "ms_bpe_17_32": round(st["ms_bpe_hi"], 4),
                     "ms_bpe_33_64_main": round(st["ms_bpe_med"], 4),
                     "class_bytes": st["class_bytes"],
                     "class_ids": st["class_ids"],
                     "ms_bpe_long": round(st["ms_bpe_long"], 4), "ms_emit": round(st["ms_emit"], 4),
                     "pieces": int(st["pieces"]), "long_pieces": int(st["long_pieces"])}
    del d_text, d_off, d_ids, d_tok
    torch.cuda.empty_cache()
    if args.kernel_only:
        log("[matrix] %s kernel %.0f MB/s (device %.3f ms, long %.3f ms), %s" % (
            name, out["kernel"]["MBps"], out["kernel"]["ms_device"], out["kernel"]["ms_bpe_long"], out["parity"]))
        return out

    # e2e: host buffers through the pinned pipeline, the C ABI with caller-owned output buffers
    # reused across calls (ctok_encode_batch), as a C / Rust caller holds them; "e2e_numpy" is
    # Tokenizer.encode_packed, which allocates fresh output arrays per call (their page faults,
    # and the munmap of the previous call's arrays, are part of it)
    import ctypes
    from complexity_tokenizer import _native as _n
    res = {}
    cap_ids = n_bytes + n_docs + 16
    o_ids = np.zeros(cap_ids, dtype=np.uint32)
    o_off = np.zeros(n_docs + 1, dtype=np.uint64)
    for label, devs_, chunk in (("e2e", None, 0), ("e2e_2shards", [0, 0], 0), ("e2e_chunk8", None, 8),
                                ("e2e_numpy", None, 0)):
        tok.devices, tok.chunk_mb = devs_, chunk

        def estep():
            if label == "e2e_numpy":
                res["r"] = tok.encode_packed(text, off)
                return
            ex = tok._host_exec(False)
            rc = _n.lib.ctok_encode_batch(tok._h, text.ctypes.data, off.ctypes.data, n_docs, o_ids.ctypes.data,
                                          cap_ids, o_off.ctypes.data, ctypes.byref(ex), None)
            assert rc == 0, _n.last_error()
            res["r"] = (o_ids[: int(o_off[-1])], o_off)

        # (timed without per-call event timing: its synchronous event reads serialise the
        # chunk pipeline; one more call collects the H2D / D2H stats)
        med = timed(estep, 5 if n_bytes > 1e6 else 20, 1)
        eids, eoff = res["r"]
        same = np.array_equal(eids, ids) and np.array_equal(eoff, toff)
        tok.encode_packed(text, off, timing=True)
        st = tok.last_stats
        out[label] = {"MBps": round(n_bytes / med / 1e6, 1), "ms": round(med * 1e3, 2),
                      "ms_h2d_first_chunk": round(st["ms_h2d"], 3), "ms_d2h_last_chunk": round(st["ms_d2h"], 3),
                      "same_as_kernel_path": bool(same)}
    tok.devices, tok.chunk_mb = None, 0

    # python-level list[str] -> list[list[int]]
    n_py = min(n_docs, args.py_docs)
    docs = [d.decode() for d in corpus.unpack(text[: int(off[n_py])], off[: n_py + 1])]
    py_bytes = int(off[n_py])
    res_py = {}

    def pstep():
        res_py["r"] = tok.encode_batch(docs)

    med = timed(pstep, 3, 1)
    exp = [ids[toff[i]:toff[i + 1]].tolist() for i in range(min(n_py, 1000))]
    out["python"] = {"MBps": round(py_bytes / med / 1e6, 2), "docs": n_py, "ms": round(med * 1e3, 1),
                     "same_as_kernel_path": res_py["r"][: len(exp)] == exp}

    # CPU baselines (faithful C port of the reference)
    with open(path) as f:
        rc = ref_c.RefC(json.load(f))
    out["cpu_port_1t"] = cpu_rate(rc, text, off, 1, args.cpu_seconds)
    out["cpu_port_nt"] = cpu_rate(rc, text, off, args.threads, args.cpu_seconds)

    # external datum: HF tokenizers (different pre-tokenizer semantics, not an oracle)
    try:
        import tokenizers
        hf = tokenizers.Tokenizer.from_file(path)
        hdocs = docs[: min(len(docs), 100_000)]
        hb = sum(len(d.encode()) for d in hdocs)
        med = timed(lambda: hf.encode_batch(hdocs), 2, 1)
        out["hf_tokenizers"] = {"MBps": round(hb / med / 1e6, 2), "docs": len(hdocs),
                                "threads": os.environ.get("RAYON_NUM_THREADS", "default"),
                                "version": tokenizers.__version__,
                                "note": "external native CPU datum, different pre-tokenizer semantics"}
    except Exception as e:  # noqa: BLE001 -- optional datum
        out["hf_tokenizers"] = {"error": repr(e)[:200]}
    log("[matrix] %s done: kernel %.0f MB/s, e2e %.0f MB/s, python %.1f MB/s, cpu %.1f/%.1f MB/s, %s" % (
        name, out["kernel"]["MBps"], out["e2e"]["MBps"], out["python"]["MBps"], out["cpu_port_1t"]["MBps"],
        out["cpu_port_nt"]["MBps"], out["parity"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1,c2,c3,c3tt,c5,c5nfc")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "matrix.json"))
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=4.0)
    ap.add_argument("--py-docs", type=int, default=100_000)
    ap.add_argument("--kernel-only", action="store_true", help="device-resident leg only (A/B runs)")
    args = ap.parse_args()
    os.environ.setdefault("RAYON_NUM_THREADS", str(args.threads))
    import torch
    # torch is here only for device buffers: its intra-op CPU pool (OMP_NUM_THREADS = 16 on the
    # box) spins after CPU tensor ops and takes the cgroup's CPU share from the host-buffer
    # pipeline's widening threads and from the Python leg (C2 E2E 20.7 vs 24.3 GB/s, Python
    # 170 vs 364 MB/s, profiles/r03/v25_matrix_omp.txt); a tokenizer-only process has no such pool
    torch.set_num_threads(1)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # measured HBM stream peak: device-to-device copy of 2 GiB (reads + writes)
    a = torch.empty(2 << 30, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    copy_gbps = 2 * a.numel() * 10 / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    torch.cuda.empty_cache()
    rows = []
    meta = {"gpu": torch.cuda.get_device_name(0), "cpu_model": cpu_model(), "cpu_threads_used": args.threads,
            "torch_intraop_threads": torch.get_num_threads(),
            "d2d_copy_GBps": round(copy_gbps, 1), "hbm_spec_GBps": 8000.0}
    log("[matrix] meta", meta)
    for c in args.configs.split(","):
        rows.append(run_config(c.strip(), args, torch, dev))
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        json.dump({"meta": meta, "rows": rows}, open(args.out, "w"), indent=1)
    print(json.dumps({"meta": meta, "rows": rows}))


if __name__ == "__main__":
    main()
