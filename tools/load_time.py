"""Loader time per fixture tokenizer: Tokenizer.from_file wall time,
median of 5, with the per-phase breakdown of the last load (CTOK_LOAD_TIMING)."""
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "complexity-tokenizer_amd"))

from datagen.build_tokenizers import fixture_path  # noqa: E402
from complexity_tokenizer import Tokenizer  # noqa: E402


def main():
    d = tempfile.mkdtemp()
    out = {}
    for name in ("gpt2_50k", "multi_32k", "llama3_128k", "llama3_tt_128k"):
        p = fixture_path(name, d)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            Tokenizer.from_file(p)
            ts.append(time.perf_counter() - t0)
        obj = json.load(open(p))
        code = ("import sys; sys.path.insert(0, %r); from complexity_tokenizer import Tokenizer; "
                "Tokenizer.from_file(%r)" % (os.path.join(ROOT, "complexity-tokenizer_amd"), p))
        env = dict(os.environ, CTOK_LOAD_TIMING="1")
        phases = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True).stderr
        out[name] = {"vocab": len(obj["model"]["vocab"]), "merges": len(obj["model"]["merges"]),
                     "load_s_median": round(statistics.median(ts), 4),
                     "phases_ms": {ln.split()[2]: float(ln.split()[3]) for ln in phases.splitlines()
                                   if ln.startswith("[ctok load]")},
                     "host_cpus": os.cpu_count()}
        print(name, out[name], flush=True)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
