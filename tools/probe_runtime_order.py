"""Probe: HIP runtime initialisation order between torch (its bundled HIP runtime) and
libctok.so (/opt/rocm HIP runtime) in one process.  Usage: python tools/probe_runtime_order.py MODE"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "complexity-tokenizer_amd")]
mode = sys.argv[1]
if os.environ.get("CTOK_FIRST"):
    import complexity_tokenizer as ct  # noqa: E402
    import torch  # noqa: E402
else:
    import torch  # noqa: E402
    import complexity_tokenizer as ct  # noqa: E402


def ctok():
    print(mode, "ctok devices", ct.device_count(), flush=True)


def th(what):
    try:
        if what == "count":
            print(mode, "torch count", torch.cuda.device_count(), flush=True)
        elif what == "init":
            torch.cuda.init()
            print(mode, "torch init ok", flush=True)
        elif what == "alloc":
            x = torch.zeros(4, device="cuda:0")
            print(mode, "torch alloc ok", float(x.sum()), flush=True)
    except Exception as e:  # noqa: BLE001
        print(mode, "torch", what, "FAILED", e, flush=True)


for step in mode.split(","):
    if step == "ctok":
        ctok()
    else:
        th(step)
