#!/usr/bin/env python3
"""HBM traffic per kernel launch from rocprofv3 PMC passes (profiling helper, not product code).

Usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json [WORKLOAD]
  WORKLOAD: bench.py's config/docs of the profiled command (e.g. c4/10000000); bench.py uses
  the file's numbers only for that workload
  FETCH_DIR: output of `rocprofv3 --pmc FETCH_SIZE ...` (…_counter_collection.csv)
  WRITE_DIR: output of `rocprofv3 --pmc WRITE_SIZE ...`

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KiB per dispatch (TCC_EA0 read /
write requests x 64 B, memory side of the L2).  MI355X_MICROARCH.md: on gfx950 FETCH_SIZE
reports exactly half the bytes of a wide (16 B/lane) coalesced streaming read; the correction
applied here is x2 on FETCH_SIZE (the dominant reads of k_segment are 16 B/lane), WRITE_SIZE
as reported.  Other access widths are uncalibrated, so `hbm_bytes_per_launch` is an estimate
with that stated correction; the raw KiB values are kept beside it.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("void ", "").split("(")[0].replace("ctok_dev::", "")
    return re.sub(r"<(\d+), (true|false)>", r"<\1>", n)


def load(d, counter):
    vals = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] == counter:
                vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    fetch_dir, write_dir, out = sys.argv[1:4]
    workload = sys.argv[4] if len(sys.argv) > 4 else None
    f = load(fetch_dir, "FETCH_SIZE")
    w = load(write_dir, "WRITE_SIZE")
    import hashlib
    lib = os.environ.get("CTOK_LIB") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                     "complexity-tokenizer_amd", "complexity_tokenizer", "libctok.so")
    with open(lib, "rb") as fh:
        lib_sha = hashlib.sha256(fh.read()).hexdigest()
    res = {"unit": "bytes per launch", "fetch_correction": 2.0, "workload": workload,
           "lib_sha256": lib_sha,  # the profiled library: bench.py reports `traffic` only for this build
           "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB -> bytes",
           "fetch_kib": f, "write_kib": w, "hbm_bytes_per_launch": {}}
    for k in sorted(set(f) | set(w)):
        res["hbm_bytes_per_launch"][k] = int((2.0 * f.get(k, 0.0) + w.get(k, 0.0)) * 1024)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(json.dumps(res["hbm_bytes_per_launch"], indent=1))


if __name__ == "__main__":
    main()
