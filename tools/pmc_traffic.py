#!/usr/bin/env python3
"""HBM traffic per kernel launch from rocprofv3 PMC passes (profiling helper, not product code).

Usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json [WORKLOAD]
  WORKLOAD: bench.py's config/docs of the profiled command (e.g. c4/10000000); bench.py uses
  the file's numbers only for that workload
  FETCH_DIR: output of `rocprofv3 --pmc FETCH_SIZE ...` (…_counter_collection.csv)
  WRITE_DIR: output of `rocprofv3 --pmc WRITE_SIZE ...`

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KiB per dispatch (TCC_EA0 read /
write requests, memory side of the L2).  Calibrated on known byte counts in this path's own access
shapes (tools/fetch_calib.hip, tools/pmc_calib.sh -> profiles/r06/fetch_calibration.txt): every L2
read request moves a 128-B line and is tallied at 64 B -- known bytes / FETCH_SIZE = 2.00 for 16-B
streaming loads, 2.00 for 4-B gathers of one dword per line, 1.97 for two dwords per line (one
request per line), 1.92 for the merge passes' text-word loads, 56 B tallied per 8-B probe of a
32 MiB table (0.875 requests: L2 misses served by the Infinity Cache, which FETCH counts);
WRITE_SIZE is exact for 16-B and consecutive 4-B stores and tallies 32 B per scattered 4-B store
(one 32-B write request each).  So `hbm_bytes_per_launch` = 2 x FETCH + WRITE is the bytes moved
beyond the L2 (Infinity-Cache hits included: an upper bound of the HBM bytes); the raw KiB values
are kept beside it.
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
           "calibration": "profiles/r06/fetch_calibration.txt",
           "note": "FETCH_SIZE x2 (calibrated: 128-B read requests tallied at 64 B) + WRITE_SIZE (exact request "
                   "bytes), KiB -> bytes; bytes moved beyond the L2, Infinity-Cache hits included",
           "fetch_kib": f, "write_kib": w, "hbm_bytes_per_launch": {}}
    for k in sorted(set(f) | set(w)):
        res["hbm_bytes_per_launch"][k] = int((2.0 * f.get(k, 0.0) + w.get(k, 0.0)) * 1024)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(json.dumps(res["hbm_bytes_per_launch"], indent=1))


if __name__ == "__main__":
    main()
