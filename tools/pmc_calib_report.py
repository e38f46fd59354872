#!/usr/bin/env python3
"""Report of tools/pmc_calib.sh (profiling helper): per calibration kernel, FETCH_SIZE and the L2
read requests by size against the kernel's known bytes and accesses (tools/fetch_calib.hip)."""
import collections
import csv
import glob
import json
import os
import re
import sys

out = sys.argv[1]


def per_kernel(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k].add(r["Dispatch_Id"])
    return {k: {c: v / len(n[k]) for c, v in acc[k].items()} for k in acc}


meta = None
for line in open(os.path.join(out, "calib_fetch.log")):
    if line.startswith("{"):
        meta = json.loads(line)
fe, rq = per_kernel(os.path.join(out, "calib_fetch")), per_kernel(os.path.join(out, "calib_req"))
wr, wq = per_kernel(os.path.join(out, "calib_write")), per_kernel(os.path.join(out, "calib_wreq"))
known = {  # kernel: (known bytes the kernel touches, accesses, what)
    "k_stream16": (meta["stream16_bytes"], meta["stream16_bytes"] / 16, "16-B coalesced streaming loads, 2 GiB"),
    "k_gather_line": (128 * meta["gather_lines"], meta["gather_lines"], "one 4-B load per 128-B line, every line of 2 GiB once"),
    "k_gather_half": (128 * meta["gather_lines"], meta["gather_half_loads"], "4-B loads at +0 and +64 of every line of 2 GiB"),
    "k_gather_tab8": (None, meta["tab8_probes"], "8-B loads at random slots of a 32 MiB table (Infinity-Cache resident)"),
    "k_text_words": (meta["text_span_bytes"], meta["text_pieces"], "5 dwords per lane at piece starts ~12 B apart, 1 GiB"),
}
print("# FETCH_SIZE calibration (tools/fetch_calib.hip; rocprofv3 --pmc, one pass FETCH_SIZE, one pass request counts)")
print("# FETCH_SIZE = (BUBBLE*128 + (RDREQ - BUBBLE - RDREQ_32B)*64 + RDREQ_32B*32) bytes; per launch")
for k, (kb, acc, what) in known.items():
    kk = next((x for x in fe if x.endswith(k)), None)
    if kk is None:
        continue
    f = fe[kk].get("FETCH_SIZE", 0.0) * 1024  # (rocprofv3 reports KB)
    r = rq.get(kk, {})
    req, r32, bub, dram = (r.get("TCC_EA0_RDREQ_sum", 0), r.get("TCC_EA0_RDREQ_32B_sum", 0), r.get("TCC_BUBBLE_sum", 0),
                           r.get("TCC_EA0_RDREQ_DRAM_sum", 0))
    line = "%-14s %-70s FETCH %.4g B" % (k, what, f)
    if kb:
        line += "  known %.4g B  known/FETCH %.3f" % (kb, kb / f if f else float("nan"))
    line += "  FETCH/access %.2f B  requests/access %.3f (32B %.3g, bubble %.3g, dram %.3g)" % (
        f / acc, req / acc, r32, bub, dram)
    print(line)

print("# WRITE_SIZE = ((WRREQ - WRREQ_64B)*32 + WRREQ_64B*64) bytes; per launch")
wknown = {
    "k_store16": (meta["store16_bytes"], meta["store16_bytes"] / 16, "16-B coalesced streaming stores, 1 GiB"),
    "k_store_line4": (4 * meta["store_lines"], meta["store_lines"], "one 4-B store per 128-B line, every line of 2 GiB once"),
    "k_store_dense4": (meta["store_dense4_bytes"], meta["store_dense4_bytes"] / 4, "4-B stores, consecutive lanes -> consecutive dwords, 1 GiB"),
}
for k, (kb, acc, what) in wknown.items():
    kk = next((x for x in wr if x.endswith(k)), None)
    if kk is None:
        continue
    f = wr[kk].get("WRITE_SIZE", 0.0) * 1024
    r = wq.get(kk, {})
    req, r64, dram = r.get("TCC_EA0_WRREQ_sum", 0), r.get("TCC_EA0_WRREQ_64B_sum", 0), r.get("TCC_EA0_WRREQ_DRAM_sum", 0)
    print("%-14s %-70s WRITE %.4g B  known %.4g B  known/WRITE %.3f  WRITE/store %.2f B  requests/store %.3f (64B %.3g, dram %.3g)"
          % (k, what, f, kb, kb / f if f else float("nan"), f / acc, req / acc, r64, dram))
