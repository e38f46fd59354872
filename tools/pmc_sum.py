#!/usr/bin/env python3
"""Per-kernel sums of a rocprofv3 --pmc pass (profiling helper, not product code):
usage pmc_sum.py DIR -- prints, for each kernel, the launch count and every counter summed over
its launches and divided by the launch count (so: per launch)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
if not files:
    sys.exit("no counter_collection.csv under %s" % d)
acc = collections.defaultdict(lambda: collections.defaultdict(float))
launches = collections.defaultdict(set)
for f in files:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("ctok_dev::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        launches[k].add(r["Dispatch_Id"])
for k in sorted(acc, key=lambda k: -max(acc[k].values())):
    n = len(launches[k])
    print("%-40s n=%d  %s" % (k[:40], n, "  ".join("%s=%.4g" % (c, v / n) for c, v in sorted(acc[k].items()))))
