#!/bin/bash
# SQ counter pass (one rocprofv3 --pmc run per call) over a short bench: instruction mix, LDS and
# wait cycles per kernel.  usage: bash tools/pmc_sq.sh TAG CONFIG "COUNTERS" [VAR=VAL ...]
#   CONFIG: c4 | c2; COUNTERS: at most 8 SQ_* names (one pass); env VAR=VAL for the variant.
# Build the C4 corpus cache first (an unprofiled bench run): a --pmc run must not fork a pool.
set -e
TAG=$1; CFG=$2; CTRS=$3; shift 3
OUT=$(pwd)/gpurun_out/sq_$TAG
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp
env "$@" timeout -s KILL 120 rocprofv3 --pmc $CTRS \
  --output-format csv -d "$OUT" -o run -- python3 "$ROOT/bench.py" --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-parity --corpus-workers 1 \
  > "$OUT/log.txt" 2>&1 || { tail -20 "$OUT/log.txt"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ctok_dev::", "")
        agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    if any(s in k for s in ("short", "segment", "emit", "mid<true, 2")):
        print(k, {c: int(sum(x) / len(x)) for c, x in sorted(v.items())})
PY
