#!/bin/bash
# SQ counter pass (one rocprofv3 --pmc run per variant) over a short C2 bench: instruction mix and
# wait cycles per kernel.  usage: bash tools/pmc_sq.sh TAG [VAR=VAL ...]  (env for the variant)
set -e
TAG=$1; shift
OUT=$(pwd)/gpurun_out/sq_$TAG
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp
env "$@" timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU \
  --output-format csv -d "$OUT" -o run -- python3 "$ROOT/bench.py" --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-parity \
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
