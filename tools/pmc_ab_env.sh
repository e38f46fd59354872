#!/bin/bash
# One SQ counter pass over tools/probe.py per environment setting (profiling helper):
#   bash tools/pmc_ab_env.sh OUTDIR CFG FIX "VAR=VAL ..." COUNTER,COUNTER,...
# (the setting is a shell assignment in front of rocprofv3, which passes it to the program)
out=$1; cfg=$2; fx=$3; sets=$4; ctrs=$5
ROOT=$(pwd)
mkdir -p "$out"
for st in $sets; do
  d="$ROOT/$out/pmc_${cfg}_${st//[^A-Za-z0-9]/_}"
  ( cd /tmp && export $st && timeout -s KILL 240 rocprofv3 --pmc $(echo "$ctrs" | tr , ' ') --output-format csv -d "$d" -o run -- \
      python3 "$ROOT/tools/probe.py" "$cfg" "$fx" 2 > "$d.log" 2>&1 ) || { echo "pmc pass failed: $st"; tail -5 "$d.log"; exit 1; }
  echo "## $st" | tee -a "$out/pmc_${cfg}.txt"
  python3 "$ROOT/tools/pmc_sum.py" "$d" | tee -a "$out/pmc_${cfg}.txt"
done
