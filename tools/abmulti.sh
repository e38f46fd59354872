#!/bin/bash
# Kernel-only probe A/B of environment settings over several configs (profiling helper):
#   bash tools/abmulti.sh OUTFILE "CFG:FIX CFG:FIX ..." "VAR=VAL VAR=VAL ..." [reps]
# Each config runs every setting (the first is usually the baseline, e.g. X=) in turn, `reps` rounds.
out=$1; cfgs=$2; sets=$3; reps=${4:-2}
for r in $(seq $reps); do
  for cf in $cfgs; do
    cfg=${cf%%:*}; fx=${cf#*:}
    for st in $sets; do
      env $st timeout -k 10 300 python -u tools/probe.py "$cfg" "$fx" 5 2>/dev/null | grep MB/s | sed "s|^|$st |" | tee -a "$out"
    done
  done
done
