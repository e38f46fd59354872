#!/bin/bash
# Alternating kernel-only probes (tools/probe.py) of two libraries on one box.
#   usage: bash tools/ab_probe.sh CFG FIX LIB_A LIB_B
set -e
for i in 1 2 3; do
  for L in $3 $4; do
    CTOK_LIB=$L timeout -k 10 200 python -u tools/probe.py $1 $2 5 2>/dev/null | grep MB/s | sed "s|^|$(basename $L) |"
  done
done
