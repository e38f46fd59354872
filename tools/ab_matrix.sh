#!/bin/bash
# A/B of environment arms on the kernel-only matrix leg (same GPU box, arms interleaved):
#   usage: bash tools/ab_matrix.sh CONFIGS REPS "ENV=VAL ..." "ENV=VAL ..." ...   ("-" = no env)
set -e
CONFIGS=$1; REPS=$2; shift 2
mkdir -p gpurun_out/abm
for i in $(seq 1 "$REPS"); do
  a=0
  for arm in "$@"; do
    envs=""; [ "$arm" != "-" ] && envs=$arm
    env $envs timeout -k 10 300 python -u tools/bench_matrix.py --configs "$CONFIGS" --kernel-only \
      --out gpurun_out/abm/arm${a}_$i.json > gpurun_out/abm/arm${a}_$i.log 2>&1 \
      || { tail -20 gpurun_out/abm/arm${a}_$i.log; exit 1; }
    echo "arm$a [$arm] rep $i:"; grep "kernel " gpurun_out/abm/arm${a}_$i.log
    a=$((a + 1))
  done
done
