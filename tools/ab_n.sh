#!/bin/bash
# A/B/C/... of several builds of libctok.so on one GPU box: bench.py round-robin over the
# libraries (CTOK_LIB), three rounds, printing throughput and the per-kernel times.
#   usage: bash tools/ab_n.sh TAG LIB1[,VAR=VAL] LIB2[,VAR=VAL] ... [-- bench args]
set -e
TAG=$1; shift
specs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do specs+=("$1"); shift; done
[ "$1" = "--" ] && shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for i in 1 2 3; do
  for k in "${!specs[@]}"; do
    spec=${specs[$k]}
    lib=${spec%%,*}; envs=""; [ "$spec" != "$lib" ] && envs=${spec#*,}
    env CTOK_LIB=$lib $envs timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 30 "$@" \
      > "$OUT/v$k.$i.json" 2> "$OUT/v$k.$i.log"
    python3 -c "
import json
d=json.loads(open('$OUT/v$k.$i.json').read().strip().splitlines()[-1])
k=d['roofline']['kernels']; p=d['pipeline']
print('v$k.$i', '$(basename $lib)', d['value'], ' '.join('%s=%.4f'%(n,v['ms']) for n,v in k.items()), 'dev=%.4f'%p['ms_device'], 'ws=%s' % p.get('workspace_B_per_byte'), str(d.get('parity'))[:24])" | tee -a "$OUT/ab.txt"
  done
done
