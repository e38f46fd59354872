#!/bin/bash
# A/B of two builds of libctok.so on the same GPU box: bench.py alternately with each library
# (CTOK_LIB), three times each, printing throughput and the per-kernel times.
#   usage: bash tools/ab.sh LIB_A[,VAR=VAL] LIB_B[,VAR=VAL] [bench args]
set -e
A=$1; B=$2; shift 2
mkdir -p gpurun_out/ab
for i in 1 2 3; do
  for v in A B; do
    spec=$A; [ $v = B ] && spec=$B
    lib=${spec%%,*}; envs=""; [ "$spec" != "$lib" ] && envs=${spec#*,}
    env CTOK_LIB=$lib $envs timeout -k 10 180 python -u bench.py --no-cpu-baseline --no-user-facing --steps 30 "$@" \
      > gpurun_out/ab/$v$i.json 2> gpurun_out/ab/$v$i.log
    python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ab/$v$i.json').read().strip().splitlines()[-1])
k=d['roofline']['kernels']; p=d['pipeline']
print('$v$i', d['value'], ' '.join('%s=%.4f'%(n,v['ms']) for n,v in k.items()), 'emit=%.4f dev=%.4f'%(p['ms_emit'],p['ms_device']), 'ws=%s' % p.get('workspace_B_per_byte'))"
  done
done
