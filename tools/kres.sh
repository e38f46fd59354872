#!/bin/bash
# VGPRs / scratch / occupancy per kernel of a HIP source (gfx950), from the compiler's
# kernel-resource-usage remarks.  usage: tools/kres.sh [file.hip] [name-regex]
F=${1:-complexity-tokenizer_amd/csrc/kernels.hip}
PAT=${2:-.}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c "$F" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass.*//' |
awk '/^Function Name/{n=$3} /^VGPRs:/{v=$2} /^ScratchSize/{sc=$NF} /^Occupancy/{print n, "vgpr=" v, "scratch=" sc, "occ=" $NF}' |
c++filt | grep -E "$PAT"
