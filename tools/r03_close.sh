#!/bin/bash
# Round-3 closing session on one MI355X: the closing measurements of tools/r03_final.sh (GPU
# tests, bench C4 + C2, kernel trace, PMC traffic), an A/B of the working tree's library against
# abl/head.so on C5 (tools/ab_probe.sh), then the config matrix.  First failure ends it.
set -e
export TAG=${TAG:-r03_close}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/r03_final.sh tests
bash tools/r03_final.sh bench
bash tools/r03_final.sh prof
if [ -f abl/head.so ]; then
  bash tools/ab_probe.sh c5 multi_32k abl/head.so complexity-tokenizer_amd/complexity_tokenizer/libctok.so > "$OUT/ab_c5.txt" 2>&1
  cat "$OUT/ab_c5.txt"
fi
bash tools/r03_final.sh matrix
echo "r03_close done"
