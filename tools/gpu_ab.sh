#!/bin/bash
# GPU tests, then an A/B of the current library against itself with an env switch on C4 and C2.
#   usage: bash tools/gpu_ab.sh TAG "VAR=VAL" [tests|notests]
set -e
TAG=${1:-ab}; ENVB=$2; TESTS=${3:-tests}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$TESTS" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
  tail -3 "$OUT/gpu_tests.log"
fi
L=complexity-tokenizer_amd/complexity_tokenizer/libctok.so
bash tools/ab.sh $L $L,$ENVB > "$OUT/ab_c4.txt" 2>&1 || { tail -20 "$OUT/ab_c4.txt"; exit 1; }
cat "$OUT/ab_c4.txt"
bash tools/ab.sh $L $L,$ENVB --config c2 > "$OUT/ab_c2.txt" 2>&1 || { tail -20 "$OUT/ab_c2.txt"; exit 1; }
cat "$OUT/ab_c2.txt"
echo "gpu_ab $TAG done"
