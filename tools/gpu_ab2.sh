#!/bin/bash
# GPU tests, then an A/B of two libraries (A = the working tree's libctok.so, B = another build) on C4 and C2.
#   usage: bash tools/gpu_ab2.sh TAG LIB_B[,VAR=VAL] [tests|notests|<pytest -k expression>] [c2]
set -e
TAG=${1:-ab}; B=$2; TESTS=${3:-tests}; C2=${4:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$TESTS" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
  tail -3 "$OUT/gpu_tests.log"
elif [ "$TESTS" != notests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "$TESTS" --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
  tail -3 "$OUT/gpu_tests.log"
fi
L=complexity-tokenizer_amd/complexity_tokenizer/libctok.so
bash tools/ab.sh $L $B > "$OUT/ab_c4.txt" 2>&1 || { tail -20 "$OUT/ab_c4.txt"; exit 1; }
cat "$OUT/ab_c4.txt"
if [ -n "$C2" ]; then
  bash tools/ab.sh $L $B --config c2 > "$OUT/ab_c2.txt" 2>&1 || { tail -20 "$OUT/ab_c2.txt"; exit 1; }
  cat "$OUT/ab_c2.txt"
fi
echo "gpu_ab2 $TAG done"
