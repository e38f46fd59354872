#!/bin/bash
# One GPU-box iteration (run through gpurun from the repo root): the GPU tests, then an optional
# step.  usage: bash tools/gpu_iter.sh TAG [ab|matrix|none]
set -e
TAG=${1:-it}; STEP=${2:-none}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -3 "$OUT/gpu_tests.log"
L=complexity-tokenizer_amd/complexity_tokenizer/libctok.so
if [ "$STEP" = ab ]; then bash tools/ab.sh $L $L,CTOK_FORCE_WIDE_SLOTS=1 --config c2; fi
if [ "$STEP" = matrix ]; then
  timeout -k 10 400 python -u tools/bench_matrix.py --configs c1,c2,c3,c5 --out "$OUT/matrix.json" > "$OUT/matrix.log" 2>&1 || { tail -30 "$OUT/matrix.log"; exit 1; }
  tail -25 "$OUT/matrix.log"
fi
echo "gpu_iter $TAG done"
