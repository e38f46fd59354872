#!/bin/bash
# A/B of host-table knobs on one library (one box): bench.py on C2, alternating the two arms.
L=complexity-tokenizer_amd/complexity_tokenizer/libctok.so
bash tools/ab.sh "$L,${1:-CTOK_MERGE16_SLACK=32}" "$L,${2:-CTOK_MERGE16_SLACK=128}" --config c2
