#!/bin/bash
# Build libctok.so from a git revision's sources (for A/B runs against the working tree):
#   usage: bash tools/build_variant.sh REV OUT.so
# The revision's include/ and complexity-tokenizer_amd/csrc/ are exported to a scratch tree and
# built there with the same Makefile; the library is copied to OUT.so.
set -e
REV=$1; OUT=$2
T=$(mktemp -d /tmp/ctok_variant.XXXX)
git archive "$REV" include complexity-tokenizer_amd/csrc | tar -x -C "$T"
mkdir -p "$T/complexity-tokenizer_amd/complexity_tokenizer"
make -C "$T/complexity-tokenizer_amd/csrc" -j8 ARCH=gfx950 > "$T/build.log" 2>&1 || { tail -20 "$T/build.log"; exit 1; }
cp "$T/complexity-tokenizer_amd/complexity_tokenizer/libctok.so" "$OUT"
rm -rf "$T"
echo "built $REV -> $OUT"
