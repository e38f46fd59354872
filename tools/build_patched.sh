#!/bin/bash
# Build libctok.so from the working tree with kernels.hip replaced by another file (A/B variants):
#   usage: bash tools/build_patched.sh KERNELS.hip OUT.so
set -e
K=$1; OUT=$2
T=$(mktemp -d /tmp/ctok_patched.XXXX)
mkdir -p "$T/complexity-tokenizer_amd/complexity_tokenizer"
cp -r include "$T/"
cp -r complexity-tokenizer_amd/csrc "$T/complexity-tokenizer_amd/"
rm -rf "$T/complexity-tokenizer_amd/csrc/build"
cp "$K" "$T/complexity-tokenizer_amd/csrc/kernels.hip"
make -C "$T/complexity-tokenizer_amd/csrc" -j8 ARCH=gfx950 > "$T/build.log" 2>&1 || { tail -20 "$T/build.log"; exit 1; }
cp "$T/complexity-tokenizer_amd/complexity_tokenizer/libctok.so" "$OUT"
rm -rf "$T"
echo "built $K -> $OUT"
