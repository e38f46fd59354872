#!/bin/bash
# Build libctok.so from a git revision's sources (for A/B runs against the working tree):
#   usage: bash tools/build_variant.sh REV OUT.so [-DNAME=VALUE ...]
# REV "worktree" takes the working tree's sources.  The sources are copied to a scratch tree and
# built there with the same Makefile (extra arguments are added to the compile flags, e.g. the
# CTOK_* compile-time knobs of kernels.hip); the library is copied to OUT.so.
set -e
REV=$1; OUT=$2; shift 2
DEFS="$*"
T=$(mktemp -d /tmp/ctok_variant.XXXX)
if [ "$REV" = worktree ]; then
  mkdir -p "$T/complexity-tokenizer_amd"
  cp -r include "$T/"
  cp -r complexity-tokenizer_amd/csrc "$T/complexity-tokenizer_amd/"
  rm -rf "$T/complexity-tokenizer_amd/csrc/build"
else
  git archive "$REV" include complexity-tokenizer_amd/csrc | tar -x -C "$T"
fi
mkdir -p "$T/complexity-tokenizer_amd/complexity_tokenizer"
make -C "$T/complexity-tokenizer_amd/csrc" -j8 ARCH=gfx950 CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function $DEFS" \
  ../complexity_tokenizer/libctok.so > "$T/build.log" 2>&1 || { tail -20 "$T/build.log"; exit 1; }
cp "$T/complexity-tokenizer_amd/complexity_tokenizer/libctok.so" "$OUT"
rm -rf "$T"
echo "built $REV $DEFS -> $OUT"
