#!/usr/bin/env python3
"""Build the synthetic tokenizer.json fixtures (no network: GPT-2 / Llama-3 files are not on disk).

The merge lists are learned offline with the HF `tokenizers` BpeTrainer on this repo's seeded
synthetic corpora (datagen/corpus.py), then re-laid-out in the shape of the real files:

  gpt2_50k     50,257 = 256 byte chars + 50,000 merges + <|endoftext|>; string-format merges
               ("a b"), "normalizer": null, ByteLevel(add_prefix_space=false)      (configs C1/C2/C4)
  llama3_128k  128,000 model.vocab + 256 added <|reserved_special_token_i|>; array-format merges;
               pre_tokenizer Sequence[Split(Llama-3 regex, Isolated), ByteLevel(use_regex=false)]
                                                                                    (config C3)
  multi_32k    32,000 vocab trained on the CJK + emoji + ASCII mixture              (config C5)
  llama3_tt_128k  llama3_128k with the merge list laid out as the tiktoken -> tokenizer.json
               conversion does for the real Llama-3 (every split of every token: 304k merges,
               several per token, not rank-monotone)                           (config C3, wide table)

Every merge is valid (both parts and their concatenation are in the vocab) and unique, so the
reference's rank/new_id quirk (src/bpe.rs:60-69) is inert on these files; in
llama3_tt_128k several merges make the same token, as in the real file (mod.rs:252-264 keeps them
all, each with its own rank).
Outputs: datagen/fixtures/<name>.json.gz.   Run: python datagen/build_tokenizers.py [names...]
"""
import gzip
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from datagen import corpus  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures")

LLAMA3_PATTERN = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*"
                  r"|\s*[\r\n]+|\s+(?!\S)|\s+")


def byte_chars():
    bs = list(range(0x21, 0x7F)) + list(range(0xA1, 0xAD)) + list(range(0xAE, 0x100))
    cs = list(bs)
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return [chr(c) for c in cs]  # in bytes_to_unicode order (GPT-2 ids 0..255)


def train_merges(texts, n_merges):
    from tokenizers import Tokenizer, models, pre_tokenizers, trainers
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
    tr = trainers.BpeTrainer(vocab_size=256 + n_merges, min_frequency=2, show_progress=False,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), special_tokens=[])
    tok.train_from_iterator(texts, tr)
    obj = json.loads(tok.to_str())
    merges = [tuple(m) if isinstance(m, list) else tuple(m.split(" ")) for m in obj["model"]["merges"]]
    assert len(merges) == n_merges, (len(merges), n_merges)
    return merges


def layout(merges, n_vocab_total=None):
    chars = byte_chars()
    vocab = {c: i for i, c in enumerate(chars)}
    for a, b in merges:
        assert a in vocab and b in vocab, (a, b)
        m = a + b
        assert m not in vocab, m
        vocab[m] = len(vocab)
    if n_vocab_total is not None:
        assert len(vocab) == n_vocab_total, (len(vocab), n_vocab_total)
    return vocab


def texts_of(text, off):
    return [t.decode("utf-8") for t in corpus.unpack(text, off)]


def build_gpt2():
    text, off = corpus.corpus_c2(250_000, seed=102)
    merges = train_merges(texts_of(text, off), 50_000)
    vocab = layout(merges, 50_256)
    vocab["<|endoftext|>"] = 50256
    return {
        "version": "1.0", "truncation": None, "padding": None,
        "added_tokens": [{"id": 50256, "content": "<|endoftext|>", "single_word": False, "lstrip": False,
                          "rstrip": False, "normalized": True, "special": True}],
        "normalizer": None,
        "pre_tokenizer": {"type": "ByteLevel", "add_prefix_space": False, "trim_offsets": True, "use_regex": True},
        "post_processor": {"type": "ByteLevel", "add_prefix_space": True, "trim_offsets": False, "use_regex": True},
        "decoder": {"type": "ByteLevel", "add_prefix_space": True, "trim_offsets": True, "use_regex": True},
        "model": {"type": "BPE", "dropout": None, "unk_token": None, "continuing_subword_prefix": "",
                  "end_of_word_suffix": "", "fuse_unk": False, "byte_fallback": False,
                  "vocab": vocab, "merges": [a + " " + b for a, b in merges]},
    }


def build_llama3():
    t3, o3 = corpus.corpus_c3(60_000, seed=103)
    t2, o2 = corpus.corpus_c2(300_000, seed=203)
    texts = texts_of(t3, o3) + texts_of(t2, o2)
    merges = train_merges(texts, 128_000 - 256)
    vocab = layout(merges, 128_000)
    added = [{"id": 128000 + i, "content": "<|reserved_special_token_%d|>" % i, "single_word": False,
              "lstrip": False, "rstrip": False, "normalized": False, "special": True} for i in range(256)]
    added[0]["content"], added[1]["content"] = "<|begin_of_text|>", "<|end_of_text|>"
    return {
        "version": "1.0", "truncation": None, "padding": None, "added_tokens": added,
        "normalizer": None,
        "pre_tokenizer": {"type": "Sequence", "pretokenizers": [
            {"type": "Split", "pattern": {"Regex": LLAMA3_PATTERN}, "behavior": "Isolated", "invert": False},
            {"type": "ByteLevel", "add_prefix_space": False, "trim_offsets": True, "use_regex": False}]},
        "post_processor": {"type": "ByteLevel", "add_prefix_space": True, "trim_offsets": False, "use_regex": True},
        "decoder": {"type": "ByteLevel", "add_prefix_space": True, "trim_offsets": True, "use_regex": True},
        "model": {"type": "BPE", "dropout": None, "unk_token": None, "continuing_subword_prefix": None,
                  "end_of_word_suffix": None, "fuse_unk": False, "byte_fallback": False, "ignore_merges": True,
                  "vocab": vocab, "merges": [[a, b] for a, b in merges]},
    }


def tiktoken_style_merges(vocab):
    """The merge list a tiktoken BPE file converts to (the layout of the real Llama-3
    tokenizer.json, ~280k merges for 128k tokens): for every token, in id (= tiktoken rank) order,
    every split into two vocab tokens, the splits ordered by their parts' ids; all merges sorted by
    the id of the token they make.  Several merges make the same token, so new ids are not strictly
    increasing in rank (the loader's rank-valued "wide" table), and a merge can consume a token that
    a later-ranked merge also makes (the table is not rank-monotone)."""
    merges = []
    for tok, rank in sorted(vocab.items(), key=lambda kv: kv[1]):
        if len(tok) == 1:
            continue
        local = [(tok[:i], tok[i:]) for i in range(1, len(tok)) if tok[:i] in vocab and tok[i:] in vocab]
        local.sort(key=lambda m: (vocab[m[0]], vocab[m[1]]))
        merges += local
    return merges  # (already in rank order: tokens were visited by id)


def build_llama3_tiktoken():
    """llama3_128k's vocab, added tokens and pre-tokenizer with tiktoken-style merges (304k)."""
    with gzip.open(os.path.join(OUT, "llama3_128k.json.gz"), "rb") as f:
        obj = json.loads(f.read())
    merges = tiktoken_style_merges(obj["model"]["vocab"])
    assert len(set(merges)) == len(merges)
    obj["model"]["merges"] = [[a, b] for a, b in merges]
    return obj


def build_multi():
    t5, o5 = corpus.corpus_c5(120_000, seed=105)
    merges = train_merges(texts_of(t5, o5), 32_000 - 256)
    vocab = layout(merges, 32_000)
    return {
        "version": "1.0", "truncation": None, "padding": None, "added_tokens": [],
        "normalizer": {"type": "NFC"},
        "pre_tokenizer": {"type": "ByteLevel", "add_prefix_space": False, "trim_offsets": True, "use_regex": True},
        "post_processor": None, "decoder": {"type": "ByteLevel"},
        "model": {"type": "BPE", "vocab": vocab, "merges": [a + " " + b for a, b in merges]},
    }


BUILDERS = {"gpt2_50k": build_gpt2, "llama3_128k": build_llama3, "multi_32k": build_multi,
            "llama3_tt_128k": build_llama3_tiktoken}


def main(names):
    os.makedirs(OUT, exist_ok=True)
    for name in names or list(BUILDERS):
        obj = BUILDERS[name]()
        path = os.path.join(OUT, name + ".json.gz")
        with gzip.GzipFile(path, "wb", mtime=0) as f:
            f.write(json.dumps(obj, ensure_ascii=False).encode("utf-8"))
        print("wrote", path, len(obj["model"]["vocab"]), "vocab", len(obj["model"]["merges"]), "merges")


def fixture_path(name: str, tmpdir: str) -> str:
    """Decompress datagen/fixtures/<name>.json.gz into tmpdir and return the tokenizer.json path."""
    src = os.path.join(OUT, name + ".json.gz")
    dst = os.path.join(tmpdir, name + ".json")
    if not os.path.exists(dst):
        with gzip.open(src, "rb") as f, open(dst, "wb") as g:
            g.write(f.read())
    return dst


if __name__ == "__main__":
    main(sys.argv[1:])
