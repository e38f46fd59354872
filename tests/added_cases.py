"""Tokenizers whose added tokens CAN match inside a pre-tokenized piece, and texts that put
them there.

The reference splits every byte-mapped word on its added tokens before BPE
(src/huggingface/mod.rs:566-610): the longest token whose first occurrence is at position 0
wins, otherwise the word is cut at the nearest first occurrence at position > 0
(find_next_added_token_in_word, :616-634); the single_word / lstrip / rstrip flags are checked
at that first occurrence only (find_added_token, :637-675), on byte-mapped chars.  Bracketed
specials such as "<|endoftext|>" never reach this code (the regex cuts them apart), so these
variants use plain letter / digit / punctuation tokens, tokens written in byte-mapped form
("Ġthe" = " the", "Ã©" = "e-acute"), overlapping tokens ("ab" / "abc") and every
flag combination.
"""
import copy
import random

G = "Ġ"  # GPT-2 char of the space byte

# (content, single_word, lstrip, rstrip)
VARIANTS = {
    # no flags: longest match at 0, nearest occurrence otherwise
    "plain": [("ing", 0, 0, 0), ("hello", 0, 0, 0), ("ll", 0, 0, 0), ("ab", 0, 0, 0), ("abc", 0, 0, 0),
              (G + "the", 0, 0, 0), ("Ã©", 0, 0, 0), ("12", 0, 0, 0), ("!!", 0, 0, 0),
              ("zz", 0, 0, 0)],
    # single_word: the byte-mapped neighbours must not be alphanumeric (G, the mapped space,
    # is a letter, so a token after an attached space fails)
    "single_word": [("ing", 1, 0, 0), ("ab", 1, 0, 0), ("abc", 0, 0, 0), ("ll", 1, 0, 0), ("hello", 0, 0, 0),
                    ("12", 1, 0, 0), ("!!", 1, 0, 0), ("Ã©", 1, 0, 0)],
    # lstrip / rstrip: byte-mapped chars are never White_Space, so they pass only at the edges
    "strip": [("ing", 0, 1, 0), ("ab", 0, 0, 1), ("abc", 0, 1, 1), ("ll", 0, 1, 0), ("hello", 0, 0, 1),
              ("12", 0, 1, 0), ("!!", 0, 0, 1), (G + "the", 0, 1, 0)],
    "all_flags": [("ing", 1, 1, 1), ("ab", 1, 1, 1), ("abc", 1, 1, 1), ("ll", 1, 1, 1), ("hello", 1, 1, 1),
                  ("e", 1, 1, 1)],
    # a mixed set with a one-letter token (it matches almost everywhere) and a duplicate content
    # (HashMap insert: the later entry's id and flags win)
    "mixed": [("a", 0, 0, 0), ("ing", 0, 0, 1), ("ab", 1, 0, 0), ("abc", 0, 1, 0), ("ll", 0, 0, 0),
              ("ll", 1, 0, 0), ("th", 0, 0, 0), ("the", 0, 0, 0), ("99", 0, 0, 0)],
}

FRAGS = ["ing", "hello", "ll", "ab", "abc", "the", "th", "e", "a", "b", "c", "x", "q", "12", "1", "9", "99",
         "!!", "!", "é", "zz", "oo", "Hello", "ING"]


def with_added(base_obj, variant, special=False):
    """base tokenizer.json object + the variant's added tokens (ids past the vocab)."""
    obj = copy.deepcopy(base_obj)
    nid = max(obj["model"]["vocab"].values()) + 1
    added = list(obj.get("added_tokens", []))
    for k, (content, sw, ls, rs) in enumerate(VARIANTS[variant]):
        added.append({"id": nid + k, "content": content, "single_word": bool(sw), "lstrip": bool(ls),
                      "rstrip": bool(rs), "normalized": False, "special": special})
    obj["added_tokens"] = added
    return obj


def _word(rng, n_frags):
    return "".join(rng.choice(FRAGS) for _ in range(n_frags))


def short_docs(n, seed):
    """Docs of words <= 32 bytes: tokens as prefix, middle, end of a word, twice in a word,
    after an attached space, after punctuation, next to digits."""
    rng = random.Random(seed)
    seps = [" ", " ", " ", "  ", "\n", ".", ", ", "'s ", "-", "\t"]
    docs = []
    for _ in range(n):
        k = rng.randint(0, 12)
        parts = []
        for _ in range(k):
            parts.append(_word(rng, rng.randint(1, 5)))
            parts.append(rng.choice(seps))
        docs.append("".join(parts))
    return docs


def long_piece_docs(seed, lengths=(33, 40, 63, 64, 65, 100, 257, 1000, 2047, 2048, 2049, 3000, 4096, 4097, 6000)):
    """Single letter runs (one piece each) of the given byte lengths built from the fragments:
    every added-token split implementation (<= 32 B thread per piece, LDS linked list up to
    2048 positions, global-memory list beyond) sees tokens at the start, inside and at the end."""
    rng = random.Random(seed)
    letters = [f for f in FRAGS if f.isalpha() and f.isascii()]
    docs = []
    for n in lengths:
        for variant in range(3):
            s = ""
            while len(s) < n:
                s += rng.choice(letters)
            s = s[:n]
            if variant == 1:
                s = "ing" + s[3:]
            elif variant == 2:
                s = s[:-5] + "hello"
            docs.append(s)
            docs.append(" " + s)  # attached space: the mapped G before the first letter
        docs.append("xab" + "é" + "ab" * (n // 2))  # first "ab" fails single_word, a later one would pass
        docs.append("!" * n)  # punctuation piece ("!!")
        docs.append("".join(rng.choice(["1", "12", "9", "99"]) for _ in range(n // 2)))  # digit piece
    return docs
