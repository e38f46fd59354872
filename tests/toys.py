"""Small hand-built tokenizer.json objects for edge-case tests (shared by CPU and GPU tests)."""
import json
import random


def byte_chars():
    bs = list(range(0x21, 0x7F)) + list(range(0xA1, 0xAD)) + list(range(0xAE, 0x100))
    cs = list(bs)
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return [chr(c) for c in cs]


def byte_map():
    """The GPT-2 char of every byte, indexed by byte (src/pretokenizers.rs:130-153); byte_chars()
    lists the same chars in the table's own order (printable bytes first)."""
    bs = list(range(0x21, 0x7F)) + list(range(0xA1, 0xAD)) + list(range(0xAE, 0x100))
    m = dict(zip(bs + [x for x in range(256) if x not in bs], byte_chars()))
    return [m[b] for b in range(256)]


def byte_char(b):
    return byte_map()[b]


def tok_json(vocab, merges, added=(), normalizer=None, pre_tokenizer=None, merges_as_arrays=False):
    obj = {"version": "1.0", "added_tokens": list(added), "normalizer": normalizer,
           "pre_tokenizer": pre_tokenizer if pre_tokenizer is not None else
           {"type": "ByteLevel", "add_prefix_space": False, "trim_offsets": True, "use_regex": True},
           "post_processor": None, "decoder": None,
           "model": {"type": "BPE", "vocab": vocab,
                     "merges": [[a, b] for a, b in merges] if merges_as_arrays else ["%s %s" % m for m in merges]}}
    return obj


def hello_kat():
    """reference src/bpe.rs:219-250 (toy vocab, lowest rank first) as a tokenizer.json."""
    vocab = {"h": 0, "e": 1, "l": 2, "o": 3, "he": 4, "ll": 5, "hel": 6, "hell": 7, "hello": 8, "lo": 9, "llo": 10}
    merges = [("h", "e"), ("he", "l"), ("hel", "l"), ("hell", "o"), ("l", "l"), ("l", "o"), ("l", "lo")]
    return tok_json(vocab, merges)


def loader_kat():
    """reference src/huggingface/mod.rs:1566-1592."""
    return {"version": "1.0", "model": {"type": "BPE", "vocab": {"h": 0, "e": 1, "l": 2, "o": 3, " ": 4, "w": 5,
                                                                  "r": 6, "d": 7}, "merges": []},
            "added_tokens": []}


def derived(base_obj, mutate):
    obj = json.loads(json.dumps(base_obj))
    mutate(obj)
    return obj


def shuffled_merges(base_obj, seed):
    """Same vocab, merge list permuted: valid merges with non-monotone ranks (improper table)."""
    def m(o):
        ms = list(o["model"]["merges"])
        random.Random(seed).shuffle(ms)
        o["model"]["merges"] = ms
    return derived(base_obj, m)


def with_invalid_merge_in_front(base_obj):
    """One merge whose parts are not in the vocab, in front: every valid merge's rank shifts by one
    (src/bpe.rs:60-69), so a merge's new id is the previous merge's and the last valid merge panics
    when used (src/bpe.rs:141); tokens then need not spell their strings (window rounds off)."""
    def m(o):
        o["model"]["merges"] = ["zzq0 qqz0"] + list(o["model"]["merges"])
    return derived(base_obj, m)


def with_invalid_merges(base_obj, seed, n_bad=50, tail_only=False):
    """Insert merges whose parts are not in the vocab: shifts BpeTokenizer.merges indices
    (reference src/bpe.rs:60-69 quirk); ranks past the valid list make lookups panic."""
    def m(o):
        ms = list(o["model"]["merges"])
        rng = random.Random(seed)
        for k in range(n_bad):
            pos = len(ms) if tail_only else rng.randrange(len(ms) + 1)
            ms.insert(pos, "zz%dq qq%dz" % (k, k))
        o["model"]["merges"] = ms
    return derived(base_obj, m)


def eager_cascade():
    """A table where applying every site of a merge at once differs from the sequential loop:
    ("ab", "a") ranks before ("a", "b"), so after the first "a b" of "abab" merges the new pair
    ("ab", "a") is the minimum, and it takes the next site's "a" (sequential: [aba, b]; every
    site at once: [ab, ab]).  Also "b a" and the byte merges of "c" runs, so pieces mix cascading
    and ordinary rounds."""
    chars = byte_chars()
    vocab = {c: i for i, c in enumerate(chars)}
    for t in ("ab", "aba", "ba", "cc", "cccc", "abab", "abc"):
        vocab[t] = len(vocab)
    merges = [("ab", "a"), ("a", "b"), ("b", "a"), ("c", "c"), ("cc", "cc"), ("ab", "ab"), ("ab", "c")]
    return tok_json(vocab, merges)


def random_proper(seed, alphabet="abc", n_merges=80, max_len=24):
    """A random rank-monotone table over the bytes of a few letters (multi-byte chars: their UTF-8
    bytes, merged in any grouping) (every merge's token exists before any merge
    consumes it is ranked, and no token is produced after one consuming it): the tables for which
    the segmented tier's window rounds apply (kernels.hip bpe_wave_seg, Tables::window).  Long
    tokens make wide windows; the whole byte alphabet is in the vocab."""
    rng = random.Random(seed)
    chars = byte_chars()
    vocab = {c: i for i, c in enumerate(chars)}
    bm = byte_map()
    toks = [bm[b] for b in dict.fromkeys(alphabet.encode())]  # the chars of the alphabet's bytes
    merges, seen, consumed = [], set(), set()
    tries = 0
    while len(merges) < n_merges and tries < 50 * n_merges:
        tries += 1
        # bias towards recent (longer) tokens so that windows get wide
        x = toks[min(len(toks) - 1, int(rng.expovariate(0.15) if rng.random() < 0.5 else rng.randrange(len(toks))))]
        y = rng.choice(toks) if rng.random() < 0.7 else toks[-1 - rng.randrange(min(4, len(toks)))]
        z = x + y
        if len(z) > max_len or (x, y) in seen or (z in vocab and z in consumed):
            continue
        seen.add((x, y))
        merges.append((x, y))
        consumed.update((x, y))
        if z not in vocab:
            vocab[z] = len(vocab)
            toks.append(z)
    return tok_json(vocab, merges)


def random_proper_from_text(seed, sample: bytes, n_merges=150, max_len=24):
    """A random rank-monotone table whose merges join pairs that occur in `sample` (bytes): like a
    BPE training run that picks a random adjacent pair of the current tokenisation instead of the
    most frequent one.  For multi-byte alphabets, where random byte pairs rarely occur in text."""
    rng = random.Random(seed)
    chars = byte_chars()
    vocab = {c: i for i, c in enumerate(chars)}
    bm = byte_map()
    seq = [bm[b] for b in sample]
    merges, seen, consumed = [], set(), set()
    tries = 0
    while len(merges) < n_merges and tries < 50 * n_merges and len(seq) > 1:
        tries += 1
        i = rng.randrange(len(seq) - 1)
        x, y = seq[i], seq[i + 1]
        z = x + y
        if len(z) > max_len or (x, y) in seen or z in consumed:
            continue
        seen.add((x, y))
        merges.append((x, y))
        consumed.update((x, y))
        if z not in vocab:
            vocab[z] = len(vocab)
        out, j = [], 0
        while j < len(seq):
            if j + 1 < len(seq) and seq[j] == x and seq[j + 1] == y:
                out.append(z)
                j += 2
            else:
                out.append(seq[j])
                j += 1
        seq = out
    return tok_json(vocab, merges)
