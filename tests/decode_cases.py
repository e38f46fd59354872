"""Inputs for the decode parity tests: texts that exercise the clean-up rules
(src/huggingface/mod.rs:749-767), white-space collapsing and lossy UTF-8, plus random id
batches (ids past the vocab, special tokens, token bytes cut mid-character)."""
import random

CLEANUP_TEXTS = [
    "", " ", "a", " a ", "a , b . c ! d ? e : f ; g", "x ,", ", x", " .", ". ", " . ", "  .", ".  ",
    '" quoted "', 'say " hi " now', '"  x', 'x  "', '" "', '""  ""', "' s", "don ' t", "' '", "( a )", "[ b ]",
    "( )", "[ ]", "(  x  )", "a - b", "a  -  b", " - - ", " - - - - - ", "a -b", "a- b", "--", " -- ",
    "x \n y", "x\t\ty", "x \u00a0 y", "\u3000x\u3000", "x\u2028y", "x\u0085y", "\u1680", "x\u200by",
    "a\u001cb", "tab\t,", "new\n.", "end .\n", " , . ! ? : ; ", "\" ' ( ) [ ] -", '"\'( [ x ] )\'"',
    ". " * 40, " ." * 70, " - " * 30, "\" " * 40, " ( [ " * 20, " " * 100 + "x" + " " * 100,
    "\n" * 50, "a" + " \n\t" * 30 + "b", "caf\u00e9 , na\u00efve .", "\u4e16\u754c , \U0001f600 !",
]


def random_batches(n_ids_table, n_docs, seed, max_len=60, special_ids=()):
    rng = random.Random(seed)
    out = []
    for _ in range(n_docs):
        n = rng.choice([0, 1, 2, 3, rng.randint(0, max_len)])
        seq = []
        for _ in range(n):
            r = rng.random()
            if r < 0.02:
                seq.append(n_ids_table + rng.randint(0, 1000))  # unknown id: dropped
            elif r < 0.05 and special_ids:
                seq.append(rng.choice(list(special_ids)))
            else:
                seq.append(rng.randrange(n_ids_table))
        out.append(seq)
    return out


def split_docs(batch, seed):
    """Cut the id sequences at random points into more documents (multi-byte characters spread
    over two documents decode as U+FFFD on both sides)."""
    rng = random.Random(seed)
    out = []
    for seq in batch:
        i = 0
        while i < len(seq):
            j = min(len(seq), i + rng.randint(1, 6))
            out.append(seq[i:j])
            i = j
        if not seq:
            out.append([])
    return out
