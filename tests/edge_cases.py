"""Edge-case documents for parity tests: regex piece boundaries, whitespace runs, contractions,
non-ASCII classes, NFC-changing input, long runs, empty docs."""

EDGE = [
    "", " ", "  ", "a", "a  b", "a b", "a\tb", "a\t1", "a\n\nb", " \n", "\n ", "   x", "x   ", "x \n y",
    "Hello, world!", "I 'll", " 's", "  's", "'s", "'sss", "'S", "'re'", "'rex", "'l", "'ll", "'llx", "don't",
    "it's", "we've", "they're", "I'm", "you'd", "''s", "5's", ".'s", " '", "x 's'", "'", "''", "'\n's",
    "hello123world", "12 34", " 12", "a1b2", "x\u00a0y", "x \u00a0y", "\u00a0 x", "x\u3000y", "x\u2009y",
    "\u0085x", "x\u200by", "caf\u00e9", "cafe\u0301", "e\u0301", "\u1100\u1161\u11a8", "\uac01",
    "\uf900\uf901", "\u212b", "A\u030a", "\u0344", "D\u0323\u0307", "q\u0307\u0323",
    "\u3053\u3093\u306b\u3061\u306f \u4e16\u754c\U0001f600\U0001f44d\U0001f3fd x",
    "\u0627\u0644\u0639\u0631\u0628\u064a\u0629 \u0661\u0662",
    "\U0001f468\u200d\U0001f469\u200d\U0001f467", "\u2014 dash \u2014", "naive\u0308", "A\u030angstro\u0308m",
    "tab\tsep\tvalues\t", "trailing space ", " leading", "multi\n\n\nnewline", "\r\n", "a\r\nb",
    "<|endoftext|>", "x<|endoftext|>y", "a" * 33, "a" * 64, "a" * 65, "ab" * 40, "\u00e9" * 40,
    " " * 40, "!" * 50, "1" * 70, "\u4e00" * 30, "\u00e9\u0301\u0327", "\u0301abc", " \u0301",
]


def long_docs():
    import random
    rng = random.Random(7)
    docs = []
    docs.append("a" * 5000)
    docs.append("ab" * 2500)
    docs.append("".join(rng.choice("abcdefghijklmnopqrstuvwxyz") for _ in range(3000)))
    docs.append("".join(rng.choice("0123456789") for _ in range(4000)))
    docs.append(" " * 3000)
    docs.append("x" + " " * 2000 + "y")
    docs.append("".join(rng.choice("一二三四五六") for _ in range(700)))
    docs.append("!?" * 1000)
    docs.append("aaab" * 800)
    docs.append("the" * 1200)
    return docs


def random_unicode_docs(n, seed, max_len=40):
    """Random strings over an alphabet that stresses the regex classes and NFC."""
    import random
    rng = random.Random(seed)
    alpha = (list(" \t\n\r'") * 3 + list("aeiostrmdlvSTE") + list("0123456789") + list(".,!?-_()\"")
             + [" ", "　", " ", "\u0085", "é", "é", "́", "̈", "世", "あ",
                "가", "ᄀ", "ᅡ", "\U0001f600", "‍", "️", "١", "²", "Ⅷ",
                "豈", "Å", "Å", "ا", "א", "ก", "ั"])
    docs = []
    for _ in range(n):
        L = rng.randint(0, max_len)
        docs.append("".join(rng.choice(alpha) for _ in range(L)))
    return docs
