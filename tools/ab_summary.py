"""Mean device time and per-stage times per library of a session's `ab:` probe log
(tools/session.sh ab:CFG:FIX:LIB_A:LIB_B writes gpurun_out/<tag>/ab_<cfg>_<fix>.txt).

usage: python tools/ab_summary.py gpurun_out/<tag>/ab_c4_gpt2_50k.txt [...]
"""
import ast
import collections
import re
import sys

KEYS = ("ms_segment", "ms_bpe_short", "ms_bpe_lo", "ms_bpe_hi", "ms_bpe_med", "ms_emit")


def summarize(path):
    dev = collections.defaultdict(list)
    stages = collections.defaultdict(list)
    for line in open(path):
        lib = line.split()[0]
        if "MB/s" in line:
            dev[lib].append(float(re.search(r"device ([\d.]+) ms", line).group(1)))
        elif "{" in line:
            stages[lib].append(ast.literal_eval(line[line.index("{"):]))
    print(path)
    for lib in dev:
        ks = stages[lib]
        parts = " ".join("%s %.3f" % (k[3:], sum(x[k] for x in ks) / len(ks)) for k in KEYS)
        print("  %-14s n=%d dev %.3f (min %.3f)  %s" % (lib, len(dev[lib]), sum(dev[lib]) / len(dev[lib]),
                                                     min(dev[lib]), parts))


if __name__ == "__main__":
    for p in sys.argv[1:]:
        summarize(p)
