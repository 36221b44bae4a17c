"""Instruction histogram of the innermost loops of one kernel in a device assembly file (hipcc -S --cuda-device-only).
A loop = a backward branch to a label inside the kernel; its body is the instruction range label..branch.
usage: python tools/isa_loops.py file.s kernel_symbol_prefix [min_len]"""
import re
import sys
from collections import Counter


def main():
    path, sym = sys.argv[1], sys.argv[2]
    minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym) and l.rstrip().endswith(":") or
                 (l.startswith(sym) and ": ;" in l))
    end = next(i for i in range(start, len(lines)) if lines[i].strip() == "s_endpgm")
    labels = {}
    for i in range(start, end):
        m = re.match(r"^(\.LBB\w+):", lines[i])
        if m:
            labels[m.group(1)] = i
    for i in range(start, end):
        m = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\w+)|\s+s_branch\s+(\.LBB\w+)", lines[i])
        if not m:
            continue
        tgt = m.group(1) or m.group(2)
        if tgt in labels and labels[tgt] < i:
            body = [l.strip().split()[0] for l in lines[labels[tgt]:i + 1]
                    if l.strip() and not l.strip().startswith((";", ".", "//")) and not l.strip().endswith(":")]
            if len(body) < minlen:
                continue
            c = Counter(body)
            v = sum(n for k, n in c.items() if k.startswith("v_"))
            print("loop %s (lines %d-%d): %d instructions, %d VALU" % (tgt, labels[tgt], i, len(body), v))
            print("   ", ", ".join("%s %d" % kv for kv in c.most_common(30)))


if __name__ == "__main__":
    main()
