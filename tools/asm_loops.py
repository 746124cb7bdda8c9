"""List the loops of one kernel in a hipcc -S file with their instruction mix.

usage: asm_loops.py FILE.s KERNEL_SUBSTRING
A loop is a backward branch to a label; its body is every line between the label and the
branch. Counts: VALU (v_*), fp64 VALU (v_*_f64), DPP moves, buffer loads/stores, scratch,
s_waitcnt, s_nop. Used to check what the steady-state loop of the K-step kernel issues.
"""
import re
import sys
from collections import Counter


def kernel_lines(path, sub):
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*:", l) and sub in l:
            start = i
        elif start is not None and l.strip().startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit("kernel not found")


def mix(body):
    c = Counter()
    for l in body:
        t = l.strip().split()
        if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
            continue
        op = t[0]
        if op.startswith("v_"):
            c["valu"] += 1
            if "f64" in op:
                c["f64"] += 1
            if "dpp" in l:
                c["dpp"] += 1
            if op.startswith("v_mov") or op.startswith("v_accvgpr"):
                c["mov"] += 1
        elif op.startswith("buffer_load"):
            c["bload"] += 1
        elif op.startswith("buffer_store"):
            c["bstore"] += 1
        elif op.startswith("scratch_") or "scratch" in op:
            c["scratch"] += 1
        elif op.startswith("s_waitcnt"):
            c["waitcnt"] += 1
        elif op.startswith("s_nop"):
            c["nop"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        c["all"] += 1
    return c


def main():
    body = kernel_lines(sys.argv[1], sys.argv[2])
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = i
    for i, l in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", l)
        if not m:
            continue
        tgt = m.group(1) or m.group(2)
        if tgt in labels and labels[tgt] < i:
            c = mix(body[labels[tgt]:i + 1])
            print(f"loop {tgt} lines {labels[tgt]}..{i}: " + ", ".join(f"{k}={v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
