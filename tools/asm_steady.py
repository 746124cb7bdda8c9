#!/usr/bin/env python3
"""Steady-state loops of one wide-kernel instance in a hipcc -S file: for each loop whose
body holds the full level work of B rows (dpp count = 4 x levels x rows), its instruction
mix (tools/asm_loops.py's counters) -- the evidence that the production loops issue the
modelled 20 fp64 + 4 DPP per level-row on average (5 per cell: the box-sum step of round 6,
22 on an even row and 18 on the odd row after it) and no scratch.

usage: asm_steady.py FILE.s KERNEL_SUBSTRING DPP_PER_TRIP
"""
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from asm_loops import kernel_lines, mix  # noqa: E402


def main():
    path, sub, dpp = sys.argv[1], sys.argv[2], int(sys.argv[3])
    body = kernel_lines(path, sub)
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = i
    seen = set()
    for i, l in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", l)
        if not m:
            continue
        tgt = m.group(1) or m.group(2)
        if tgt in labels and labels[tgt] < i:
            c = mix(body[labels[tgt]:i + 1])
            key = tuple(sorted(c.items()))
            if c.get("dpp") == dpp and c.get("f64", 0) == 5 * dpp and key not in seen:
                seen.add(key)
                role = "first wave (loads)" if c.get("bload") else (
                    "last wave (stores)" if c.get("bstore") else "middle wave (LDS in/out)")
                print(f"{role}: " + ", ".join(f"{k}={v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
