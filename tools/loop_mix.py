#!/usr/bin/env python3
"""Instruction mix of the hot loops in a kernel's ISA (tools/kernel_asm.sh):
for every loop with more than 40 VALU instructions, counts per opcode,
s_nop wait states, and the dependency behind each s_nop (producer opcode and
distance).  Usage: python3 tools/loop_mix.py FILE.s"""
import collections
import re
import sys


def regs(txt):
    out = []
    for m in re.finditer(r"v\[(\d+):(\d+)\]|v(\d+)", txt):
        out += [int(m.group(3))] if m.group(3) else list(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def main(path):
    lines = [l.rstrip() for l in open(path)]
    heads = [i for i, l in enumerate(lines) if "Loop Header" in l]
    for h in heads:
        end = next((j for j in range(h + 1, len(lines)) if lines[j].strip().startswith("s_cbranch_scc")), None)
        if end is None:
            continue
        body = [l.strip() for l in lines[h + 1:end + 1] if l.strip() and not l.strip().startswith(";")
                and not l.strip().startswith(".")]
        valu = [l for l in body if l.startswith("v_")]
        if len(valu) < 40:
            continue
        mix = collections.Counter(l.split()[0] for l in body)
        nops = [(k, l) for k, l in enumerate(body) if l.startswith("s_nop")]
        wait_states = sum(int(l.split()[1]) + 1 for _, l in nops)
        print(f"loop @ line {h + 1}: {len(valu)} VALU, {len(nops)} s_nop ({wait_states} wait states)")
        for op, n in mix.most_common():
            print(f"   {n:4d} {op}")
        why = collections.Counter()
        for k, l in nops:
            nxt = body[k + 1] if k + 1 < len(body) else ""
            parts = nxt.split(None, 1)
            srcs = set(regs(parts[1].split(",", 1)[1])) if len(parts) > 1 and "," in parts[1] else set()
            d, found = 0, "?"
            for j in range(k - 1, max(k - 8, -1), -1):
                if body[j].startswith("s_"):
                    continue
                d += 1
                a = body[j].split(None, 1)
                if len(a) > 1 and set(regs(a[1].split(",")[0])) & srcs:
                    found = f"{a[0]} at distance {d}"
                    break
            why[f"{l} before {parts[0] if parts else '?'} <- {found}"] += 1
        for k, n in why.most_common():
            print(f"   nop x{n}: {k}")


if __name__ == "__main__":
    main(sys.argv[1])
