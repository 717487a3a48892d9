#!/usr/bin/env python3
"""Issue-cost estimate of a kernel's VALU stream from its ISA (profiles/r05an/vib*.json):
fast (~2.5 cycles per wave64 instruction on gfx950): bitop3, and, or, xor, not, mov, add,
sub, lshrrev with VGPR / inline / literal operands; slow (~4.2): any SGPR or SGPR-pair/VCC
source, lshlrev, and the other opcodes (bfi, perm, alignbit, bfe, add3, or3, mad, f64 ...).

  python profiles/r05_isa_cost.py loop.s
"""
import re
import sys
from collections import Counter

FAST = {"v_bitop3_b32", "v_and_b32_e32", "v_or_b32_e32", "v_xor_b32_e32", "v_xor_b32_e64", "v_not_b32_e32",
        "v_mov_b32_e32", "v_mov_b32", "v_add_u32_e32", "v_add_u32_e64", "v_sub_u32_e32", "v_lshrrev_b32_e32",
        "v_lshrrev_b32_e64", "v_subrev_u32_e32"}
SREG = re.compile(r"(?<![a-z_])(s\d+|s\[\d+:\d+\]|vcc|exec)(?![\w])")


def classify(line):
    op = line.split()[0]
    operands = line.split(None, 1)[1] if len(line.split(None, 1)) > 1 else ""
    operands = re.sub(r"bitop3:\S+", "", operands)
    srcs = operands.split(",", 1)[1] if "," in operands else ""
    if op.startswith("v_cmp"):
        srcs = operands.split(",", 1)[1] if "," in operands else ""   # dst is the SGPR pair
    has_s = bool(SREG.search(srcs))
    if op in FAST and not has_s:
        return "fast", op
    return "slow", op + (" (s)" if has_s else "")


def main():
    lines = [l.strip() for l in open(sys.argv[1]) if re.match(r"\s+v_", l)]
    c = Counter()
    ops = Counter()
    for l in lines:
        k, op = classify(l)
        c[k] += 1
        if k == "slow":
            ops[op] += 1
    print(f"VALU {len(lines)}: fast {c['fast']}, slow {c['slow']}; cycles ~ {2.5 * c['fast'] + 4.25 * c['slow']:.0f}")
    for op, n in ops.most_common(30):
        print(f"  {n:4d} {op}")


if __name__ == "__main__":
    main()
