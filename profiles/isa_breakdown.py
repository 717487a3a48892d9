#!/usr/bin/env python3
"""Instruction breakdown of the code-specialised detector loop (cvd_k1b_spec), from the
ISA the JIT would build for a decoder (csrc/spec_resource.py compiles it exactly as
cvd_rtc.cpp does; no GPU needed).

The main loop (4 steps per iteration) is split into its basic blocks; each VALU
instruction is assigned to a functional class from its opcode and, for the
ambiguous 32-bit adds/perms, from the operand pattern the kernel source produces:

  acs      butterfly add-compare-select (v_pk_min_u16, the VOP2 adds of the
           no-broadcast steps, v_pk_add_u16 broadcasts, e-pair perms)
  pack     16-bit pairs -> nibble keys (byte perms, shift-adds, offset subtract)
  zero     step-minimum test on the keys (haszero nibble test, or-reductions)
  norm     key normalisation (minus mu in every nibble) and the running offset
  hash     key hash for the P̂1 row table (64-bit multiply-accumulates, mixes)
  cursor   row-table cursor: filter bits/test, address math, selects, key compare
  tref     T_ref count (halves differences, pair-swap test)
  f64      log-likelihood adds
  stream   received-word extraction, branch-metric pair setup
  other    everything else (moves, compares feeding branches)

Blocks are reported as "always" (straight-line step code) or "conditional" (guarded
by exec-mask branches: filter-positive loads, key compare, probing, hashing), with
their static VALU counts.  A wave executes a conditional block whenever ANY of its
64 lanes takes it, so for the mixed lanes of a wave most of them run every step.

  python profiles/isa_breakdown.py [m6] [--isa out.s] [-D...] [--steps S --nth K]

(-DCVD_K1B_BITSLICE=1: the bit-sliced kernel k1s, six steps per iteration; its classes are
the opcode classes above, which for k1s mostly land in "logic" (v_bitop3) and "pack" (v_perm))
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "detecting-convolutional-codes-via-markovian-statistics_amd", "csrc")


def build_isa(cfg, defs, path):
    subprocess.run([sys.executable, os.path.join(CSRC, "spec_resource.py"), cfg, *defs, "--isa", path],
                   check=True, capture_output=True, text=True)
    return open(path).read().splitlines()


def main_loop(lines, nth=0):
    """Lines of the largest outermost loop (Depth=1) of the kernel body (the step
    loop; the prologue's LDS table fill is a small loop of its own).  nth = 1: the loop with
    the most v_bitop3 (the bit-sliced kernel's lockstep loop)."""
    found = []
    end = next((i for i, l in enumerate(lines) if l.startswith(".Lfunc_end")), len(lines))
    for hdr in (i for i, l in enumerate(lines[:end]) if "Loop Header: Depth=1" in l):
        label = lines[hdr].split(":")[0]
        backs = [i for i, l in enumerate(lines[:end]) if re.search(r"\bs_(c)?branch\w*\s+" + re.escape(label) + r"\b", l)]
        if backs:
            size = max(backs) - hdr
            if nth == 1:   # k1s: the lockstep loop is the one with the most bit-sliced logic
                size = sum("v_bitop3" in l for l in lines[hdr:max(backs) + 1])
            found.append((size, hdr, max(backs)))
    found.sort(reverse=True)
    nth = 0
    _, a, b = found[nth]
    return lines[a:b + 1]


def blocks(loop):
    out, cur, name = [], [], "entry"
    for l in loop:
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):", l.strip()) or re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            if cur:
                out.append((name, cur))
            name, cur = m.group(1), []
            continue
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            continue
        cur.append(s)
    if cur:
        out.append((name, cur))
    return out


def classify(ins):
    op = ins.split()[0]
    if not op.startswith("v_"):
        return None
    if op.startswith("v_pk_min_u16") or op.startswith("v_pk_add_u16") or op.startswith("v_pk_sub_u16"):
        return "acs"
    if op.startswith("v_mad_u64_u32") or op.startswith("v_mul_lo_u32") or op.startswith("v_lshl_add_u64") \
            or "xor_b32_sdwa" in op:
        return "hash"
    if op.startswith("v_add_f64"):
        return "f64"
    if op.startswith("v_bcnt") or op.startswith("v_mad_i32_i24") or op.startswith("v_bfe_u32") \
            or op.startswith("v_alignbit"):
        return "stream"
    if op.startswith("v_perm_b32"):
        return "pack"           # byte collapse of pairs (the two e-pair perms per step counted below)
    if op.startswith("v_lshl_add_u32"):
        return "pack"
    if op.startswith("v_add_u32") and "0xeeeeeeef" in ins:
        return "zero"
    if op.startswith("v_bitop3_b32") and "bitop3:0x30" in ins:
        return "zero"
    if op.startswith("v_add_u32") or op.startswith("v_sub_u32") and "_e32" in op:
        return "acs_or_norm"
    if op.startswith("v_cndmask") or op.startswith("v_cmp") or op.startswith("v_mov"):
        return "cursor"
    if op.startswith("v_xor_b32") or op.startswith("v_or3_b32") or op.startswith("v_and_or") \
            or op.startswith("v_bitop3") or op.startswith("v_and_b32") or op.startswith("v_or_b32"):
        return "logic"
    if op.startswith("v_lshlrev") or op.startswith("v_lshrrev") or op.startswith("v_lshl_or") \
            or op.startswith("v_add3"):
        return "cursor"
    return "other"


def main():
    args = sys.argv[1:]
    isa = None
    if "--isa" in args:
        i = args.index("--isa")
        isa = args[i + 1]
        del args[i:i + 2]
    steps, nth = 4, 0
    if "--steps" in args:
        i = args.index("--steps")
        steps = int(args[i + 1])
        del args[i:i + 2]
    if "--nth" in args:
        i = args.index("--nth")
        nth = int(args[i + 1])
        del args[i:i + 2]
    if "-DCVD_K1B_BITSLICE=1" in args and steps == 4:
        steps, nth = 6, 1     # k1s: six steps per lockstep iteration
    defs = [a for a in args if a.startswith("-")]
    rest = [a for a in args if not a.startswith("-")]
    cfg = rest[0] if rest else "m6"
    with tempfile.TemporaryDirectory() as d:
        path = isa or os.path.join(d, "k.s")
        lines = build_isa(cfg, defs, path)
    loop = main_loop(lines, nth)
    bl = blocks(loop)
    # straight-line blocks: not entered through an exec-mask branch (s_and_saveexec /
    # s_cbranch_execz in the preceding block) and not part of the probe loops
    always = collections.Counter()
    cond = collections.Counter()
    ops = collections.Counter()
    guarded = False
    per_block = []
    for name, ins in bl:
        vc = collections.Counter(c for c in map(classify, ins) if c)
        tgt = cond if guarded else always
        tgt.update(vc)
        per_block.append({"block": name, "guarded": guarded, "valu": sum(vc.values())})
        for x in ins:
            if x.startswith("v_"):
                ops[x.split()[0]] += 1
        # a block ending in s_cbranch_execz guards its fall-through successor;
        # s_or_b64 exec restores the full mask
        guarded = any(x.startswith("s_cbranch_execz") for x in ins[-2:])
        if any(x.startswith("s_or_b64 exec") for x in ins[:2]):
            guarded = False
    out = {
        "kernel": "cvd_k1b_spec", "config": cfg, "defines": defs, "steps_per_iteration": steps,
        "valu_per_step_always": {k: v / steps for k, v in sorted(always.items())},
        "valu_per_step_conditional": {k: v / steps for k, v in sorted(cond.items())},
        "valu_per_step_total_static": (sum(always.values()) + sum(cond.values())) / steps,
        "opcodes_per_step": {k: v / steps for k, v in ops.most_common()},
        "blocks": per_block,
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
