"""Issue-cycle model of the detector's VALU stream: the opcode mix of the
code-specialised kernel's step loop (profiles/isa_breakdown.py, static, per
step) weighted by the measured issue cost of each instruction class
(profiles/valu_issue_bench.hip -> profiles/valu_issue_cycles.json).

  average cycles per VALU instruction = sum(count_op * cycles(class(op))) / sum(count_op)

The static mix counts every block of the loop once per step, the conditional
(hashed-lookup, key compare) blocks included; the dynamic count comes from the
SQ_INSTS_VALU counter.  Used by profiles/summarize.py, which stores the average
in the PMC summary for bench.py's roofline.valu.
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def op_class(op):
    """Microbenchmark class of an opcode (names as in valu_issue_bench.hip)."""
    if op.startswith(("v_pk_min", "v_pk_max")):
        return "v_pk_min_u16 (VOP3P)"
    if op.startswith("v_pk_"):
        return "v_pk_add_u16 (VOP3P)"
    if op.startswith("v_perm"):
        return "v_perm_b32 (VOP3)"
    if op.startswith(("v_mad_u64", "v_lshl_add_u64", "v_mad_i64")):
        return "v_mad_u64_u32 (VOP3)"
    if op.startswith(("v_add_f64", "v_mul_f64", "v_fma_f64")):
        return "v_add_f64"
    if op.startswith(("v_mul_lo", "v_mul_hi")):
        return "v_mul_lo_u32 (VOP3)"
    if op.startswith("v_lshl_add_u32"):
        return "v_lshl_add_u32 (VOP3)"
    if op.startswith("v_or3"):
        return "v_or3_b32 (VOP3)"
    if op.endswith("_e32"):
        # VOP2 / VOPC / VOP1 encodings
        if op.startswith(("v_lshlrev", "v_lshrrev", "v_ashrrev")):
            return "v_lshlrev_b32 (VOP2)"
        if op.startswith("v_cndmask"):
            return "v_add_u32 (VOP2)"   # VOP2 select (the e64 form is measured; VOP2 priced as an add)
        if op.startswith("v_sub"):
            return "v_sub_u32 (VOP2)"
        if op.startswith(("v_xor", "v_and", "v_or")):
            return "v_xor_b32 (VOP2)"
        return "v_add_u32 (VOP2)"
    # everything else is a VOP3(-encoded) instruction: bitop3, and_or, lshl_or,
    # add3, bfe, alignbit, mad_i32_i24, bcnt, e64 compares and selects, SDWA
    return "v_bitop3_b32 (VOP3)"


def load_cycles(path=None):
    path = path or os.path.join(HERE, "valu_issue_cycles.json")
    with open(path) as f:
        d = json.load(f)
    return {r["op"]: r["cycles_per_wave_inst_per_simd"] for r in d["results"]}, d


import re

# ─── round 5: operand-aware prices (profiles/valu_issue_cycles_r05.json, from profiles/r05an) ───
# On gfx950 the issue cost depends on the operands as much as on the opcode: bitop3, and, or,
# xor, not, mov, add, sub and lshrrev issue at ~2.4-2.8 cycles per wave64 instruction with
# VGPR, inline-constant or literal sources and at ~4.1-4.4 with any SGPR (or SGPR-pair / VCC)
# source; lshlrev, bfi, perm, alignbit, bfe, add3, or3, and_or, lshl_or, min, med3, mul*, mad,
# 64-bit shifts, packed and f64 ops and cndmask issue at ~4.2-4.6 whatever their operands.
# (The class table above priced every VOP3 op, bitop3 included, at its SGPR-operand cost.)
FAST_R05 = {"v_bitop3_b32": 2.70, "v_and_b32": 2.57, "v_or_b32": 2.54, "v_xor_b32": 2.60, "v_not_b32": 2.43,
            "v_mov_b32": 2.39, "v_add_u32": 2.50, "v_sub_u32": 2.49, "v_subrev_u32": 2.49, "v_lshrrev_b32": 2.41}
SLOW_R05 = {"v_add_f64": 4.57, "v_mul_f64": 4.57, "v_add3_u32": 4.64, "v_mad_u64_u32": 4.43, "v_lshl_add_u64": 4.43,
            "v_mul_lo_u32": 4.41}
SLOW_DEFAULT_R05 = 4.25      # every other opcode, and a fast opcode with a scalar source
_SREG = re.compile(r"(?<![\w\[])(s\d+|s\[\d+:\d+\]|vcc|exec|m0)(?!\w)")


def line_cycles_r05(line):
    """(class, cycles) of one VALU instruction line of the ISA (operand-aware)."""
    parts = line.split(None, 1)
    op = re.sub(r"_e(32|64)$", "", parts[0])
    operands = re.sub(r"bitop3:\S+|op_sel\S*|clamp|offset:\S+", "", parts[1] if len(parts) > 1 else "")
    fields = [f.strip() for f in operands.split(",")]
    # sources: everything after the destination(s) (v_cmp*: the SGPR-pair / VCC destination;
    # v_mad_u64_u32: the carry-out SGPR pair after the vector destination)
    nd = 2 if op in ("v_mad_u64_u32", "v_mad_i64_i32") else 1
    srcs = ",".join(fields[nd:])
    scalar = bool(_SREG.search(srcs))
    if op in FAST_R05:
        return (op + (" (scalar src)" if scalar else ""), SLOW_DEFAULT_R05 if scalar else FAST_R05[op])
    return (op, SLOW_R05.get(op, SLOW_DEFAULT_R05))


def weighted_line_cycles(lines_per_step):
    """(average issue cycles per VALU instruction, per-class breakdown) of a mix of ISA lines
    (line -> instructions per step), priced by line_cycles_r05."""
    tot_n, tot_c, by = 0.0, 0.0, {}
    for line, n in lines_per_step.items():
        if not line.startswith("v_"):
            continue
        cls, cyc = line_cycles_r05(line)
        tot_n += n
        tot_c += n * cyc
        b = by.setdefault(cls, [0.0, 0.0])
        b[0] += n
        b[1] += n * cyc
    return tot_c / max(tot_n, 1e-9), {k: {"insts_per_step": v[0], "cycles_per_step": v[1]} for k, v in by.items()}


def weighted_cycles(opcodes_per_step, cycles):
    """(average issue cycles per VALU instruction, per-class breakdown) of a mix."""
    tot_n, tot_c, by = 0.0, 0.0, {}
    for op, n in opcodes_per_step.items():
        if not op.startswith("v_"):
            continue
        c = op_class(op)
        tot_n += n
        tot_c += n * cycles[c]
        b = by.setdefault(c, [0.0, 0.0])
        b[0] += n
        b[1] += n * cycles[c]
    return tot_c / max(tot_n, 1e-9), {k: {"insts_per_step": v[0], "cycles_per_step": v[1]} for k, v in by.items()}
