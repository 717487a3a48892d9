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
