"""The operand-aware VALU issue prices (profiles/valu_model.py, line_cycles_r05) that price
bench.py's roofline.valu: vector / constant sources fast, any scalar source slow, and the
opcodes measured slow whatever their operands (profiles/r05an).  CPU only."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles"))
import valu_model as vm  # noqa: E402


def test_operand_kinds():
    assert vm.line_cycles_r05("v_bitop3_b32 v1, v2, v3, v4 bitop3:0xca")[1] < 3.0
    assert vm.line_cycles_r05("v_bitop3_b32 v1, s2, v3, v4 bitop3:0xca")[1] > 4.0
    assert vm.line_cycles_r05("v_bitop3_b32 v1, v2, 0, v4 bitop3:0xca")[1] < 3.0       # inline constant
    assert vm.line_cycles_r05("v_xor_b32_e32 v1, 0x55555555, v2")[1] < 3.0               # literal
    assert vm.line_cycles_r05("v_and_b32_e32 v1, s88, v2")[1] > 4.0
    assert vm.line_cycles_r05("v_lshrrev_b32_e32 v1, 4, v2")[1] < 3.0
    assert vm.line_cycles_r05("v_lshlrev_b32_e32 v1, 4, v2")[1] > 4.0                    # any lshlrev
    assert vm.line_cycles_r05("v_cndmask_b32_e32 v1, 0, v2, vcc")[1] > 4.0
    assert vm.line_cycles_r05("v_perm_b32 v1, v2, v3, v4")[1] > 4.0
    # the carry-out SGPR pair of v_mad_u64_u32 is a destination, not a source
    assert vm.line_cycles_r05("v_mad_u64_u32 v[2:3], s[8:9], v4, v5, 0")[0] == "v_mad_u64_u32"


def test_mix_average():
    avg, by = vm.weighted_line_cycles({"v_bitop3_b32 v1, v2, v3, v4 bitop3:0x96": 3.0,
                                       "v_bitop3_b32 v1, s2, v3, v4 bitop3:0x96": 1.0})
    assert abs(avg - (3 * 2.70 + 4.25) / 4) < 1e-9
    assert set(by) == {"v_bitop3_b32", "v_bitop3_b32 (scalar src)"}
