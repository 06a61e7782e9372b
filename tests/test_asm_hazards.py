"""The shipped schedule against the MFMA-result -> inline-asm hazard (verdict r05 item 1), on the CPU:
tools/asm_hazard_check.py disassembles the gfx950 code object inside the in-tree libdpk.so and checks every
inline-asm permlane swap whose register was last written by an MFMA for the MFMA's wait states.  The checker
itself is pinned on small synthetic listings first (a short pad is caught, a long enough one passes, a later
VALU write shadows the MFMA, an unconditional branch ends the walk)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import asm_hazard_check as H  # noqa: E402

LIB = os.path.join(ROOT, "diffpose-nw_amd", "diffpose_amd", "libdpk.so")


def _listing(*body):
    return "0000000000001000 <f>:\n" + "".join(f"\t{b}  // 000000001000: 00000000\n" for b in body)


def _check(*body):
    return H.check(H.parse(_listing(*body)))


def test_checker_flags_a_short_pad():
    v, traced, swaps = _check("v_mfma_f32_4x4x4_16b_f16 v[0:3], v[4:5], v[6:7], v[0:3]",
                              "s_nop 1",
                              "v_permlane32_swap_b32_e32 v0, v1")
    assert swaps == 1 and traced == 1 and len(v) == 1 and v[0][5] == 2 and v[0][6] == 5


def test_checker_passes_enough_wait_states():
    v, traced, _ = _check("v_mfma_f32_16x16x32_bf16 v[0:3], v[4:7], v[8:11], v[0:3]",
                          "s_nop 5", "v_add_f32_e32 v20, v21, v22", "v_mov_b32_e32 v23, v24",
                          "v_permlane16_swap_b32_e32 v2, v30")
    assert traced == 1 and not v          # 6 + 1 + 1 = 8 wait states, 8 needed
    v, _, _ = _check("v_mfma_f32_16x16x4_f32 v[0:3], v4, v5, v[0:3]", "s_nop 7",
                     "v_permlane16_swap_b32_e32 v2, v30")
    assert len(v) == 1 and v[0][6] == 10   # the f32 form needs 10


def test_checker_respects_later_writes_and_branches():
    v, traced, _ = _check("v_mfma_f32_4x4x1_16b_f32 v[0:3], v4, v5, v[0:3]",
                          "v_mov_b32_e32 v0, v9",
                          "v_permlane32_swap_b32_e32 v0, v12")
    assert traced == 0 and not v          # v0 rewritten by a VALU op: hipcc padded that one itself
    v, traced, _ = _check("v_mfma_f32_4x4x1_16b_f32 v[0:3], v4, v5, v[0:3]",
                          "s_branch 4",
                          "v_permlane32_swap_b32_e32 v0, v12")
    assert traced == 0 and not v          # not a fall-through predecessor


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(H.OBJDUMP)),
                    reason="needs the built libdpk.so and llvm-objdump")
def test_shipped_library_has_no_short_mfma_to_permlane_distance():
    v, traced, swaps = H.check(H.parse(H.disassemble(LIB)))
    assert swaps > 1000                    # the lane reductions of every instance
    assert traced > 0                      # some swaps do take MFMA results: the check is exercised
    assert not v, v[:5]
