"""Static check of the MFMA-result -> inline-asm hazard in the built library (verdict r05 item 1).

hipcc pads the wait states between an MFMA and a compiler-visible reader of its result registers, but not
for a reader inside inline asm.  The only such readers in the kernels are the lane reductions'
`v_permlane16/32_swap` (csrc/dpk_sampler.inc: rs4rows, sum4rows2, max4rows2, attention's denominator swap),
and `mfma_pad` puts the wait states ahead of the ones that take MFMA accumulators.  This tool checks the
shipped schedule instead of trusting the source: it pulls the gfx950 code object out of libdpk.so's offload
bundle, disassembles it (llvm-objdump), and for every permlane swap walks back along the instruction stream
to the instruction that last wrote each of its registers; when that is an MFMA, the wait states between them
(one per instruction, N + 1 per `s_nop N`) must reach the MFMA's requirement.  The walk follows fall-through
code only: it stops at an unconditional branch or the function start, so a writer reached through a jump is
not seen (none of the swaps sits at a jump target's first instructions in today's code; the walk reports how
many swaps it traced back to an MFMA, so a change that moved them all out of reach would show).

  python tools/asm_hazard_check.py [path/to/libdpk.so]     # exit 1 on a violation
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

# wait states a VALU read of an MFMA's result registers needs on gfx950: hipcc's own pads before a
# compiler-visible reader (tools/mfma_hazard_probe.hip: s_nop 3 after v_mfma_f32_4x4x1_16b_f32, 4 after the
# 4x4x4_16b f16/bf16 forms, 7 after the 16x16x16 / 16x16x32 f16/bf16 forms, 9 after v_mfma_f32_16x16x4_f32)
# plus one for the s_nop's own count; 32x32 forms by the same pass-count rule
def required_states(mnemonic):
    m = mnemonic
    if "4x4x1" in m and "f32" in m.split("4x4x1")[1][:6]:
        return 4
    if "_4x4x" in m:
        return 5
    if "16x16x4" in m and ("f32" in m.split("16x16x4")[1][:6] or m.endswith("x4f32")):
        return 10
    if "16x16" in m:
        return 8
    if "32x32" in m:
        return 18
    return 18


REG = re.compile(r"\b([va])(?:(\d+)|\[(\d+):(\d+)\])")


def regs(text):
    out = set()
    for kind, one, lo, hi in REG.findall(text):
        if one:
            out.add((kind, int(one)))
        else:
            out.update((kind, r) for r in range(int(lo), int(hi) + 1))
    return out


def code_object(so_path):
    d = open(so_path, "rb").read()
    i = d.find(b"__CLANG_OFFLOAD_BUNDLE__")
    if i < 0:
        raise SystemExit(f"{so_path}: no clang offload bundle")
    n = struct.unpack_from("<Q", d, i + 24)[0]
    p = i + 32
    for _ in range(n):
        off, size, ts = struct.unpack_from("<QQQ", d, p)
        p += 24
        triple = d[p:p + ts].decode()
        p += ts
        if "gfx950" in triple:
            return d[i + off:i + off + size]
    raise SystemExit(f"{so_path}: no gfx950 code object")


def disassemble(so_path):
    with tempfile.TemporaryDirectory() as t:
        co = os.path.join(t, "co.elf")
        open(co, "wb").write(code_object(so_path))
        return subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", co], check=True, capture_output=True,
                              text=True).stdout


def parse(dis):
    """[(function, [(mnemonic, operand text), ...]), ...]"""
    funcs, cur, name = [], None, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            name, cur = m.group(1), []
            funcs.append((name, cur))
            continue
        if cur is None or not line.startswith("\t"):
            continue
        ins = line.split("//")[0].strip()
        if not ins:
            continue
        mn, _, ops = ins.partition(" ")
        cur.append((mn, ops.strip()))
    return funcs


def writes(mn, ops):
    """registers an instruction writes (first operand of VALU ops, vector loads and MFMAs; both of a swap)"""
    if mn.startswith("v_permlane") and "swap" in mn:
        return regs(ops)
    if mn.startswith("v_") or mn.startswith(("buffer_load", "global_load", "ds_read", "flat_load", "scratch_load")):
        first = ops.split(",")[0]
        return regs(first)
    return set()


def check(funcs):
    violations, traced, swaps = [], 0, 0
    for name, ins in funcs:
        for k, (mn, ops) in enumerate(ins):
            if not (mn.startswith("v_permlane") and "swap" in mn):
                continue
            swaps += 1
            pending = regs(ops)
            states = 0
            j = k - 1
            while j >= 0 and pending and states < 24:
                pm, po = ins[j]
                if pm == "s_branch" or pm == "s_endpgm" or pm.startswith("s_setpc"):
                    break
                w = writes(pm, po) & pending
                if w:
                    if pm.startswith("v_mfma"):
                        traced += 1
                        need = required_states(pm)
                        if states < need:
                            violations.append((name, k, mn, ops, pm, states, need))
                    pending -= w
                m = re.match(r"s_nop\s+(\w+)", f"{pm} {po}")
                states += (int(m.group(1), 0) + 1) if m else 1
                j -= 1
    return violations, traced, swaps


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "diffpose-nw_amd", "diffpose_amd", "libdpk.so")
    v, traced, swaps = check(parse(disassemble(so)))
    print(f"{swaps} permlane swaps, {traced} of their registers last written by an MFMA, {len(v)} short of its wait states")
    for name, k, mn, ops, pm, states, need in v[:20]:
        print(f"  {name[:80]} #{k}: {mn} {ops} after {pm}: {states} < {need} wait states")
    return 1 if v else 0


if __name__ == "__main__":
    sys.exit(main())
