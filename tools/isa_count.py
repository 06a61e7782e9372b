"""Instruction mix of one device function inside the sampler kernel (build container only).

Inserts asm comment markers at the entry and the last closing brace of the named
__device__ function, compiles the kernel source to gfx950 assembly and counts the
instructions between the first pair of markers inside the chosen kernel instance.
  python tools/isa_count.py layer_norm [--kernel _ZN3dpk13sample_kernelILi0ELb1ELb0EE]
"""
import argparse
import collections
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "diffpose-nw_amd", "csrc", "dpk_sampler.inc")
KSRC = os.path.join(ROOT, "diffpose-nw_amd", "csrc", "dpk_kernels.hip")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("func")
    ap.add_argument("--kernel", default="_ZN3dpk13sample_kernelILi0ELb1ELi0EE")
    ap.add_argument("--nth", type=int, default=0, help="which marked region inside the kernel")
    ap.add_argument("--ignore-returns", action="store_true",
                    help="no end marker at early returns (a never-taken guard such as attention's pose >= P)")
    a = ap.parse_args()
    s = open(SRC).read()
    i = s.index(f"__device__ __forceinline__ void {a.func}(")
    b = s.index(") {", i) + 2   # the body (not a default argument such as Hook{})
    # matching closing brace
    depth, j = 0, b
    while True:
        if s[j] == "{":
            depth += 1
        elif s[j] == "}":
            depth -= 1
            if depth == 0:
                break
        j += 1
    body = s[b + 1:j]
    s2 = s[:b + 1] + '\n    asm volatile(";MARK_BEGIN" ::: "memory");' + (body if a.ignore_returns else body.replace("return;", 'asm volatile(";MARK_END" ::: "memory"); return;')) \
        + '    asm volatile(";MARK_END" ::: "memory");\n' + s[j:]
    # the device functions live in dpk_sampler.inc, included by dpk_kernels.hip: compile a copy of
    # both from a scratch directory
    os.makedirs("/tmp/isa_count", exist_ok=True)
    for inc in os.listdir(os.path.dirname(SRC)):
        if inc.endswith(".inc"):
            open(os.path.join("/tmp/isa_count", inc), "w").write(open(os.path.join(os.path.dirname(SRC), inc)).read())
    open("/tmp/isa_count/dpk_sampler.inc", "w").write(s2)
    tmp = "/tmp/isa_count/dpk_kernels.hip"
    open(tmp, "w").write(open(KSRC).read())
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form", "-mllvm", "-misched-cluster=0", "-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule=1", f"-I{ROOT}/include", "-Wno-unused-result", "--cuda-device-only", "-S",
                    tmp, "-o", "/tmp/isa_count.s"], check=True, stderr=subprocess.DEVNULL)
    asm = open("/tmp/isa_count.s").read()
    k = asm.index(a.kernel)
    k = asm.index(a.kernel + "EvNS_10SampleArgsEPKfPKc:", k) if (a.kernel + "EvNS_10SampleArgsEPKfPKc:") in asm else k
    pos = k
    for _ in range(a.nth + 1):
        st = asm.index(";MARK_BEGIN", pos)
        nxt = asm.find(";MARK_BEGIN", st + 1)
        if nxt < 0:
            nxt = len(asm)
        en = asm.rindex(";MARK_END", st, nxt)      # the last exit of this inlined copy
        pos = en
    ins = [l.strip() for l in asm[st:en].splitlines()
           if l.strip() and not l.strip().startswith((";", "."))]
    c = collections.Counter(x.split()[0] for x in ins)
    print(len(ins), "instructions")
    print(c.most_common(40))


if __name__ == "__main__":
    main()
