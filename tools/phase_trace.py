"""Per-phase cycle breakdown of one DDIM step of the sampler kernel.

Uses a trace build of libdpk (-DDPK_TRACE=1). In that build, lane 0 of every wave stamps
s_memtime before and after each workgroup barrier of one chosen step, and inside every GEMM at
the end of its k-loop and of its epilogue. Per phase (summed over the 5 layers) it reports the
slowest wave's segments, averaged over workgroups: GEMM startup+k-loop, epilogue, VALU compute
up to the barrier, and the barrier wait.

  python tools/phase_trace.py --build     # build container: hipcc -> build/trace/libdpk_trace.so
  python tools/phase_trace.py --run       # GPU box: B=1024, K=50, trace step 10
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.environ.get("DPK_TRACE_SO", os.path.join(ROOT, "build", "trace", "libdpk_trace.so"))

# stamp sequence of one DDIM step: every workgroup barrier stamps before ("pre") and after
# ("post"); every gemm_wave stamps at the end of its k-loop ("loop") and of its epilogue ("epi")
# the f16x3 GEMMs run a wave's column tiles in passes and stamp per pass
def _events(gemm_mode="fp32"):
    # LN1 is mapped wave = pose in 4-pose tiles: no barrier between LN1 and graph1 (round 6 removed the
    # fused-LayerNorm builds, which had no LN phases)
    fused, ln1pose = False, True
    ev = []
    bar = lambda n: ev.extend([(n, "pre"), (n, "post")])
    # the half-width-operand GEMMs run a wave's column tiles in passes (gemmh_wg): f16x3 QKV 3 x 3 tiles,
    # fc1 2 x 3; bf16 one pass each
    npass = {"QKV": 3, "fc1": 2} if gemm_mode == "f16x3" else {}

    def gemm(n):
        for _ in range(npass.get(n.split(".")[-1], 1)):
            ev.extend([(n, "loop"), (n, "epi")])
    bar("input_prep"); gemm("input_gemm"); bar("input_gemm")
    for l in range(5):
        p = f"L{l}."
        if not fused:
            bar(p + "LN0")
        gemm(p + "QKV"); bar(p + "QKV")
        bar(p + "attention"); gemm(p + "O"); bar(p + "O")
        if not fused and not ln1pose:
            bar(p + "LN1")
        bar(p + ("LN1+graph1" if fused or ln1pose else "graph1")); gemm(p + "fc1"); bar(p + "fc1")
        gemm(p + "fc2"); bar(p + "fc2")
        bar(p + "graph2+cheb1"); gemm(p + "C1"); bar(p + "C1")
        bar(p + "cheb_prep2"); gemm(p + "C2"); bar(p + "C2")
    bar("out_gemm"); bar("out_graph+ddim")
    return ev


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = [os.path.join(ROOT, "diffpose-nw_amd", "csrc", f) for f in ("dpk_kernels.hip", "dpk_metrics.hip", "dpk_gmm.hip")]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-ffp-contract=off", "-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form", "-mllvm", "-misched-cluster=0", "-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule=1", "-Wno-unused-result", f"-I{ROOT}/include", "-DDPK_TRACE=1"] + src + ["-o", SO]
    cmd += os.environ.get("DPK_TRACE_EXTRA", "").split()
    subprocess.run(cmd, check=True)
    print("built", SO)


def run(step=10, frames=1024, gemm_mode="fp32"):
    EVENTS = _events(gemm_mode)
    os.environ["DPK_LIB"] = SO
    sys.path.insert(0, os.path.join(ROOT, "diffpose-nw_amd"))
    import numpy as np
    import torch
    from diffpose_amd import _lib
    from diffpose_amd.data import synthetic_batch
    from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
    from diffpose_amd.schedule import get_beta_schedule, make_seq
    from diffpose_amd.weights import synthetic_state_dict

    L = _lib.lib()
    L.dpk_debug_trace.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong]
    L.dpk_debug_trace.restype = ctypes.c_int
    m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
    m.load_state_dict(synthetic_state_dict())
    m.set_gemm_mode(gemm_mode)
    x = torch.from_numpy(synthetic_batch(frames)[0]).cuda()
    seq = make_seq("uniform", 50, 50)
    b = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3, num_diffusion_timesteps=51)).float()
    out = torch.empty_like(x)
    m.sample(x, seq, b, out=out)                 # warm
    L.dpk_debug_trace(m._h, step, None, 0)
    m.profile(True)
    m.sample(x, seq, b, out=out)
    ms = m.kernel_times_ms()[-1]
    nblk = (frames + 3) // 4
    buf = np.zeros(nblk * 4 * 256, dtype=np.uint64)
    n = L.dpk_debug_trace(m._h, step, buf.ctypes.data, buf.size)
    assert n == buf.size, n
    ne = len(EVENTS)
    t = buf.reshape(nblk, 4, 256)[:, :, :ne].astype(np.int64)
    assert (t > 0).all(), "missing stamps"
    d = np.diff(t, axis=2)                      # interval k ends at event k+1
    step_cyc = float((t[:, :, -1] - t[:, :, 0]).mean())
    # per phase: compute = previous barrier exit -> this barrier entry (slowest wave), split for
    # GEMMs into startup+k-loop / epilogue; wait = barrier entry -> exit
    agg = {}
    for k in range(ne - 1):
        name, kind = EVENTS[k + 1]
        key = name.split(".", 1)[1] if name.startswith("L") and "." in name else name
        part = {"pre": "compute", "post": "wait", "loop": "loop", "epi": "epilogue"}[kind]
        if kind == "loop" and EVENTS[k][1] == "epi":
            part = "loop"                       # next pass of the same GEMM
        if kind == "pre" and EVENTS[k][1] == "epi":
            part = "after_epi"
        a = agg.setdefault(key, {})
        a[part] = a.get(part, 0.0) + float(d[:, :, k].max(1).mean())
    # per-wave view: mean over workgroups of each wave's segments per phase (summed over layers),
    # to expose imbalance between the 4 waves
    perw = {}
    for k in range(ne - 1):
        name, kind = EVENTS[k + 1]
        if kind not in ("pre", "loop", "epi"):
            continue
        key = name.split(".", 1)[1] if name.startswith("L") and "." in name else name
        perw.setdefault(key, np.zeros(4))
        perw[key] += d[:, :, k].mean(0)
    total = sum(sum(v.values()) for v in agg.values())
    print(f"kernel {ms:.3f} ms for {len(seq)} steps; traced step {step}: {step_cyc:.0f} cycles (sum of slowest-wave "
          f"segments {total:.0f}); implied clock {step_cyc / (ms / len(seq) * 1e-3) / 1e9:.2f} GHz")
    cols = ["loop", "epilogue", "after_epi", "compute", "wait"]
    print(f"{'phase':<14}" + "".join(f"{c:>11}" for c in cols) + f"{'total':>10}{'%':>7}")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1].values())):
        tot = sum(v.values())
        print(f"{k:<14}" + "".join(f"{v.get(c, 0):>11.0f}" for c in cols) + f"{tot:>10.0f}{100 * tot / total:>7.1f}")
    print("per-wave compute (loop + epilogue + compute segments, mean over workgroups):")
    for k, v in perw.items():
        print(f"  {k:<14}" + "".join(f"{x:>10.0f}" for x in v) + f"   spread {v.max() - v.min():>7.0f}")
    print(json.dumps({"step_cycles": step_cyc, "phases": {k: {c: round(x, 1) for c, x in v.items()} for k, v in agg.items()}}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--step", type=int, default=10)
    ap.add_argument("--gemm", choices=("fp32", "f16x3", "bf16"), default="fp32")
    ap.add_argument("--so", default=None, help="traced library to run (default build/trace/libdpk_trace.so)")
    a = ap.parse_args()
    if a.so:
        SO = a.so
    if a.build:
        build()
    if a.run:
        run(a.step, gemm_mode=a.gemm)
