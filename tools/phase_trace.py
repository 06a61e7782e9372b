"""Per-phase cycle breakdown of one DDIM step of the sampler kernel.

Uses a trace build of libdpk (-DDPK_TRACE=1). In that build, lane 0 of every wave stamps
s_memtime before and after each workgroup barrier of one chosen step. Per phase it reports:
- wall: the barrier-exit to barrier-exit delta, averaged over workgroups;
- the slowest and the fastest wave's compute time up to the barrier.
Each phase type is summed over the 5 layers.

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
SO = os.path.join(ROOT, "build", "trace", "libdpk_trace.so")

LAYER = ["LN0", "QKV", "attention", "O", "LN1", "graph1", "fc1", "fc2", "graph2+b2", "cheb_prep1", "C1",
         "cheb_prep2", "C2"]
NAMES = ["input_prep", "input_gemm"] + [f"L{l}.{n}" for l in range(5) for n in LAYER] + ["cheb_out", "out_gemm+ddim"]


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = [os.path.join(ROOT, "diffpose-nw_amd", "csrc", f) for f in ("dpk_kernels.hip", "dpk_metrics.hip")]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-ffp-contract=off", "-fno-slp-vectorize", "-Wno-unused-result", f"-I{ROOT}/include", "-DDPK_TRACE=1"] + src + ["-o", SO]
    cmd += os.environ.get("DPK_TRACE_EXTRA", "").split()
    subprocess.run(cmd, check=True)
    print("built", SO)


def run(step=10, frames=1024):
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
    t = buf.reshape(nblk, 4, 256).astype(np.int64)
    nb = len(NAMES)
    pre = t[:, :, 0:2 * nb:2]          # before barrier p
    post = t[:, :, 1:2 * nb:2]         # after barrier p
    assert (pre > 0).all() and (post > 0).all(), "missing stamps"
    step_cyc = (post[:, :, -1] - post[:, :, 0]).mean()
    rows = []
    for p in range(1, nb):
        wall = (post[:, 0, p] - post[:, 0, p - 1]).mean()
        comp = pre[:, :, p] - post[:, :, p - 1]
        rows.append((NAMES[p], wall, comp.max(1).mean(), comp.min(1).mean()))
    agg = {}
    for name, wall, cmax, cmin in rows:
        key = name.split(".", 1)[1] if name.startswith("L") else name
        a = agg.setdefault(key, [0.0, 0.0, 0.0])
        a[0] += wall
        a[1] += cmax
        a[2] += cmin
    total = sum(v[0] for v in agg.values())
    print(f"kernel {ms:.3f} ms for {len(seq)} steps; traced step {step}: {step_cyc:.0f} cycles "
          f"(sum of phases {total:.0f}); implied clock {step_cyc / (ms / len(seq) * 1e-3) / 1e9:.2f} GHz")
    print(f"{'phase':<14}{'wall cyc':>10}{'%':>7}{'max wave':>10}{'min wave':>10}")
    for k, (w, cmax, cmin) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print(f"{k:<14}{w:>10.0f}{100 * w / total:>7.1f}{cmax:>10.0f}{cmin:>10.0f}")
    print(json.dumps({"step_cycles": float(step_cyc), "phases": {k: [round(v, 1) for v in vals] for k, vals in agg.items()}}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--step", type=int, default=10)
    a = ap.parse_args()
    if a.build:
        build()
    if a.run:
        run(a.step)
