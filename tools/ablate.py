"""Phase-ablation timing for the sampler kernel (timing-only builds; outputs are wrong).

  python tools/ablate.py --build          # in the build container: hipcc one .so per mask
  python tools/ablate.py --run            # on the GPU box: time each variant (B=1024, K=50)

Mask bits (DPK_ABLATE in csrc/dpk_kernels.hip): 1 attention, 2 GraphNet graph products,
4 Chebyshev T1/T2 products, 8 LayerNorm, 16 the six per-layer GEMMs; single GEMMs:
32 QKV, 64 O-proj, 128 fc1, 256 fc2, 512 Cheb1, 1024 Cheb2.  DPK_MASKS=a,b,c selects masks.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build", "ablate")
MASKS = [int(m) for m in os.environ.get("DPK_MASKS", "0,1,2,4,8,16,15,31").split(",")]
EXTRA = os.environ.get("DPK_ABLATE_EXTRA", "")


def build():
    from concurrent.futures import ThreadPoolExecutor

    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(ROOT, "diffpose-nw_amd", "csrc", "dpk_kernels.hip")

    def one(m):
        so = os.path.join(OUT, f"libdpk_a{m}.so")
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-ffp-contract=off", "-Wno-unused-result", f"-I{ROOT}/include", f"-DDPK_ABLATE={m}", src,
               "-o", so] + EXTRA.split()
        subprocess.run(cmd, check=True, capture_output=True)
        return so

    with ThreadPoolExecutor(max_workers=min(6, os.cpu_count() or 1)) as ex:
        for so in ex.map(one, MASKS):
            print("built", so)


def time_one(reps=5):
    sys.path.insert(0, os.path.join(ROOT, "diffpose-nw_amd"))
    import torch
    from diffpose_amd.data import synthetic_batch
    from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
    from diffpose_amd.schedule import get_beta_schedule, make_seq
    from diffpose_amd.weights import synthetic_state_dict

    m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
    m.load_state_dict(synthetic_state_dict())
    x = torch.from_numpy(synthetic_batch(1024)[0]).cuda()
    seq = make_seq("uniform", 50, 50)
    b = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3, num_diffusion_timesteps=51)).float()
    out = torch.empty_like(x)
    m.sample(x, seq, b, out=out)
    torch.cuda.synchronize()
    m.profile(True)
    for _ in range(reps):
        m.sample(x, seq, b, out=out)
    ts = m.kernel_times_ms()
    return min(ts), sum(ts) / len(ts)


def run():
    res = {}
    names = os.environ.get("DPK_LIBS")
    libs = names.split(",") if names else [f"libdpk_a{m}.so" for m in MASKS]
    for m in libs:
        so = os.path.join(OUT, m)
        env = dict(os.environ, DPK_LIB=so)
        r = subprocess.run([sys.executable, __file__, "--time"], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(r.stderr[-2000:])
            raise SystemExit(r.returncode)
        res[m] = json.loads(r.stdout.strip().splitlines()[-1])
        print(m, res[m], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--time", action="store_true")
    a = ap.parse_args()
    if a.build:
        build()
    if a.run:
        run()
    if a.time:
        mn, avg = time_one()
        print(json.dumps({"min_ms": round(mn, 3), "avg_ms": round(avg, 3)}))
