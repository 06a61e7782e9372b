"""Time the golden-pinned CPU oracle beside the imported reference (build container only).

SURVEY §8d: the GPU box cannot run the reference (it does not travel), so bench.py's
cpu_baseline times the oracle there.  This script shows, in the container where both exist,
that the two run at the same speed on the same inputs: the reference's generalized_steps +
GCNdiff (models/gcndiff.py, common/utils_diff.py) and oracle/gcndiff_oracle.py, same weights,
same frames, same K, same torch thread count, best of --repeats after one untimed warm-up call.

  PYTHONPATH=/root/reference python tools/cpu_speed_compare.py [--frames 128 --K 10 --threads 8]
"""
import argparse
import os
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diffpose-nw_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--frames", type=int, default=128)
    ap.add_argument("--K", type=int, default=10)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--repeats", type=int, default=3)
    args = ap.parse_args()
    sys.path.insert(0, args.ref)
    sys.dont_write_bytecode = True
    import torch

    torch.Tensor.cuda = lambda self, *a, **k: self          # the reference hard-codes .cuda()
    torch.set_num_threads(args.threads)
    from models.gcndiff import GCNdiff
    from models.GraFormer import adj_mx_from_edges
    from common.utils_diff import generalized_steps

    from diffpose_amd.data import synthetic_batch
    from diffpose_amd.schedule import get_beta_schedule, make_seq
    from diffpose_amd.weights import synthetic_state_dict
    from oracle import gcndiff_oracle as O

    cfg = types.SimpleNamespace(model=types.SimpleNamespace(
        hid_dim=96, emd_dim=96, coords_dim=[5, 5], num_layer=5, n_head=4, dropout=0.25, n_pts=17))
    edges = torch.tensor([[0, 1], [1, 2], [2, 3], [0, 4], [4, 5], [5, 6], [0, 7], [7, 8], [8, 9], [9, 10],
                          [8, 11], [11, 12], [12, 13], [8, 14], [14, 15], [15, 16]], dtype=torch.long)
    adj = adj_mx_from_edges(num_pts=17, edges=edges, sparse=False)
    sd = synthetic_state_dict()
    model = GCNdiff(adj, cfg)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model.eval()
    P, oadj = O.params_to_torch(sd), O.adjacency()
    mask = torch.ones(1, 1, 17, dtype=torch.bool)
    x = torch.from_numpy(synthetic_batch(args.frames)[0])
    seq = make_seq("uniform", 50, args.K) if 50 % args.K == 0 else list(range(args.K))
    b = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                           num_diffusion_timesteps=51)).float()

    def ref_run(xx):
        return generalized_steps(xx, mask, seq, model, b, eta=0.0)[0][-1]

    def ora_run(xx):
        return O.generalized_steps(xx, mask, seq, lambda a, m, t: O.gcndiff_forward(P, oadj, a, m, t), b)[0][-1]

    res = {}
    outs = {}
    for name, fn in (("reference", ref_run), ("oracle", ora_run)):
        fn(x[:8])
        ts = []
        for _ in range(args.repeats):
            t0 = time.perf_counter()
            outs[name] = fn(x)
            ts.append(time.perf_counter() - t0)
        res[name] = ts
    same = torch.equal(outs["reference"], outs["oracle"])
    cpu = "unknown"
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            cpu = line.split(":", 1)[1].strip()
            break
    print(f"host '{cpu}', torch {torch.__version__}, {args.threads} threads; {args.frames} frames x K={args.K}")
    for name, ts in res.items():
        best = min(ts)
        print(f"{name:10s} best {best:.3f} s -> {args.frames / best * args.K / 50:.1f} poses/s at K=50 "
              f"(runs: {', '.join(f'{t:.3f}' for t in ts)})")
    print(f"ratio oracle/reference time: {min(res['oracle']) / min(res['reference']):.3f}; outputs bit-identical: {same}")


if __name__ == "__main__":
    main()
