"""Probe (GPU box): when does HIP run a graph's user-object release callback relative to an in-flight
replay?  A captured dpk_sample (long: K=100 over 4,096 poses) is replayed asynchronously and the graph is
destroyed at once; the handle's capture-resource counters (dpk_debug_resources: `released`) are read
before the replay can have finished.  released = 1 while the replay's event is still pending means the
runtime releases early (the handle must drain the device before recycling); 0 until completion means
it defers the release to the end of the launches, as CUDA documents for cudaGraphExecDestroy."""
import gc
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "diffpose-nw_amd"), ROOT]
import torch  # noqa: E402

from diffpose_amd.data import synthetic_batch  # noqa: E402
from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges  # noqa: E402
from diffpose_amd.schedule import get_beta_schedule, make_seq  # noqa: E402
from diffpose_amd.weights import synthetic_state_dict  # noqa: E402

os.environ["DPK_CAPTURE_RELEASE"] = "1"
dev = torch.device("cuda", 0)
m = HipGCNdiff(adj_mx_from_edges(), None, device=dev)
m.load_state_dict(synthetic_state_dict())
x = torch.from_numpy(synthetic_batch(8192, seed=1)[0]).to(dev)
b = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3, num_diffusion_timesteps=101)).float()
seq = make_seq("uniform", 100, 100)
out = torch.empty_like(x)
s = torch.cuda.Stream(device=dev)
s.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(s):
    m.sample(x, seq, b, out=out)
torch.cuda.current_stream(dev).wait_stream(s)
torch.cuda.synchronize()
for trial in range(3):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        m.sample(x, seq, b, out=out)
    r0 = m.debug_resources()
    done = torch.cuda.Event()
    t0 = time.perf_counter()
    g.replay()
    done.record()
    t_rep = (time.perf_counter() - t0) * 1e3
    pending0 = not done.query()
    del g
    t_del = (time.perf_counter() - t0) * 1e3
    gc.collect()
    t_gc = (time.perf_counter() - t0) * 1e3
    pending1 = not done.query()
    rel1 = m.debug_resources()["released"]
    print(f"  replay enqueued at {t_rep:.1f} ms (pending {pending0}); graph deleted at {t_del:.1f} ms, gc done at "
          f"{t_gc:.1f} ms: replay still pending {pending1}, released {rel1}")
    seen = []
    while not done.query():
        seen.append((round((time.perf_counter() - t0) * 1e3, 2), m.debug_resources()["released"]))
        time.sleep(0.002)
    t_done = (time.perf_counter() - t0) * 1e3
    after = m.debug_resources()["released"]
    early = [t for t, r in seen if r]
    print(f"trial {trial}: tracked {r0['tracked']}; replay done after {t_done:.1f} ms; polls while in flight {len(seen)}; "
          f"released while in flight: {'YES at %.1f ms' % early[0] if early else 'no'}; released after: {after}")
    m.sample(x[:8].contiguous(), seq, b)     # an uncaptured call recycles it
    torch.cuda.synchronize()
