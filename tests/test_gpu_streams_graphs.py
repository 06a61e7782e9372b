"""GPU: stream order and graph capture of the C ABI (verdict r01 items 4-5, advisor r01).

The reference loop (common/utils_diff.py:46-68) runs eagerly on one stream; north_star asks
for the K-step loop as a hipGraph.  Here the loop is one persistent launch, and a caller
captures whole steps (bench.py --graph).  These tests pin the semantics diffpose_kernels.h
promises:
  * a captured dpk_sample replays bitwise equal to the eager call;
  * a later dpk_set_schedule (larger K) neither breaks the captured graph (it keeps reading
    the schedule it was captured with) nor the eager call with the new schedule;
  * launches with different schedules on two streams, with no synchronisation between them,
    give the sequential results (the old schedule outlives its in-flight launch);
  * dpk_eps on two streams at once uses one projection buffer per stream.
All comparisons are bitwise: the kernel is deterministic per pose.
"""
import numpy as np
import pytest
import torch

from diffpose_amd.data import synthetic_batch
from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
from diffpose_amd.schedule import get_beta_schedule, make_seq
from diffpose_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu


def _betas(T=51):
    return torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3,
                                              num_diffusion_timesteps=T)).float()


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _model(dev, sd=None):
    m = HipGCNdiff(adj_mx_from_edges(), None, device=dev)
    m.load_state_dict(sd if sd is not None else synthetic_state_dict())
    return m


def test_graph_capture_replays_bitwise(dev):
    m = _model(dev)
    x = torch.from_numpy(synthetic_batch(300, seed=11)[0]).to(dev)
    seq = make_seq("uniform", 50, 10)
    eager = m.sample(x, seq, _betas()).clone()
    out = torch.empty_like(x)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        m.sample(x, seq, _betas(), out=out)
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        m.sample(x, seq, _betas(), out=out)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, eager)
    m.close()


def _capture(dev, m, x, seq, out):
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        m.sample(x, seq, _betas(), out=out)
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        m.sample(x, seq, _betas(), out=out)
    return g


def test_graph_capture_step_split_replays_bitwise(dev):
    """2,560 poses (config 5's per-GPU share): the captured launch runs the step-split last round
    on a flag slot of its own; every replay leaves the flags at 0 for the next, and eager calls
    on the capture stream in between (their own slot) do not disturb it."""
    m = _model(dev)
    x = torch.from_numpy(synthetic_batch(2560, seed=14)[0]).to(dev)
    seq = make_seq("uniform", 50, 10)
    eager = m.sample(x, seq, _betas()).clone()
    m.set_tail_plan("four")
    assert torch.equal(m.sample(x, seq, _betas()), eager)
    m.set_tail_plan("step_split")
    out = torch.empty_like(x)
    g = _capture(dev, m, x, seq, out)
    for _ in range(3):
        out.zero_()
        g.replay()
        assert torch.equal(m.sample(x, seq, _betas()), eager)
        torch.cuda.synchronize()
        assert torch.equal(out, eager)
    del g
    m.close()


def test_step_split_on_three_streams_without_sync(dev):
    """Step-split launches (1,100 poses, 3 schedules) on three streams at once: one flag slot per
    stream, results equal to the sequential ones."""
    m = _model(dev)
    x = torch.from_numpy(synthetic_batch(1100, seed=15)[0]).to(dev)
    seqs = [make_seq("uniform", 50, 50), make_seq("uniform", 50, 10), make_seq("uniform", 50, 25)]
    ref = [_model(dev).sample(x, q, _betas()).clone() for q in seqs]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(device=dev) for _ in seqs]
    outs = [torch.empty_like(x) for _ in seqs]
    for _ in range(2):
        for st, q, o in zip(streams, seqs, outs):
            st.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(st):
                m.sample(x, q, _betas(), out=o)
        torch.cuda.synchronize()
        for o, r in zip(outs, ref):
            assert torch.equal(o, r)
    m.close()


def test_flag_slots_exhausted_fall_back_to_two_pose_tiles(dev):
    """A handle has 64 flag slots; a capture keeps its slot while its graph lives (these graphs all
    stay alive).  Once they are gone a capture runs the 2-pose tail plan instead (bitwise that plan's eager result), and
    the graphs captured earlier still replay the step-split result."""
    m = _model(dev)
    x = torch.from_numpy(synthetic_batch(1100, seed=16)[0]).to(dev)
    seq = make_seq("uniform", 50, 2)
    ref2 = m.sample(x, seq, _betas()).clone()
    m.set_tail_plan("two_pose")
    ref1 = m.sample(x, seq, _betas()).clone()
    m.set_tail_plan("step_split")
    assert not torch.equal(ref1, ref2)
    outs, graphs = [], []
    for _ in range(66):
        outs.append(torch.empty_like(x))
        graphs.append(_capture(dev, m, x, seq, outs[-1]))
    for g, o in zip(graphs, outs):
        o.zero_()
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(outs[0], ref2)
    assert torch.equal(outs[-1], ref1)
    del graphs
    m.close()


def test_set_schedule_after_capture_keeps_graph_and_eager_correct(dev):
    m = _model(dev)
    x = torch.from_numpy(synthetic_batch(64, seed=12)[0]).to(dev)
    seq_a, seq_b = make_seq("uniform", 50, 10), make_seq("uniform", 50, 25)
    ref_a = m.sample(x, seq_a, _betas()).clone()
    ref_b = _model(dev).sample(x, seq_b, _betas()).clone()
    out = torch.empty_like(x)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        m.sample(x, seq_a, _betas(), out=out)
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        m.sample(x, seq_a, _betas(), out=out)
    # a larger K after capture: a new device schedule; the graph keeps the one it captured
    assert torch.equal(m.sample(x, seq_b, _betas()), ref_b)
    for _ in range(2):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, ref_a)
    # and back again: eager with seq_a still matches, and the graph still replays
    assert torch.equal(m.sample(x, seq_a, _betas()), ref_a)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref_a)
    del g
    m.close()


def test_two_streams_two_schedules_without_sync(dev):
    m = _model(dev)
    x = torch.from_numpy(synthetic_batch(1024, seed=13)[0]).to(dev)
    seqs = [make_seq("uniform", 50, 50), make_seq("uniform", 50, 10), make_seq("uniform", 50, 25)]
    ref = [_model(dev).sample(x, q, _betas()).clone() for q in seqs]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(device=dev) for _ in seqs]
    outs = [torch.empty_like(x) for _ in seqs]
    for _ in range(2):
        for st, q, o in zip(streams, seqs, outs):
            st.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(st):          # the K=50 launch is still running when the next
                m.sample(x, q, _betas(), out=o)   # schedule replaces it on the host
        torch.cuda.synchronize()
        for o, r in zip(outs, ref):
            assert torch.equal(o, r)
    m.close()


def test_eps_on_two_streams_without_sync(dev):
    m = _model(dev)
    x = torch.from_numpy(synthetic_batch(1024, seed=14)[0]).to(dev)
    mask = torch.ones(1, 1, 17, dtype=torch.bool, device=dev)
    t1 = torch.full((1024,), 49.0, device=dev)
    t2 = torch.arange(1024, device=dev, dtype=torch.float32) % 50
    r1, r2 = m(x, mask, t1, 0).clone(), m(x, mask, t2, 0).clone()
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    for _ in range(3):
        s1.wait_stream(torch.cuda.current_stream(dev))
        s2.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s1):
            e1 = m(x, mask, t1, 0)
        with torch.cuda.stream(s2):
            e2 = m(x, mask, t2, 0)
        with torch.cuda.stream(s1):
            e1b = m(x, mask, t2, 0)
        torch.cuda.synchronize()
        assert torch.equal(e1, r1) and torch.equal(e2, r2) and torch.equal(e1b, r2)
    m.close()


def test_weights_reload_reaches_captured_graph(dev):
    """Replays read the weight arena by pointer: new weights (and the schedule projections
    recomputed from them) are what the graph computes after dpk_load_weights."""
    sd2 = synthetic_state_dict(seed=7)
    m = _model(dev)
    x = torch.from_numpy(synthetic_batch(40, seed=15)[0]).to(dev)
    seq = make_seq("uniform", 50, 10)
    ref2 = _model(dev, sd2).sample(x, seq, _betas()).clone()
    out = torch.empty_like(x)
    m.sample(x, seq, _betas(), out=out)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        m.sample(x, seq, _betas(), out=out)
    m.load_state_dict(sd2)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref2)
    del g
    m.close()


def test_captured_eps_keeps_its_buffer(dev):
    """advisor r02: a captured dpk_eps owns its projection buffer.  Capture eps at N on a stream,
    then run an uncaptured eps at 2N on that same stream (which grows the stream's own buffer):
    replays still give the eager result."""
    m = _model(dev)
    x = torch.from_numpy(synthetic_batch(256, seed=16)[0]).to(dev)
    mask = torch.ones(1, 1, 17, dtype=torch.bool, device=dev)
    t = (torch.arange(128, device=dev, dtype=torch.float32) * 3) % 50
    t2 = torch.full((256,), 11.0, device=dev)
    eager = m(x[:128].contiguous(), mask, t, 0).clone()
    eager2 = m(x, mask, t2, 0).clone()
    s = torch.cuda.Stream(device=dev)
    xin = x[:128].contiguous()
    out = torch.empty_like(xin)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        out.copy_(m(xin, mask, t, 0))               # uncaptured call: sizes the spare
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        out.copy_(m(xin, mask, t, 0))
    with torch.cuda.stream(s):                      # 2N uncaptured on the capture stream
        big = m(x, mask, t2, 0)
    torch.cuda.synchronize()
    assert torch.equal(big, eager2)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, eager)
    del g
    m.close()


def test_two_eps_graphs_replay_concurrently(dev):
    """Two dpk_eps graphs captured on torch's (shared) capture stream with different timesteps,
    replayed at the same time on two streams: each keeps its own projection buffer."""
    m = _model(dev)
    x = torch.from_numpy(synthetic_batch(512, seed=17)[0]).to(dev)
    mask = torch.ones(1, 1, 17, dtype=torch.bool, device=dev)
    ta = torch.full((512,), 49.0, device=dev)
    tb = torch.arange(512, device=dev, dtype=torch.float32) % 50
    ra, rb = m(x, mask, ta, 0).clone(), m(x, mask, tb, 0).clone()
    oa, ob = torch.empty_like(x), torch.empty_like(x)
    graphs = []
    for t, o in ((ta, oa), (tb, ob)):
        o.copy_(m(x, mask, t, 0))                   # the uncaptured call before each capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            o.copy_(m(x, mask, t, 0))
        graphs.append(g)
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    for _ in range(4):
        oa.zero_()
        ob.zero_()
        torch.cuda.synchronize()
        with torch.cuda.stream(s1):
            graphs[0].replay()
        with torch.cuda.stream(s2):
            graphs[1].replay()
        torch.cuda.synchronize()
        assert torch.equal(oa, ra) and torch.equal(ob, rb)
    del graphs
    m.close()


def test_captured_eps_without_spare_is_refused(dev):
    """Nothing is allocated inside a capture: a captured dpk_eps larger than the spare that the
    uncaptured calls left fails with DPK_E_STATE (and the eager path still works after it)."""
    from diffpose_amd._lib import DpkError

    m = _model(dev)
    x = torch.from_numpy(synthetic_batch(200, seed=18)[0]).to(dev)
    mask = torch.ones(1, 1, 17, dtype=torch.bool, device=dev)
    t = torch.full((200,), 3.0, device=dev)
    m(x[:64].contiguous(), mask, t[:64], 0)           # spare of 64 poses
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with pytest.raises(DpkError) as ei:
        with torch.cuda.graph(g):
            m(x, mask, t, 0)
    assert ei.value.code == -4
    torch.cuda.synchronize()
    ref = _model(dev)(x, mask, t, 0)
    assert torch.equal(m(x, mask, t, 0), ref)
    m.close()


def test_capture_of_an_eps_loop_replays_bitwise(dev):
    """advisor r03 (medium): one capture holding several dpk_eps calls — generalized_steps over a
    plain callable (host loop: model(x, mask, t) then the DDIM update, K=4 steps, so 4 captured
    dpk_eps on one stream).  They share the capture's projection buffer (sequential graph nodes);
    replays equal the eager loop bitwise, and a second capture of the same loop works too."""
    from diffpose_amd import utils_diff

    m = _model(dev)
    x = torch.from_numpy(synthetic_batch(96, seed=19)[0]).to(dev)
    mask = torch.ones(1, 1, 17, dtype=torch.bool, device=dev)
    seq = make_seq("uniform", 50, 4)
    fwd = lambda a, mk, t, c: m(a, mk, t, c)   # noqa: E731  (not a HipGCNdiff: the host-loop path)
    upd = HipGCNdiff.__new__(HipGCNdiff)
    utils_diff._init_schedule_only(upd, dev)
    eager = utils_diff.generalized_steps(x, mask, seq, fwd, _betas(), updater=upd)[0][-1].clone()
    graphs, outs = [], []
    for _ in range(2):
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):                       # warm-up: sizes the spare, sets the schedule
            utils_diff.generalized_steps(x, mask, seq, fwd, _betas(), updater=upd)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        out = torch.empty_like(x)
        with torch.cuda.graph(g):
            out.copy_(utils_diff.generalized_steps(x, mask, seq, fwd, _betas(), updater=upd)[0][-1])
        graphs.append(g)
        outs.append(out)
    for _ in range(3):
        for g, o in zip(graphs, outs):
            o.zero_()
            g.replay()
        torch.cuda.synchronize()
        assert all(torch.equal(o, eager) for o in outs)
    del graphs
    upd.close()
    m.close()


def test_capture_resources_follow_the_graph(dev, monkeypatch):
    """A capture hands its graph a HIP user object (DPK_CAPTURE_RELEASE, default 1): the schedule, the
    dpk_eps buffer and the step-split flag slot the captured launches read stay held while the graph
    (or its executable) lives — torch.cuda.CUDAGraph keeps only the executable after capture — and
    are recycled by the next uncaptured call once it is destroyed.  Probe of the runtime's user-object
    semantics: released must stay 0 until the graph is gone."""
    import gc

    monkeypatch.setenv("DPK_CAPTURE_RELEASE", "1")
    m = _model(dev)
    x = torch.from_numpy(synthetic_batch(1100, seed=20)[0]).to(dev)
    mask = torch.ones(1, 1, 17, dtype=torch.bool, device=dev)
    t = torch.full((1100,), 7.0, device=dev)
    seq = make_seq("uniform", 50, 4)
    eager = m.sample(x, seq, _betas(), mask=mask).clone()
    eager_eps = m(x, mask, t, 0).clone()
    torch.cuda.synchronize()
    free0 = m.debug_resources()["free_slots"]
    out, eo = torch.empty_like(x), torch.empty_like(x)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):                     # the same mask object: no mask upload inside the capture
        m.sample(x, seq, _betas(), mask=mask, out=out)
        eo.copy_(m(x, mask, t, 0))
    r1 = m.debug_resources()
    print("\nafter capture:", r1)
    if r1["tracked"] == 0:
        pytest.skip("the runtime did not retain the user object (resources kept until dpk_destroy)")
    assert r1["captures"] == 1 and r1["released"] == 0, r1
    for _ in range(2):
        out.zero_()
        eo.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, eager) and torch.equal(eo, eager_eps)
    assert m.debug_resources()["released"] == 0
    del g
    gc.collect()
    torch.cuda.synchronize()
    import time

    for _ in range(100):                  # the runtime may run the destructor on its own thread
        r2 = m.debug_resources()
        if r2["released"]:
            break
        time.sleep(0.01)
    print("graph destroyed:", r2)
    assert r2["released"] == 1, r2
    assert torch.equal(m.sample(x, seq, _betas(), mask=mask), eager)     # recycles them
    torch.cuda.synchronize()
    r3 = m.debug_resources()
    print("after the next call:", r3)
    assert r3["captures"] == 0 and r3["free_slots"] >= free0 - 1 and r3["eps_spare_poses"] >= 1100
    m.close()


def test_sweep_while_another_thread_captures(dev, monkeypatch):
    """advisor r04: handle B's uncaptured dpk_sample recycles a released capture's resources (cap_sweep)
    while thread A holds a global-mode capture open (torch.cuda.graph's default) on handle A.  cap_sweep
    does not drain the device (a hipDeviceSynchronize there, even in relaxed capture mode, invalidates A's
    capture on this runtime: round 6 measured it); it relies on graph destruction waiting for in-flight
    replays (tools/probe_user_object_release.py).  A's capture must complete and replay bitwise, and B's
    launch gives the eager result."""
    import gc
    import threading
    import time

    monkeypatch.setenv("DPK_CAPTURE_RELEASE", "1")
    mA, mB = _model(dev), _model(dev)
    x = torch.from_numpy(synthetic_batch(64, seed=23)[0]).to(dev)
    mask = torch.ones(1, 1, 17, dtype=torch.bool, device=dev)
    seq = make_seq("uniform", 50, 4)
    eager = mA.sample(x, seq, _betas(), mask=mask).clone()
    assert torch.equal(mB.sample(x, seq, _betas(), mask=mask), eager)
    # B: a capture whose graph is destroyed, so B's next uncaptured call has a release to sweep
    outB = torch.empty_like(x)
    gB = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gB):
        mB.sample(x, seq, _betas(), mask=mask, out=outB)
    if mB.debug_resources()["tracked"] == 0:
        pytest.skip("the runtime did not retain the user object (nothing is swept)")
    del gB
    gc.collect()
    torch.cuda.synchronize()
    for _ in range(100):
        if mB.debug_resources()["released"]:
            break
        time.sleep(0.01)
    assert mB.debug_resources()["released"] == 1
    # A: warm up on the capture's side stream, then hold the capture open while B sweeps
    sA = torch.cuda.Stream(device=dev)
    sA.wait_stream(torch.cuda.current_stream(dev))
    outA = torch.empty_like(x)
    with torch.cuda.stream(sA):
        mA.sample(x, seq, _betas(), mask=mask, out=outA)
    torch.cuda.current_stream(dev).wait_stream(sA)
    torch.cuda.synchronize()
    sB = torch.cuda.Stream(device=dev)
    resB = torch.empty_like(x)
    opened, done = threading.Event(), threading.Event()
    errs = []

    def thread_b():
        try:
            assert opened.wait(60)
            with torch.cuda.device(dev), torch.cuda.stream(sB):
                mB.sample(x, seq, _betas(), mask=mask, out=resB)    # preallocated: no allocator call
        except Exception as e:  # surfaced below
            errs.append(repr(e))
        finally:
            done.set()

    tb = threading.Thread(target=thread_b)
    tb.start()
    gA = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gA):
        mA.sample(x, seq, _betas(), mask=mask, out=outA)
        opened.set()
        assert done.wait(120)
    tb.join(60)
    assert not errs, errs
    torch.cuda.synchronize()
    assert torch.equal(resB, eager)
    outA.zero_()
    gA.replay()
    torch.cuda.synchronize()
    assert torch.equal(outA, eager)
    assert mB.debug_resources()["released"] == 0     # B's call recycled the release
    mB.sample(x, seq, _betas(), mask=mask)
    assert mB.debug_resources()["released"] == 0
    del gA
    mA.close()
    mB.close()
