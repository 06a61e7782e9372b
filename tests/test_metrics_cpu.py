"""CPU: the metrics oracle against the reference's golden vectors (g7), and the product's
host-side per-action accounting (diffpose_amd.metrics) against the reference's own
test_calculation / print_error results on the same per-frame errors."""
import numpy as np
import torch

from oracle import metrics_oracle as M
from diffpose_amd import metrics


def test_oracle_metrics_match_reference(golden):
    g = golden("g7_metrics.npz")
    pred, tgt = g["pred"], g["tgt"]
    assert np.array_equal(M.p_mpjpe_per_pose(pred.copy(), tgt.copy()), g["per_pose_p2"])
    assert M.p_mpjpe(pred.copy(), tgt.copy()) == g["loss_p2"]
    assert M.mpjpe(torch.from_numpy(pred), torch.from_numpy(tgt)).item() == g["loss_p1"]


def _book(g):
    pred, tgt = g["pred"], g["tgt"]
    acts = [str(a) for a in g["actions"]]
    err = metrics.define_error_list(metrics.TEST_ACTIONS)
    for lo, hi in g["bounds"]:
        p1 = M.mpjpe_per_pose(torch.from_numpy(pred[lo:hi]), torch.from_numpy(tgt[lo:hi])).double().numpy()
        p2 = M.p_mpjpe_per_pose(pred[lo:hi].copy(), tgt[lo:hi].copy()).astype(np.float64)
        metrics.test_calculation(p1, p2, acts[lo:hi], err)
    return err


def test_action_accounting_matches_reference(golden):
    g = golden("g7_metrics.npz")
    err = _book(g)
    assert list(g["action_names"]) == metrics.TEST_ACTIONS
    for i, a in enumerate(metrics.TEST_ACTIONS):
        assert abs(err[a]["p1"].avg - g["action_p1"][i]) <= 1e-6 * max(1.0, g["action_p1"][i])
        assert abs(err[a]["p2"].avg - g["action_p2"][i]) <= 1e-6 * max(1.0, g["action_p2"][i])
    p1, p2 = metrics.print_error(None, err, 1)
    # the reference books fp32 torch scalars; ours books float64 of the same per-frame values
    assert abs(p1 - float(g["p1"])) <= 1e-4 and abs(p2 - float(g["p2"])) <= 1e-4
    assert err["SittingDown"]["p1"].count == 0          # unseen action still averaged in as 0


def test_action_helpers():
    assert metrics.action_name("Walking 1") == "Walking" and metrics.action_name("Photo") == "Photo"
    assert metrics.define_actions("All") == metrics.TEST_ACTIONS
    assert metrics.define_actions("Eating") == ["Eating"]
    import pytest

    with pytest.raises(ValueError):
        metrics.define_actions("Dancing")
    with pytest.raises(ValueError):
        metrics.test_calculation(np.zeros(2), np.zeros(2), ["Eating"], metrics.define_error_list(["Eating"]))
