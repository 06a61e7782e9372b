"""CPU: the C-ABI library builds, loads and exports every symbol include/*.h declares.

No compute call is made here (there is no GPU in the build container); argument
validation paths that return before touching the device are exercised.
"""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT
from diffpose_amd import _lib

HEADER = os.path.join(ROOT, "include", "diffpose_kernels.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dpk_[a-z0-9_]+)\s*\(", src)))


def test_library_exists():
    assert os.path.exists(_lib.LIB_PATH), "run `python __graft_entry__.py` (build) first"


def test_exports_match_header():
    decl = declared_functions()
    assert set(decl) == set(_lib.EXPORTS)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    syms = set(re.findall(r"\bT (dpk_\w+)", out))
    missing = [d for d in decl if d not in syms]
    assert not missing, f"not exported: {missing}"


def test_load_and_query_without_gpu():
    L = _lib.lib()
    assert L.dpk_version() >= 100
    g = _lib.kernel_geometry()
    assert g["poses_per_workgroup"] >= 1 and g["threads_per_workgroup"] % 64 == 0
    assert 0 < g["lds_bytes"] <= 160 * 1024


def test_argument_validation_without_gpu():
    L = _lib.lib()
    h = ctypes.c_void_p()
    assert L.dpk_create(None, ctypes.byref(h)) == -1
    # shapes outside what either path runs are refused before any device call (DPK_E_UNSUPPORTED);
    # other shapes than the compiled one (hid 96, 4 heads, 17 joints) pass to the generic path and
    # only then need a device (none here: DPK_E_HIP)
    for cfg, rc in (((100, 5, 8, 17, 5, 5), -2),      # hid_dim not a multiple of n_head
                    ((96, 5, 4, 40, 5, 5), -2),       # more than 32 joints (one mask word per pose)
                    ((96, 5, 4, 17, 3, 4), -2),       # GCNdiff needs coords in == out (or GCNpose's 2 -> 3)
                    ((128, 5, 4, 17, 5, 5), -3),      # generic path: another hid_dim
                    ((96, 5, 4, 17, 3, 3), -3)):      # generic path: other coords
        c = _lib.DpkConfig(*cfg, 0)
        assert L.dpk_create(ctypes.byref(c), ctypes.byref(h)) == rc, cfg
    assert L.dpk_eps(None, None, None, None, 0, None) == -1
    assert L.dpk_last_error(None) == b"null handle"
    assert L.dpk_pose(None, None, None, None, 0, 1, 0, None) == -1
    assert L.dpk_set_pose_masks(None, None, 0) == -1
    # num_layers is a run-time value (config num_layer): 1..5 on the compiled sampler, more on the
    # generic path; 0 is rejected before any device call, 3 and 6 pass the shape check and only then
    # need a device (none here: DPK_E_HIP)
    for nl, rc in ((0, -2), (6, -3), (3, -3)):
        cfg = _lib.DpkConfig(96, nl, 4, 17, 5, 5, 0)
        assert L.dpk_create(ctypes.byref(cfg), ctypes.byref(h)) == rc, nl
    # metrics entry validates before launching: negative F, H < 1, unknown root mode, null outputs
    assert L.dpk_pose_metrics(None, None, -1, 1, 0, None, None, None, None) == -1
    assert L.dpk_pose_metrics(None, None, 4, 0, 0, None, None, None, None) == -1
    assert L.dpk_pose_metrics(None, None, 4, 1, 3, None, None, None, None) == -1
    assert L.dpk_pose_metrics(None, None, 4, 1, 0, None, None, None, None) == -1
    assert L.dpk_pose_metrics(None, None, 0, 1, 0, None, None, None, None) == 0


def test_no_oracle_in_product_path():
    pkg = os.path.join(ROOT, "diffpose-nw_amd")
    for dp, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                txt = open(os.path.join(dp, f)).read()
                assert "oracle" not in re.sub(r"#.*|//.*", "", txt).replace("no oracle", ""), f


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_lib, "_LIB", None)
    with pytest.raises(ImportError):
        _lib.lib()
