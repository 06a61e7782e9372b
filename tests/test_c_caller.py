"""The C ABI from plain C (tests/c/dpk_c_caller.c: gcc, include/diffpose_kernels.h only, no Python
or HIP headers), the binding INTEGRATION.md §4 shows.  CPU: the header compiles as C11 with
-Wall -Wextra -Werror and the program links against libdpk.so.  GPU: the C caller runs the sampler
on 1,100 poses (the step-split last round, plans 2 and 0 bitwise equal inside the C program) and
matches the Python HipGCNdiff path on the same inputs within the fp32 bar."""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c", "dpk_c_caller.c")
LIBDIR = os.path.join(ROOT, "diffpose-nw_amd", "diffpose_amd")
PREBUILT = os.path.join(ROOT, "build", "c", "dpk_c_caller")


def _compile(out):
    subprocess.run(["gcc", "-std=c11", "-O2", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"), SRC,
                    "-L", LIBDIR, "-ldpk", "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{LIBDIR}",
                    "-Wl,-rpath,/opt/rocm/lib", "-o", str(out)], check=True, capture_output=True, text=True)


def test_c_caller_compiles_and_links(tmp_path):
    if not shutil.which("gcc") or not os.path.exists(os.path.join(LIBDIR, "libdpk.so")):
        pytest.skip("gcc or libdpk.so missing")
    _compile(tmp_path / "dpk_c_caller")
    assert os.path.getsize(tmp_path / "dpk_c_caller") > 0


def _write_weights(path, sd):
    with open(path, "wb") as f:
        f.write(struct.pack("<i", len(sd)))
        for k, v in sd.items():
            a = np.ascontiguousarray(v, dtype="<f4").ravel()
            f.write(struct.pack("<i", len(k)))
            f.write(k.encode())
            f.write(struct.pack("<q", a.size))
            f.write(a.tobytes())


@pytest.mark.gpu
def test_c_caller_runs_the_sampler(tmp_path):
    import torch

    from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges
    from diffpose_amd.schedule import get_beta_schedule, make_seq
    from diffpose_amd.weights import synthetic_state_dict

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    exe = PREBUILT if os.path.exists(PREBUILT) else str(tmp_path / "dpk_c_caller")
    if exe != PREBUILT:
        _compile(exe)
    sd = synthetic_state_dict()
    _write_weights(tmp_path / "w.bin", sd)
    n, k = 1100, 10
    p = subprocess.run([exe, str(tmp_path / "w.bin"), str(n), str(k), str(tmp_path / "out.bin")],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    raw = open(tmp_path / "out.bin", "rb").read()
    assert struct.unpack_from("<i", raw, 0)[0] == n
    x = np.frombuffer(raw, "<f4", n * 85, 4).reshape(n, 17, 5)
    out_c = np.frombuffer(raw, "<f4", n * 85, 4 + n * 340).reshape(n, 17, 5)
    assert struct.unpack_from("<i", raw, 4 + 2 * n * 340)[0] == 1          # plan 2 == plan 0 bitwise
    m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
    m.load_state_dict(sd)
    b = torch.from_numpy(get_beta_schedule("linear", beta_start=1e-4, beta_end=1e-3, num_diffusion_timesteps=51)).float()
    seq = make_seq("uniform", 50, k)
    out_py = m.sample(torch.from_numpy(x.copy()).cuda(), seq, b).cpu().numpy()
    m.close()
    # the same kernel on the same inputs and schedule tables: bitwise
    assert np.array_equal(out_py, out_c), float(np.abs(out_py.astype(np.float64) - out_c).max())
    # and parity proper: frames from every tile kind (full rounds, the step-split last round) vs the oracle
    from conftest import record_delta
    from oracle import gcndiff_oracle as O

    sel = np.array([0, 1, 2, 3, 517, 1023, 1024, 1025, 1060, 1097, 1098, 1099])
    P, adj = O.params_to_torch(sd), O.adjacency()
    xs, _ = O.generalized_steps(torch.from_numpy(x[sel].copy()), torch.ones(1, 1, 17, dtype=torch.bool), seq,
                                lambda a_, m_, t_: O.gcndiff_forward(P, adj, a_, m_, t_), b)
    assert record_delta(float(np.abs(out_c[sel].astype(np.float64) - xs[-1].double().numpy()).max()), 5e-6)
