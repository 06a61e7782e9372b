"""Diffusion schedule: betas, the fp32 cumulative-alpha table, the skip sequence.

Restates, in host NumPy, the schedule pieces the reference evaluates per step:

* ``get_beta_schedule`` — reference ``common/utils_diff.py:7-37`` (fp64, five kinds);
  the runner casts the result to fp32 (``runners/diffpose_frame.py:43-49``).
* ``alpha_bar_table`` — the table ``compute_alpha`` (``common/utils_diff.py:40-43``)
  indexes: ``cumprod(1 - cat([0], beta))`` evaluated in fp32, sequentially, exactly
  as the CPU reference does.  Entry ``t+1`` is ᾱ_t; entry 0 is 1.
* ``make_seq`` — the timestep sequence of ``test_hyber`` (``runners/diffpose_frame.py:310-317``).
* ``ddim_coeffs`` — the per-step scalars of ``generalized_steps``
  (``common/utils_diff.py:55-65``) in fp32, same operation order.
"""
from __future__ import annotations

import numpy as np


def get_beta_schedule(beta_schedule: str, *, beta_start: float, beta_end: float,
                      num_diffusion_timesteps: int) -> np.ndarray:
    """fp64 betas (reference common/utils_diff.py:7-37)."""
    T = int(num_diffusion_timesteps)
    if beta_schedule == "quad":
        betas = np.linspace(beta_start ** 0.5, beta_end ** 0.5, T, dtype=np.float64) ** 2
    elif beta_schedule == "linear":
        betas = np.linspace(beta_start, beta_end, T, dtype=np.float64)
    elif beta_schedule == "const":
        betas = beta_end * np.ones(T, dtype=np.float64)
    elif beta_schedule == "jsd":
        betas = 1.0 / np.linspace(T, 1, T, dtype=np.float64)
    elif beta_schedule == "sigmoid":
        x = np.linspace(-6, 6, T)
        betas = (1.0 / (np.exp(-x) + 1.0)) * (beta_end - beta_start) + beta_start
    else:
        raise NotImplementedError(beta_schedule)
    assert betas.shape == (T,)
    return betas


def alpha_bar_table(betas) -> np.ndarray:
    """fp32 table a[0..T] of ``(1 - cat([0], beta)).cumprod(0)`` (common/utils_diff.py:41-42).

    The factors ``1 - beta`` are fp32; torch's CPU cumprod carries the running
    product in double (``acc_type<float, /*cuda=*/false>``) and rounds each
    output to fp32 — reproduced here so the table is bit-identical.
    """
    b = np.asarray(betas, dtype=np.float32)
    factors = np.concatenate([np.ones(1, np.float32), (np.float32(1.0) - b).astype(np.float32)])
    out = np.empty(factors.shape[0], dtype=np.float32)
    acc = 1.0
    for k in range(factors.shape[0]):
        acc = acc * float(factors[k])
        out[k] = np.float32(acc)
    return out


def make_seq(skip_type: str, test_num_diffusion_timesteps: int, test_timesteps: int):
    """Timestep sequence of test_hyber (runners/diffpose_frame.py:310-317)."""
    if skip_type == "uniform":
        skip = test_num_diffusion_timesteps // test_timesteps
        return list(range(0, test_num_diffusion_timesteps, skip))
    if skip_type == "quad":
        seq = np.linspace(0, np.sqrt(test_num_diffusion_timesteps * 0.8), test_timesteps) ** 2
        return [int(s) for s in list(seq)]
    raise NotImplementedError(skip_type)


def step_pairs(seq):
    """(t, next_t) in execution order (common/utils_diff.py:49-52)."""
    seq = list(seq)
    seq_next = [-1] + seq[:-1]
    return list(zip(reversed(seq), reversed(seq_next)))


def ddim_coeffs(abar: np.ndarray, seq, eta: float = 0.0) -> np.ndarray:
    """Per-step fp32 scalars [K, 6] = (sqrt(1-at), sqrt(at), sqrt(an), c1, c2, t).

    Evaluated in fp32 in the reference's operation order
    (common/utils_diff.py:59-65); ``at``=ᾱ[t+1], ``an``=ᾱ[next_t+1].
    """
    f = np.float32
    T1 = abar.shape[0]
    rows = []
    for t, tn in step_pairs(seq):
        if not (0 <= t + 1 < T1 and 0 <= tn + 1 < T1):
            raise IndexError(f"timestep {t} / {tn} outside the alpha table of {T1} entries")
        at, an = f(abar[t + 1]), f(abar[tn + 1])
        s1a = f(np.sqrt(f(f(1) - at)))
        sa = f(np.sqrt(at))
        san = f(np.sqrt(an))
        inner = f(f(f(f(1) - f(at / an)) * f(f(1) - an)) / f(f(1) - at))
        c1 = f(f(eta) * f(np.sqrt(inner)))
        c2 = f(np.sqrt(f(f(f(1) - an) - f(c1 * c1))))
        rows.append((s1a, sa, san, c1, c2, f(t)))
    return np.asarray(rows, dtype=np.float32).reshape(-1, 6)
