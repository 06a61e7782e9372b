"""Drop-in ``common/utils_diff.py``: get_beta_schedule, compute_alpha, generalized_steps.

``generalized_steps(x, src_mask, seq, model, b, **kwargs) -> (xs, x0_preds)`` keeps
the reference signature and return shape (reference ``common/utils_diff.py:46-68``):
``xs`` is a list of K+1 tensors whose first element IS the input object, and
``x0_preds`` a list of K tensors.

* ``model`` a :class:`HipGCNdiff` → the whole loop runs as one persistent HIP kernel
  (``dpk_sample``) writing the trajectory into two preallocated stacks.
* any other callable ``model(xt, mask, t, cemd)`` → the loop runs on the host, each
  step's DDIM update in the HIP ``dpk_ddim_update`` kernel.

The noise of ``c1 * randn`` (eta > 0).  The reference draws ``torch.randn_like(x)`` once per step,
in execution order (``common/utils_diff.py:65``); ``noise=`` selects what z is:

* ``"torch"`` (the default when eta > 0): the same K draws, ``torch.randn_like(x)`` on x's
  device from torch's default generator, so the trajectory is the reference's under the same seed;
* ``"torch-cpu"``: the K draws from the CPU generator (the reference run on a CPU), uploaded;
* ``"philox"``: counter-based draws inside the kernel, keyed by (``seed``, step, element) — no
  [K,N,17,5] buffer, not the reference's numbers;
* a [K,N,17,5] tensor: slice k is step k's z.

At eta = 0 the noise term is 0·z and nothing is drawn unless ``noise`` asks for it (the reference
still advances torch's RNG by K draws there; ``noise="torch"`` reproduces that too).
"""
from __future__ import annotations

import threading

import numpy as np

import torch

from .gcndiff import HipGCNdiff
from .schedule import alpha_bar_table, get_beta_schedule, step_pairs  # noqa: F401  (re-exported)


def compute_alpha(beta, t):
    """(1 - cat([0], beta)).cumprod(0)[t+1] as (N,1,1) (common/utils_diff.py:40-43); host table."""
    b = beta.detach().cpu().numpy() if torch.is_tensor(beta) else np.asarray(beta)
    table = torch.from_numpy(alpha_bar_table(b))
    idx = torch.as_tensor(t).long().cpu() + 1
    out = table.index_select(0, idx).view(-1, 1, 1)
    return out.to(beta.device) if torch.is_tensor(beta) else out


NOISE_SOURCES = ("torch", "torch-cpu", "philox")


def draw_noise(x, K: int, source="torch", generator=None):
    """The K per-step draws z of the reference's ``torch.randn_like(x)`` (common/utils_diff.py:65) as
    one [K, *x.shape] float32 tensor on x's device, in execution order; None for "philox" / None
    (the kernel's counter-based draws).  A tensor ``source`` is checked and returned."""
    if source is None or (isinstance(source, str) and source == "philox"):
        return None
    shape = (int(K),) + tuple(x.shape)
    if torch.is_tensor(source):
        if tuple(source.shape) != shape:
            raise ValueError(f"noise must have shape {shape}, got {tuple(source.shape)}")
        return source.to(device=x.device, dtype=torch.float32).contiguous()
    if source == "torch":
        if generator is not None:
            return torch.stack([torch.randn(x.shape, generator=generator, device=x.device) for _ in range(K)])
        return torch.stack([torch.randn_like(x, dtype=torch.float32) for _ in range(K)])
    if source == "torch-cpu":
        draws = [torch.randn(tuple(x.shape), generator=generator) if generator is not None
                 else torch.randn(tuple(x.shape)) for _ in range(K)]
        return torch.stack(draws).to(x.device)
    raise ValueError(f"noise must be one of {NOISE_SOURCES}, None or a tensor, got {source!r}")


def generalized_steps(x, src_mask, seq, model, b, **kwargs):
    eta = float(kwargs.get("eta", 0))
    seed = int(kwargs.get("seed", 0))
    seq = [int(s) for s in seq]
    with torch.no_grad():
        noise = draw_noise(x, len(seq), kwargs.get("noise", "torch" if eta != 0 else None), kwargs.get("generator"))
        if isinstance(model, HipGCNdiff):
            xs_t, x0s_t = model.sample(x, seq, b, eta=eta, mask=src_mask, seed=seed, trajectory=True, noise=noise)
            return [x] + [xs_t[k] for k in range(1, xs_t.shape[0])], [x0s_t[k] for k in range(x0s_t.shape[0])]
        # generic callable: host loop, HIP DDIM update
        upd = kwargs.get("updater")
        if upd is None:
            upd = schedule_handle(x.device)
        upd.set_schedule(seq, b, eta)
        n = x.size(0)
        xs, x0s = [x], []
        for step, (i, _j) in enumerate(step_pairs(seq)):
            t = torch.full((n,), float(i), device=x.device)
            et = model(xs[-1], src_mask, t, 0)
            xn, x0 = upd.ddim_update(xs[-1], et, step, seed=seed, noise=None if noise is None else noise[step])
            x0s.append(x0)
            xs.append(xn)
        return xs, x0s


# One schedule-only DDIM handle per (device, thread), reused by every generic-callable call: the
# reference's sampler allocates nothing persistent (common/utils_diff.py:46-68), so neither should
# a call here (a handle costs dpk_create, device buffers and a schedule upload).  A handle serves one
# thread (include/diffpose_kernels.h), so the cache is thread-local: a thread's handles are destroyed
# with its thread-local storage when it exits (HipGCNdiff.__del__), and clear_schedule_handles() closes
# the calling thread's handles at once (a thread pool no longer keeps one handle per thread it
# ever ran until the process ends).
_SCHED_TLS = threading.local()


def _sched_cache() -> dict:
    c = getattr(_SCHED_TLS, "handles", None)
    if c is None:
        c = _SCHED_TLS.handles = {}
    return c


def schedule_handle(device) -> HipGCNdiff:
    """The cached schedule-only handle of ``device`` for the calling thread (created on first use)."""
    dev = torch.device(device)
    key = (dev.type, dev.index or 0)
    cache = _sched_cache()
    upd = cache.get(key)
    if upd is None:
        upd = HipGCNdiff.__new__(HipGCNdiff)
        _init_schedule_only(upd, dev)
        cache[key] = upd
    return upd


def clear_schedule_handles() -> int:
    """Close the calling thread's cached schedule-only handles; returns how many were closed."""
    cache = _sched_cache()
    n = len(cache)
    for upd in cache.values():
        upd.close()
    cache.clear()
    return n


def _init_schedule_only(obj: HipGCNdiff, device) -> None:
    """A handle used only for its schedule table and the DDIM update kernel."""
    import ctypes

    from . import _lib
    from .weights import COORDS, HID, N_HEAD, N_LAYERS, N_PTS

    obj.device = torch.device(device)
    L = _lib.lib()
    cfg = _lib.DpkConfig(HID, N_LAYERS, N_HEAD, N_PTS, COORDS[0], COORDS[1], obj.device.index or 0)
    h = ctypes.c_void_p()
    _lib.check(None, "dpk_create", L.dpk_create(ctypes.byref(cfg), ctypes.byref(h)))
    obj._h = h
    obj.n_pts = N_PTS
    obj._mask_key = None
    obj._mask_ref = None
    obj._sched_key = None
    obj.training = False
