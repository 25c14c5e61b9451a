"""Shared helpers for the GPU parity tests (HIP path vs the CPU oracle)."""
import numpy as np
import torch

from conftest import fixture_params, load_fixture
from formula import FULL, SMALL
from oracle import dreamer_oracle as O

CFG = {"small": SMALL, "full": FULL}


def build(which, dev, fx=None, B=None, H=None, S=None):
    """A dreamer_amd.Dreamer on `dev` holding the fixture's parameters."""
    from dreamer_amd import Dreamer
    cfg = dict(CFG[which])
    if fx is not None:
        cfg.update(batch_size=int(fx["cfg_B"]), horizon=int(fx["cfg_H"]), sequence_length=int(fx["cfg_S"]),
                   buffer_size=int(fx["buf_capacity"]))
    if B is not None:
        cfg["batch_size"] = B
    if H is not None:
        cfg["horizon"] = H
    if S is not None:
        cfg["sequence_length"] = S
    torch.manual_seed(0)
    d = Dreamer(cfg, dev)
    P = fixture_params(which, fx if fx is not None else load_fixture("small_epoch"))
    d.load_state_dict({k: v.to(dev) for k, v in P.items()})
    return d, P


def cpu(t):
    return t.detach().float().cpu()


def close(a, b, rtol, atol, what):
    a, b = cpu(a), cpu(b)
    assert a.shape == b.shape, f"{what}: shape {tuple(a.shape)} vs {tuple(b.shape)}"
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = err > tol
    assert not bool(bad.any()), (f"{what}: {int(bad.sum())}/{bad.numel()} out of tol, max|d|={float(err.max()):.3g}, "
                                 f"max rel={float((err / (b.abs() + 1e-12)).max()):.3g}")


def flip_report(z_gpu, z_ref, logits_ref, q, cols):
    """Compare one-hot latents; return (n_flips, worst relative margin of the
    oracle's top-2 p_hat/q scores at the flipped groups)."""
    a = cpu(z_gpu).reshape(-1, cols).argmax(-1)
    b = cpu(z_ref).reshape(-1, cols).argmax(-1)
    flips = (a != b).nonzero().flatten()
    if len(flips) == 0:
        return 0, 0.0
    p = torch.softmax(cpu(logits_ref).reshape(-1, cols), -1)
    p = 0.99 * p + 0.01 / cols
    score = (p / p.sum(-1, keepdim=True)) / cpu(q).reshape(-1, cols)
    top = score[flips].topk(2, dim=-1).values
    margin = float(((top[:, 0] - top[:, 1]) / top[:, 0]).max())
    return len(flips), margin
