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


def pscan_status(eng):
    """Status word of the persistent posterior scan (scan.hip counter block in
    the observe workspace's ring): 0 = every hand-off completed in time."""
    B = eng.B
    off = 4 * (2 * B * 600 + 2 * B * 200 + 4 * B * 32) + 48 * 128
    return int(eng.ws_obs.view(torch.uint8)[off:off + 4].view(torch.int32).item())


def pdream_status(eng):
    """Status word of the persistent imagination unroll (dream.hip: its
    counter block closes the imagination workspace): 0 = every hand-off
    completed in time."""
    from dreamer_amd import _lib as L
    B, H = eng.B, eng.H
    total = L.query("dr_imagine_workspace_bytes", eng.d, B, H)
    pd = 4 * H * B * 200 + 8 * (H + 1) * B * 32
    pb = (4 * B * H * (4 * 200 + 200 + 2 * 1800 + 600 + 1664 + 2 * 200 + 1024 + 600) + 8 * 8 * 32 * 4) if B <= 64 else 0
    cnt = (total - pb) - 7 * 16 * 32 * 4  # the unroll's block ends where the BPTT's starts (256-byte multiples)
    word = lambda o: int(eng.ws_im.view(torch.uint8)[o:o + 4].view(torch.int32).item())
    # (status, the GRU stage's counter of rows 0..15: 60 unit slices x H steps when it ran), and, at
    # B <= 64, the BPTT's (status, Q7's counter of rows 0..15: 51 column blocks x H steps)
    st = (word(cnt + 6 * 16 * 32 * 4), word(cnt + 2 * 16 * 32 * 4))
    if B <= 64:
        pcnt = total - 8 * 8 * 32 * 4
        st += (word(pcnt + 7 * 8 * 32 * 4), word(pcnt + 6 * 8 * 32 * 4))
    return st


def assert_persistent_ran(eng):
    """At B <= 128 the warm start and the unroll ran as the persistent kernels
    (scan.hip, dream.hip) and, at B <= 64, the BPTT (bptt.hip): status words 0,
    the unroll's GRU counter 60 H, the BPTT's Q7 counter 51 H, the fault slot 0."""
    B, H = eng.B, eng.H
    if B > 128:
        return
    assert pscan_status(eng) == 0
    st = pdream_status(eng)
    assert st[:2] == (0, 60 * H), st
    if B <= 64:
        assert st[2:] == (0, 51 * H), st
    assert float(eng.dr.agent.fault_slot()) == 0.0
