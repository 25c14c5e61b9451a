"""The CPU oracle's world-model training step against the reference's own
outputs (tests/golden/make_golden_wm.py ran WorldModel.training_step from
/root/reference with autocast disabled).  Losses bit-exact; gradients exact
on the reduced config, within 1e-6 relative of the largest entry at full width
(autograd's reduction order differs from torch.distributions' KL graph)."""
import numpy as np
import pytest
import torch

from conftest import fixture_params, load_fixture
from oracle import dreamer_oracle as O

CASES = [("small", "small_wm"), ("full", "full_wm")]
SAMPLE = 997


def _t(a):
    return torch.from_numpy(np.asarray(a).copy())


def window(fx):
    S, cap, T = int(fx["cfg_S"]), int(fx["buf_capacity"]), int(fx["cfg_H"])
    idx = (fx["starts"][:, None] + np.arange(S)[None, :]) % cap
    obs = torch.tensor(fx["buf_frames"][idx], dtype=torch.float32)
    act = torch.tensor(fx["buf_actions"][idx])
    rew = torch.tensor(fx["buf_rewards"][idx])
    cont = torch.tensor(fx["buf_continues"][idx])
    return obs, act, rew, cont, T


@pytest.fixture(scope="module", params=CASES, ids=[c[0] for c in CASES])
def case(request):
    which, name = request.param
    fx = load_fixture(name)
    return which, fx, fixture_params(which, fx)


def _sampled(t):
    f = t.reshape(-1)
    return f[::SAMPLE] if f.numel() > 4 * SAMPLE else f


def test_wm_train_step(case):
    which, fx, P = case
    R, C = int(fx["cfg_rows"]), int(fx["cfg_cols"])
    obs, act, rew, cont, T = window(fx)
    keys = [str(k) for k in fx["wm_keys"]]
    for k in keys:
        P[k] = P[k].clone().requires_grad_(True)
    o = O.wm_train_step(obs, act, rew, cont, P, _t(fx["q"]), R, C, T, keys)
    assert torch.equal(o["total"].detach(), _t(fx["total"]))
    assert torch.equal(o["hiddens"].detach(), _t(fx["hiddens"]))
    assert torch.equal(o["latents"].detach(), _t(fx["latents"]))
    # the fp16-autocast reference run is a loose check of the same step
    assert abs(float(o["total"]) - float(fx["total_fp16"])) < 1e-4 * abs(float(fx["total"]))
    for k, g in zip(keys, o["grads_clipped"]):
        ref = _t(fx["grad_" + k])
        got = g if which == "small" else _sampled(g)
        tol = 0.0 if which == "small" else 1e-6 * max(1e-3, float(ref.abs().max()))
        assert float((got.reshape(ref.shape) - ref).abs().max()) <= tol, k


def test_wm_adamw(case):
    """one AdamW step (lr 1e-4, wd 1e-6, eps 1e-5) from the clipped grads
    reproduces the reference's post-step parameters."""
    which, fx, P = case
    keys = [str(k) for k in fx["wm_keys"]]
    for k in keys:
        g = _t(fx["grad_" + k])
        p = P[k].detach()
        if which != "small":
            p = _sampled(p)
        p2, _, _ = O.adamw_step(p.reshape(g.shape), g, torch.zeros_like(g), torch.zeros_like(g), 1, 1e-4)
        ref = _t(fx["post_" + k])
        assert float((p2 - ref.reshape(p2.shape)).abs().max()) <= 1e-7, k
