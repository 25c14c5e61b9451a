"""World-model training step on the HIP path (dr_wm_train_grads via
WorldModel.training_step) vs the reference's own outputs (tests/golden/*_wm.npz,
made by make_golden_wm.py from WorldModel.training_step with autocast off).
Run on the MI355X box: pytest -m gpu.

Tolerances (fp32): the posterior scan's hiddens / logits at rtol 2e-4 /
atol 2e-5 (15-step recurrence, reordered f32 sums); one-hot indices exact;
losses rtol 1e-4; gradients (after clip_grad_norm_) per tensor within
2e-3 relative + 2e-4 x max|ref| (the decoder / encoder weight gradients sum
~10^5-10^6 products in a different order than MKL/oneDNN); parameters after
the AdamW step within 2.1 x lr (Adam's first step moves each weight by about
lr * sign(g), so only a sign flip of a near-zero gradient can differ)."""
import numpy as np
import pytest
import torch

from conftest import load_fixture
from gpu_helpers import build, close, cpu, flip_report
from test_oracle_wm import window

pytestmark = pytest.mark.gpu
SAMPLE = 997


def _t(a, dev=None):
    t = torch.from_numpy(np.asarray(a).copy())
    return t if dev is None else t.to(dev)


def _sampled(t):
    f = t.reshape(-1)
    return f[::SAMPLE] if f.numel() > 4 * SAMPLE else f


def _run(which, gpu, step=True):
    fx = load_fixture(which + "_wm")
    d, _ = build(which, gpu, fx)
    wm = d.world_model
    obs, act, rew, cont, T = window(fx)
    out = {}
    loss = wm.train_step_hip(obs.to(gpu), act.to(gpu), rew.to(gpu), cont.to(gpu), noise_q=_t(fx["q"], gpu),
                             outputs=out, step=step)
    torch.cuda.synchronize()
    return fx, d, wm, out, loss


@pytest.mark.parametrize("which", ["small", "full"])
def test_wm_step_matches_reference(which, gpu):
    fx, d, wm, out, loss = _run(which, gpu)
    B, T = int(fx["cfg_B"]), int(fx["cfg_H"])
    C = int(fx["cfg_cols"])
    # posterior scan (time-major on the GPU, batch-first in the fixture)
    close(out["hiddens"], _t(fx["hiddens"]).transpose(0, 1), 2e-4, 2e-5, "posterior hiddens")
    close(out["post_logits"], _t(fx["post_logits"]).transpose(0, 1), 2e-4, 2e-5, "posterior logits")
    lat_ref = _t(fx["latents"]).transpose(0, 1)
    q = _t(fx["q"]).reshape(T, B, -1)
    n_flip, _ = flip_report(out["latents"], lat_ref, _t(fx["post_logits"]).transpose(0, 1), q, C)
    assert n_flip == 0, f"{n_flip} posterior one-hot flips"
    # losses
    ls = cpu(wm.last_losses)
    for i, k in ((0, "total"), (1, "loss_pred"), (2, "kl_dyn"), (3, "kl_rep")):
        ref = float(fx[k])
        assert abs(float(ls[i]) - ref) <= 1e-4 * max(1.0, abs(ref)), (k, float(ls[i]), ref)
    assert int(wm.last_skip.item()) == 0
    assert abs(float(wm.last_sqnorm.sqrt()) - float(fx["norm"])) <= 2e-4 * float(fx["norm"])
    # clipped gradients (left in the flat buffer by the fused AdamW) and updated parameters
    named = dict(d.named_parameters())
    keys = [str(k) for k in fx["wm_keys"]]
    for k in keys:
        p = named[k]
        g = p.grad if which == "small" else _sampled(p.grad)
        ref = _t(fx["grad_" + k])
        g = g.reshape(ref.shape)
        close(g, ref, 2e-3, 2e-4 * max(float(ref.abs().max()), 1e-6), "grad " + k)
        pv = p.detach() if which == "small" else _sampled(p.detach())
        close(pv.reshape(ref.shape), _t(fx["post_" + k]).reshape(ref.shape), 1e-6, 2.1e-4, "param " + k)


def test_wm_step_deterministic(gpu):
    """two runs from the same weights and noise give bit-identical gradients"""
    _, d1, _, _, _ = _run("small", gpu, step=False)
    _, d2, _, _, _ = _run("small", gpu, step=False)
    for (n, p1), (_, p2) in zip(d1.world_model.named_parameters(), d2.world_model.named_parameters()):
        assert torch.equal(p1.grad, p2.grad), n


def test_wm_step_skips_nonfinite(gpu):
    """a non-finite loss leaves the parameters untouched (WorldModel.py:191-193)"""
    fx = load_fixture("small_wm")
    d, _ = build("small", gpu, fx)
    wm = d.world_model
    obs, act, rew, cont, T = window(fx)
    rew = rew.clone()
    rew[0, 0] = float("nan")
    before = [p.detach().clone() for p in wm.parameters()]
    wm.train_step_hip(obs.to(gpu), act.to(gpu), rew.to(gpu), cont.to(gpu), noise_q=_t(fx["q"], gpu))
    torch.cuda.synchronize()
    assert int(wm.last_skip.item()) == 1
    for b, p in zip(before, wm.parameters()):
        assert torch.equal(b, p.detach())


@pytest.mark.parametrize("which", ["small", "full"])
def test_decoder_forward(which, gpu):
    """Decoder.forward on HIP (dr_decoder_fwd) vs the oracle's restatement
    (pinned by the WM fixtures' losses) on random states; rtol 1e-4 / atol 1e-5."""
    from oracle import dreamer_oracle as O
    fx = load_fixture(which + "_wm")
    d, P = build(which, gpu, fx)
    R, C = int(fx["cfg_rows"]), int(fx["cfg_cols"])
    Hd = d.world_model.hidden_dims
    g = torch.Generator().manual_seed(3)
    h = torch.randn(3, 2, Hd, generator=g)
    lg = torch.randn(3, 2, R, C, generator=g)
    z = torch.nn.functional.one_hot(lg.argmax(-1), C).float()
    with torch.no_grad():
        mu = d.world_model.decoder(h.to(gpu), z.to(gpu))
    ref = O.decoder_forward(h, z, P, (d.world_model.observation_dim_x, d.world_model.observation_dim_y))
    close(mu, ref, 1e-4, 1e-5, "decoder mu")
