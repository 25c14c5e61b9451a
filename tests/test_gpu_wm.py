"""World-model training step on the HIP path (dr_wm_train_grads via
WorldModel.training_step) vs the reference's own outputs (tests/golden/*_wm.npz,
made by make_golden_wm.py from WorldModel.training_step with autocast off), and
at BASELINE shapes (B = 64 and the bench's B = 256, T = 15, CarRacing widths,
64 x 64 frames) vs the CPU oracle's restatement of the same step on the same
replay windows and tie-guarded noise.  Run on the MI355X box: pytest -m gpu.

Tolerances (fp32): the posterior scan's hiddens / logits at rtol 2e-4 /
atol 2e-5 (15-step recurrence, reordered f32 sums); one-hot indices exact;
losses rtol 1e-4; gradients (after clip_grad_norm_) per tensor within
2e-3 relative + 2e-4 x max|ref| (the decoder / encoder weight gradients sum
~10^5-10^6 products in a different order than MKL/oneDNN).  Parameters after
the AdamW step: against AdamW (the oracle's torch-order restatement) applied to
the GPU's OWN clipped gradients at |d| <= 1e-7 + 1e-6 |p| (pins the fused
optimiser), and against the reference's / oracle's post-step parameters at
|d| <= 1e-6 + 1e-6 |p| on every element whose gradient is determined to
to 1 % by the two sides (|g_ref| > 100 |g_gpu - g_ref|): there Adam's first
step, lr g / (|g| + eps), differs by at most lr / 400.  The rest are Adam's
sign(g) * lr ambiguity (a gradient whose summation-order error rivals its size
moves the weight by ~lr either way); they are counted and reported, not
banded -- the AdamW-on-own-gradients check above covers every element."""
import numpy as np
import pytest
import torch

from conftest import fixture_params, load_fixture
from gpu_helpers import build, close, cpu, flip_report
from oracle import dreamer_oracle as O
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
    P0 = fixture_params(which, fx)
    sub = (lambda t: t.reshape(-1)) if which == "small" else _sampled
    n_amb = check_grads_and_params(named, keys, P0, lambda k: _t(fx["grad_" + k]),
                                   lambda k: _t(fx["post_" + k]), sub, which)
    print(f"{which}: {n_amb} parameters at Adam's sign ambiguity (|g| below the gradient tolerance)")


def check_grads_and_params(named, keys, P0, g_ref_of, post_ref_of, sub, label, lr=1e-4):
    """Clipped gradients and post-AdamW parameters (module doc).  named: the
    GPU model's parameters after the step (p.grad = the clipped gradient the
    fused AdamW used); P0: the parameters before it; g_ref_of / post_ref_of:
    the reference's clipped gradient / post-step parameter of a key, possibly
    subsampled by `sub`.  Returns the number of sign-ambiguous elements."""
    n_amb = 0
    for k in keys:
        p = named[k]
        g_ref = g_ref_of(k)
        g_gpu = cpu(p.grad)
        atol = 2e-4 * max(float(g_ref.abs().max()), 1e-6)
        close(sub(g_gpu).reshape(g_ref.shape), g_ref, 2e-3, atol, f"{label} grad {k}")
        # the fused AdamW (step 1) on the GPU's own clipped gradients
        p0 = P0[k].detach().float().reshape(g_gpu.shape)
        pn, _, _ = O.adamw_step(p0, g_gpu, torch.zeros_like(p0), torch.zeros_like(p0), 1, lr)
        got = cpu(p)
        close(got, pn, 1e-6, 1e-7, f"{label} AdamW(step 1) on the GPU's grads {k}")
        # the reference's post-step parameters, away from Adam's sign ambiguity: where the two
        # gradients agree to 1 % the first Adam step, lr g / (|g| + eps), differs by <= lr / 400
        want = post_ref_of(k).reshape(-1)
        gs = g_ref.reshape(-1)
        live = gs.abs() > 100 * (sub(g_gpu).reshape(-1) - gs).abs()
        n_amb += int((~live).sum())
        err = (sub(got).reshape(-1) - want).abs()
        bad = live & (err > 1e-6 + 1e-6 * want.abs())
        assert not bool(bad.any()), (label, k, int(bad.sum()), float(err[live].max()))
    return n_amb


def _baseline_wm_case(gpu, B, T=15, seed=0, precision="fp32"):
    """CarRacing widths at 64 x 64, reference default init under
    torch.manual_seed(0), SURVEY 8d synthetic replay (bench.synthetic_replay),
    B windows of T = horizon steps; the oracle's step on the CPU with a
    tie-guarded posterior noise draw."""
    import bench
    from baseline_case import TieGuard
    from dreamer_amd import Dreamer
    from test_gpu_baseline import CAR
    cfg = dict(CAR)
    cfg.update(batch_size=B, sequence_length=64, horizon=T, precision=precision)
    torch.manual_seed(0)
    d = Dreamer(cfg, gpu)
    wm = d.world_model
    R, C = wm.latent_num_rows, wm.latent_num_columns
    n = 4096
    frames, acts, rews, conts = bench.synthetic_replay(n, (64, 64), 3, seed=seed)
    starts = np.random.RandomState(300 + B).randint(0, n - T + 1, size=B)
    idx = starts[:, None] + np.arange(T)[None, :]
    obs = torch.tensor(frames[idx], dtype=torch.float32)
    act = torch.tensor(acts[idx])
    rew = torch.tensor(rews[idx]).unsqueeze(-1)
    cont = torch.tensor(conts[idx]).unsqueeze(-1)
    q = torch.empty(T, B * R, C).exponential_(generator=torch.Generator().manual_seed(400 + B))
    names = [nm for nm, _ in wm.named_parameters()]
    P0 = {("world_model." + k): v.detach().cpu().clone() for k, v in wm.state_dict().items()}
    P = {k: v.clone().requires_grad_(True) for k, v in P0.items()}
    torch.set_num_threads(16)
    with TieGuard() as tg:  # widens near-tie margins of q in place, the oracle's draws unchanged
        ref = O.wm_train_step(obs, act, rew, cont, P, q, R, C, T, ["world_model." + nm for nm in names],
                              betas=(wm.beta_pred, wm.beta_dyn, wm.beta_rep))
    out = {}
    wm.train_step_hip(obs.to(gpu), act.to(gpu), rew.to(gpu), cont.to(gpu), noise_q=q.to(gpu), outputs=out,
                      step=True)
    torch.cuda.synchronize()
    return d, wm, out, ref, q, names, P0, tg


@pytest.mark.parametrize("B", [64, 256])
def test_wm_step_matches_oracle_at_baseline_shape(B, gpu):
    """WorldModel.training_step (WorldModel.py:148-202) at B = 64 (configs[1])
    and the bench's B = 256, T = 15, full widths: the shapes whose split-K and
    tile routing the small fixtures do not reach.  Posterior states, indices,
    losses, the gradient norm, every clipped gradient and every post-AdamW
    parameter against the oracle (module doc for the tolerances)."""
    d, wm, out, ref, q, names, P0, tg = _baseline_wm_case(gpu, B)
    T = wm.horizon
    C = wm.latent_num_columns
    close(out["hiddens"], ref["hiddens"].transpose(0, 1), 2e-4, 2e-5, "posterior hiddens")
    close(out["post_logits"], ref["post_logits"].transpose(0, 1), 2e-4, 2e-5, "posterior logits")
    n_flip, _ = flip_report(out["latents"], ref["latents"].transpose(0, 1), ref["post_logits"].transpose(0, 1),
                            q.reshape(T, B, -1), C)
    assert n_flip == 0, f"{n_flip} posterior one-hot flips"
    ls = cpu(wm.last_losses)
    for i, k in ((0, "total"), (1, "loss_pred"), (2, "kl_dyn"), (3, "kl_rep")):
        r = float(ref[k])
        assert abs(float(ls[i]) - r) <= 1e-4 * max(1.0, abs(r)), (k, float(ls[i]), r)
    assert int(wm.last_skip.item()) == 0
    assert abs(float(wm.last_sqnorm.sqrt()) - float(ref["norm"])) <= 2e-4 * float(ref["norm"])
    named = {"world_model." + n: p for n, p in wm.named_parameters()}
    keys = ["world_model." + n for n in names]
    gref = dict(zip(keys, ref["grads_clipped"]))
    post = {}
    for k in keys:  # the oracle's own AdamW step (lr 1e-4, WorldModel.py:63-69) on its clipped gradients
        p0 = P0[k]
        post[k], _, _ = O.adamw_step(p0, gref[k], torch.zeros_like(p0), torch.zeros_like(p0), 1, 1e-4)
    n_amb = check_grads_and_params(named, keys, P0, lambda k: gref[k], lambda k: post[k],
                                   lambda t: t.reshape(-1), f"B{B}")
    print(f"WM step B={B} T={T}: loss {float(ls[0]):.6f} (oracle {float(ref['total']):.6f}), "
          f"guarded {tg.guarded}/{tg.draws} draws, {n_amb} sign-ambiguous parameters")


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


def _nw(a, b):
    a, b = a.detach().float().cpu().reshape(-1), b.detach().float().cpu().reshape(-1)
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def test_wm_step_bf16_vs_fp32_oracle(gpu):
    """bf16 perf mode's WorldModel.training_step (precision='bf16': every
    convolution of the encoder, decoder and their data / weight gradients as a
    one-term bf16 implicit GEMM with f32 accumulation) at the
    bench's B = 256, T = 15 against the fp32 oracle on the same windows and
    noise.  Statistical bounds, not parity: a bf16 rounding of the encoder
    features moves posterior logits by ~1e-3 relative, so a few near-tie draws
    take the other class and those rows' states then differ.  Reported: the
    posterior flip fraction, normwise errors of hiddens / logits, the losses,
    the gradient norm and the worst per-tensor normwise gradient error (the
    bounds and the first measured values are in the asserts' comments)."""
    d, wm, out, ref, q, names, P0, tg = _baseline_wm_case(gpu, 256, precision="bf16")
    T, C = wm.horizon, wm.latent_num_columns
    B = 256
    lat = out["latents"].detach().float().cpu().reshape(T, B, -1, C).argmax(-1)
    lat_ref = ref["latents"].transpose(0, 1).reshape(T, B, -1, C).argmax(-1)
    flip = float((lat != lat_ref).float().mean())
    m = {"flip_fraction": flip,
         "hiddens": _nw(out["hiddens"], ref["hiddens"].transpose(0, 1)),
         "post_logits": _nw(out["post_logits"], ref["post_logits"].transpose(0, 1))}
    ls = cpu(wm.last_losses)
    for i, k in ((0, "total"), (1, "loss_pred"), (2, "kl_dyn"), (3, "kl_rep")):
        m[k] = (float(ls[i]), float(ref[k]))
    m["norm"] = (float(wm.last_sqnorm.sqrt()), float(ref["norm"]))
    named = {"world_model." + n: p for n, p in wm.named_parameters()}
    keys = ["world_model." + n for n in names]
    gerr = {k: _nw(named[k].grad, g) for k, g in zip(keys, ref["grads_clipped"])}
    worst = sorted(gerr.items(), key=lambda kv: -kv[1])[:5]
    m["grad_worst5"] = worst
    gall = torch.cat([named[k].grad.detach().float().cpu().reshape(-1) for k in keys])
    rall = torch.cat([g.reshape(-1) for g in ref["grads_clipped"]])
    m["grad_all"] = _nw(gall, rall)
    print(f"bf16 WM step B=256 T={T} vs the fp32 oracle: {m}")
    # first run (round 4, MI355X): flips 1.7e-4 of the draws, hiddens 1.7e-2 / logits 1.4e-2 normwise (the
    # rows a flip sent elsewhere), total loss 6e-7 relative, gradient norm 7e-6, all gradients 5.9e-5
    # normwise, worst tensor 1.8e-2 (encoder conv1 weight)
    assert int(wm.last_skip.item()) == 0
    assert flip <= 2e-3, m
    assert m["hiddens"] <= 0.1 and m["post_logits"] <= 0.1, m
    assert abs(m["total"][0] - m["total"][1]) <= 1e-3 * abs(m["total"][1]), m
    for k in ("kl_dyn", "kl_rep"):
        assert abs(m[k][0] - m[k][1]) <= 5e-3 * max(1.0, abs(m[k][1])), m
    assert abs(m["norm"][0] - m["norm"][1]) <= 5e-3 * m["norm"][1], m
    assert m["grad_all"] <= 1e-3, m
    assert worst[0][1] <= 0.1, m
