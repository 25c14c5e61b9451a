"""BASELINE configs[4]: proprioceptive vector observations (observation_dims =
[D]) with an MLP encoder / decoder in place of the conv stacks.

The reference has no such mode (its Encoder is always convolutional,
VariationalAutoEncoder.py:33-42), so this mode's parity is UNPINNED against
the reference: the HIP path is checked against the oracle's restatement of
the framework's own definition (oracle.encoder_logits / decoder_forward on
(B, S, D) observations; include/dreamer_hip.h dr_dims.obs_dim), with the
same tolerances as the image-mode tests.  Everything downstream of the
encoder (GRU, heads, imagination, actor-critic update) is the pinned image-
mode code."""
import numpy as np
import pytest
import torch

from formula import FULL
from gpu_helpers import close, cpu, flip_report

pytestmark = pytest.mark.gpu
D_OBS = 24


def _dreamer(gpu, **kw):
    from dreamer_amd import Dreamer
    cfg = dict(FULL)
    cfg.update(observation_dims=[D_OBS], **kw)
    torch.manual_seed(0)
    return Dreamer(cfg, gpu)


def _params(d):
    return {k: v.detach().cpu().clone() for k, v in d.state_dict().items()}


def test_vector_encoder_features_and_encode(gpu):
    """dr_encoder_features + dr_observe_scan (Encoder.encode) vs the oracle: logits
    rtol 2e-4 / atol 2e-5, sampled indices exact (flip report)."""
    from oracle import dreamer_oracle as O
    d = _dreamer(gpu)
    wm = d.world_model
    R, C = d.latent_state_dims
    g = torch.Generator().manual_seed(5)
    B, S = 6, 4
    obs = torch.randn(B, S, D_OBS, generator=g)
    h = torch.randn(B, S, d.hidden_state_dims, generator=g) * 0.5
    with torch.no_grad():
        z, logits = wm.encoder.encode(h.to(gpu), obs.to(gpu))
    P = _params(d)
    ref = O.encoder_logits(h, obs, P).view(B, S, R, C)
    close(logits, ref, 2e-4, 2e-5, "vector encoder logits")
    assert torch.allclose(cpu(z).sum(-1), torch.ones(B, S, R))


def test_vector_decoder_forward(gpu):
    from oracle import dreamer_oracle as O
    d = _dreamer(gpu)
    R, C = d.latent_state_dims
    g = torch.Generator().manual_seed(3)
    h = torch.randn(3, 2, d.hidden_state_dims, generator=g)
    z = torch.nn.functional.one_hot(torch.randn(3, 2, R, C, generator=g).argmax(-1), C).float()
    with torch.no_grad():
        mu = d.world_model.decoder(h.to(gpu), z.to(gpu))
    assert tuple(mu.shape) == (3, 2, D_OBS)
    close(mu, O.decoder_forward(h, z, _params(d), None), 1e-4, 1e-5, "vector decoder mu")


def test_vector_wm_step_matches_oracle(gpu):
    """dr_wm_train_phase in vector mode (MLP encoder / decoder forward and
    backward, MSE without Tanh) vs autograd through the oracle's loss: the
    posterior scan, losses and every raw world-model gradient."""
    from oracle import dreamer_oracle as O
    B, S, H = 4, 8, 6
    d = _dreamer(gpu, batch_size=B, sequence_length=S, horizon=H)
    wm = d.world_model
    R, C = d.latent_state_dims
    A = d.action_dims
    g = torch.Generator().manual_seed(21)
    obs = torch.randn(B, S, D_OBS, generator=g)
    act = torch.rand(B, S, A, generator=g) * 2 - 1
    rew = torch.randn(B, S, 1, generator=g)
    cont = (torch.rand(B, S, 1, generator=g) > 0.1).float()
    q = torch.empty(H, B * R, C).exponential_(generator=g)
    names = [n for n, _ in wm.named_parameters()]
    P = {("world_model." + k): v.detach().cpu().clone().requires_grad_(True) for k, v in wm.state_dict().items()}
    ref = O.wm_train_step(obs, act, rew, cont, P, q, R, C, H, ["world_model." + n for n in names],
                          betas=(wm.beta_pred, wm.beta_dyn, wm.beta_rep))
    out = {}
    wm.train_step_hip(obs.to(gpu), act.to(gpu), rew.to(gpu), cont.to(gpu), noise_q=q.to(gpu), outputs=out,
                      step=False)
    torch.cuda.synchronize()
    close(out["hiddens"], ref["hiddens"].transpose(0, 1), 2e-4, 2e-5, "posterior hiddens")
    close(out["post_logits"], ref["post_logits"].transpose(0, 1), 2e-4, 2e-5, "posterior logits")
    n_flip, _ = flip_report(out["latents"], ref["latents"].transpose(0, 1), ref["post_logits"].transpose(0, 1),
                            q.reshape(H, B, -1), C)
    assert n_flip == 0, f"{n_flip} posterior one-hot flips"
    ls = cpu(wm.last_losses)
    for i, k in ((0, "total"), (1, "loss_pred"), (2, "kl_dyn"), (3, "kl_rep")):
        r = float(ref[k])
        assert abs(float(ls[i]) - r) <= 1e-4 * max(1.0, abs(r)), (k, float(ls[i]), r)
    for n, p, gr in zip(names, wm.parameters(), ref["grads"]):
        close(p.grad.reshape(gr.shape), gr, 2e-3, 2e-4 * max(float(gr.abs().max()), 1e-6), "grad " + n)


def test_vector_epoch_vs_oracle_B4096(gpu):
    """BASELINE configs[4] at its batch: one train_Agent epoch (Dreamer.py:264-287)
    with vector observations at B = 4096, S = 64, H = 15 (M = 4096-row chain
    tiles, 61,440 returns through update_S's radix select) against the CPU
    oracle on the same replay windows and tie-guarded explicit noise, with
    test_gpu_baseline.compare's checks and tolerances: exact warm-start and
    imagined indices, h0 / hiddens / actions / heads / returns at 1e-4, losses
    1e-4, S 1e-6, clipped gradients, post-AdamW parameters.  Unpinned against
    the reference (it has no vector encoder); everything past the MLP encoder
    is the pinned image-mode code."""
    from baseline_case import oracle_epoch
    from test_gpu_baseline import compare, run_gpu_epoch
    B, S, H = 4096, 64, 15
    n = 8192
    d = _dreamer(gpu, batch_size=B, sequence_length=S, horizon=H, buffer_size=n)
    R, C = d.latent_state_dims
    A = d.action_dims
    P = _params(d)
    rng = np.random.default_rng(0)
    frames = rng.standard_normal((n, D_OBS)).astype(np.float32)
    acts = rng.uniform(-1, 1, (n, A)).astype(np.float32)
    r = rng.standard_normal(n).astype(np.float32)
    rews = (np.sign(r) * np.log1p(np.abs(r))).astype(np.float32)
    conts = np.ones(n, np.float32)
    conts[::1000] = 0.0
    starts = np.random.RandomState(4096).randint(0, n - S + 1, size=B)
    g = torch.Generator().manual_seed(4097)
    q_warm = torch.empty(S // 2, B * R, C).exponential_(generator=g)
    eps = torch.randn(H, B, 1, A, generator=g)
    q = torch.empty(H, B * R, C).exponential_(generator=g)
    idx = starts[:, None] + np.arange(S)[None, :]
    obs = torch.tensor(frames[idx])
    act = torch.tensor(acts[idx])
    S0 = 3.0
    torch.set_num_threads(16)
    ref = oracle_epoch(P, obs, act, S, H, R, C, q_warm, eps, q, S0)
    ref["P0"] = P
    eng, pre = run_gpu_epoch(d, frames, acts, rews, conts, n, 0, starts, q_warm, eps, q, S0)
    n_tiny = compare(d, eng, pre, ref, C, "vector B4096", S0)
    print(f"configs[4] B=4096 epoch: guarded {ref['guarded']}/{ref['draws']} draws, {n_tiny} near-zero-gradient "
          f"params, actor loss {pre['la']:.6g}, critic loss {pre['lc']:.6g}, S {pre['S']:.6g}")


def test_vector_train_agent_and_acting(gpu):
    """train_Agent from an f32 vector replay ring at B=256 (configs[4] widths,
    smaller batch): finite losses, one-hot warm-start latents; the unfused
    batch-1 act_step runs and returns actions in (-1, 1)."""
    d = _dreamer(gpu, batch_size=256, sequence_length=64, horizon=15, buffer_size=2048)
    rng = np.random.default_rng(0)
    n = 2048
    d.buffer.load_arrays(rng.standard_normal((n, D_OBS)).astype(np.float32),
                         rng.uniform(-1, 1, (n, d.action_dims)).astype(np.float32),
                         rng.standard_normal(n).astype(np.float32), np.ones(n, np.float32))
    np.random.seed(1)
    la, lc = d.train_Agent()
    torch.cuda.synchronize()
    assert np.isfinite(float(la)) and np.isfinite(float(lc))
    z0 = cpu(d.engine.latents[:, 0])
    assert torch.equal(z0.reshape(-1, d.latent_state_dims[1]).sum(-1) > 0.5,
                       torch.ones(z0.numel() // d.latent_state_dims[1], dtype=torch.bool))
    with torch.no_grad():
        a, mu, sg, z, h = d.act_step(rng.standard_normal(D_OBS).astype(np.float32))
        a2, _, _, _, _ = d.act_step(rng.standard_normal(D_OBS).astype(np.float32), z, h, a)
    torch.cuda.synchronize()
    assert tuple(a2.shape) == (1, 1, d.action_dims) and bool((cpu(a2).abs() < 1).all())
