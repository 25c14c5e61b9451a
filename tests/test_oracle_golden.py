"""The CPU oracle against the reference's own outputs (golden fixtures made by
tests/golden/make_golden.py from /root/reference).  Bit-exact."""
import numpy as np
import pytest
import torch

from conftest import fixture_params, load_fixture
from oracle import dreamer_oracle as O

CASES = [("small", "small_epoch"), ("full", "full_epoch")]


def _t(a):
    return torch.from_numpy(np.asarray(a).copy())


@pytest.fixture(scope="module", params=CASES, ids=[c[0] for c in CASES])
def case(request):
    which, name = request.param
    fx = load_fixture(name)
    return which, fx, fixture_params(which, fx)


def test_replay_starts(case):
    _, fx, _ = case
    np.random.seed(int(fx["np_seed"]))
    st = O.replay_starts(int(fx["buf_size"]), int(fx["buf_capacity"]), int(fx["buf_next_idx"]),
                         int(fx["cfg_S"]), int(fx["cfg_B"]))
    assert np.array_equal(st, fx["starts"])


def _gather(fx):
    S, cap = int(fx["cfg_S"]), int(fx["buf_capacity"])
    idx = (fx["starts"][:, None] + np.arange(S)[None, :]) % cap
    obs = torch.tensor(fx["buf_frames"][idx], dtype=torch.float32)
    act = torch.tensor(fx["buf_actions"][idx], dtype=torch.float32)
    return obs, act


def test_warm_start_and_dream(case):
    _, fx, P = case
    R, C, S, H = (int(fx[k]) for k in ("cfg_rows", "cfg_cols", "cfg_S", "cfg_H"))
    obs, act = _gather(fx)
    z0, h0 = O.warm_start(obs, act, S, P, _t(fx["q_warm"]), R, C)
    assert torch.equal(z0, _t(fx["z0"])) and torch.equal(h0, _t(fx["h0"]))
    out = O.dream(z0, h0, P, _t(fx["eps"]), _t(fx["q"]), H, R, C)
    for got, key in zip(out, ["latents", "hiddens", "actions", "rewards", "continues", "mus", "sigmas"]):
        assert torch.equal(got, _t(fx[key])), key


def test_train_step_and_optimiser(case):
    _, fx, P = case
    R, C, H = (int(fx[k]) for k in ("cfg_rows", "cfg_cols", "cfg_H"))
    ap = [P["agent." + k].clone().requires_grad_(True) for k in O.ACTOR_KEYS]
    cp = [P["agent." + k].clone().requires_grad_(True) for k in O.CRITIC_KEYS]
    P2 = dict(P)
    P2.update({"agent." + k: t for k, t in zip(O.ACTOR_KEYS, ap)})
    P2.update({"agent." + k: t for k, t in zip(O.CRITIC_KEYS, cp)})
    z, h, a, r, c, mu, sg = O.dream(_t(fx["z0"]), _t(fx["h0"]), P2, _t(fx["eps"]), _t(fx["q"]), H, R, C)
    ts = O.train_step(z, h, r, c, a, mu, sg, P2, 1.0, ap, cp)
    assert torch.equal(ts["loss_actor"], _t(fx["loss_actor"]))
    assert torch.equal(ts["loss_critic"], _t(fx["loss_critic"]))
    assert torch.equal(ts["R"], _t(fx["R"]))
    assert float(ts["S"]) == float(fx["S_after"])
    for k, g in zip(O.ACTOR_KEYS + O.CRITIC_KEYS, ts["grad_actor_clipped"] + ts["grad_critic_clipped"]):
        assert torch.equal(g, _t(fx["gradc_agent." + k])), k
    # one AdamW step (Agent.py:63-76) + target EMA (Agent.py:90-94)
    for keys, grads, lr in ((O.ACTOR_KEYS, ts["grad_actor_clipped"], 8e-5),
                            (O.CRITIC_KEYS, ts["grad_critic_clipped"], 1e-4)):
        for k, g in zip(keys, grads):
            p = P["agent." + k]
            pn, _, _ = O.adamw_step(p, g, torch.zeros_like(p), torch.zeros_like(p), 1, lr)
            ref = _t(fx["post_agent." + k])
            assert torch.allclose(pn, ref, rtol=0, atol=1e-9), k
            if k.startswith("critic"):
                tk = "agent.target_" + k
                tn = P[tk] * (1.0 - 0.02) + 0.02 * ref
                assert torch.allclose(tn, _t(fx["post_" + tk]), rtol=0, atol=1e-9), tk


@pytest.mark.parametrize("which", ["small", "full"])
def test_blocks(which):
    fx = load_fixture(which + "_blocks")
    P = fixture_params(which, load_fixture(which + "_epoch") if which == "small" else None)
    h, z, a, obs = (_t(fx[k]) for k in ("h", "z", "a", "obs"))
    R, C = z.shape[-2:]
    assert torch.equal(O.gru(z, h, a, P), _t(fx["gru"]))
    x = torch.cat((z.flatten(2), a), -1).squeeze(1)
    man = O.gru_manual(x, h.squeeze(1), *(P["world_model.sequence_model.GRU." + k]
                                         for k in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")))
    assert torch.allclose(man.unsqueeze(1), _t(fx["gru"]), atol=2e-6)
    assert torch.equal(O.encoder_logits(h, obs, P), _t(fx["enc_logits"]))
    assert torch.equal(O.prior_logits(h, P, R, C), _t(fx["prior_logits"]))
    assert torch.equal(O.reward_predict(h, z, P), _t(fx["reward"]))
    p, lg = O.continue_forward(h, z, P)
    assert torch.equal(p, _t(fx["cont_prob"])) and torch.equal(lg, _t(fx["cont_logit"]))
    mu, sg = O.actor_forward(h, z, P)
    assert torch.equal(mu, _t(fx["actor_mu"])) and torch.equal(sg, _t(fx["actor_sigma"]))
    assert torch.equal(O.critic_value(h, z, P), _t(fx["critic_value"]))
    assert torch.equal(O.critic_logits(h, z, P), _t(fx["critic_logits"]))
    ze, _ = O.encode(h, obs, P, _t(fx["q_enc"]), R, C)
    assert torch.equal(ze, _t(fx["enc_z"]))
    zp, _ = O.prior_predict(h, P, _t(fx["q_prior"]), R, C)
    assert torch.equal(zp, _t(fx["prior_z"]))
    v = _t(fx["u_v"])
    assert torch.equal(O.symlog(v), _t(fx["u_symlog"]))
    assert torch.equal(O.symexp(v), _t(fx["u_symexp"]))
    assert torch.equal(O.twohot(O.symlog(v), torch.linspace(-20, 20, 255)), _t(fx["u_twohot"]))


def test_unimix_scalar_semantics():
    """0.99*p + 0.01/C on a float32 tensor == float32 fma-free arithmetic with
    the constants rounded to float32 (what the HIP sampler does)."""
    p = torch.rand(1000)
    ref = 0.99 * p + 0.01 * (1.0 / 32)
    f32 = (p.numpy() * np.float32(0.99)) + np.float32(0.01 * (1.0 / 32))
    assert np.array_equal(ref.numpy(), f32)


# ---------------------------------------------------------------------------
# BASELINE configs[0] shape (CarRacing widths, B=16 S=50 H=15, S0 = 5):
# tests/golden/baseline_b16.npz, inputs regenerated (tests/baseline_case.py)
# ---------------------------------------------------------------------------
def test_baseline_b16_oracle_matches_reference():
    from baseline_case import regen_fixture
    from conftest import state_layout
    fx = load_fixture("baseline_b16")
    B, S, H, R, C = (int(fx[k]) for k in ("cfg_B", "cfg_S", "cfg_H", "cfg_rows", "cfg_cols"))
    P, frames, q_warm, eps, q = regen_fixture(fx, dict(state_layout("full")))
    np.random.seed(int(fx["np_seed"]))
    st = O.replay_starts(int(fx["buf_size"]), int(fx["buf_capacity"]), int(fx["buf_next_idx"]), S, B)
    assert np.array_equal(st, fx["starts"])
    idx = (st[:, None] + np.arange(S)[None, :]) % int(fx["buf_capacity"])
    obs = torch.tensor(frames[idx], dtype=torch.float32)
    act = torch.tensor(fx["buf_actions"][idx])
    z0, h0 = O.warm_start(obs, act, S, P, q_warm, R, C)
    assert np.array_equal(z0.reshape(-1, C).argmax(-1).numpy(), fx["z0_idx"])
    assert torch.equal(h0, _t(fx["h0"]))
    ap = [P["agent." + k].clone().requires_grad_(True) for k in O.ACTOR_KEYS]
    cp = [P["agent." + k].clone().requires_grad_(True) for k in O.CRITIC_KEYS]
    P2 = dict(P)
    P2.update({"agent." + k: t for k, t in zip(O.ACTOR_KEYS, ap)})
    P2.update({"agent." + k: t for k, t in zip(O.CRITIC_KEYS, cp)})
    z, h, a, r, c, mu, sg = O.dream(z0, h0, P2, eps, q, H, R, C)
    assert np.array_equal(z.reshape(-1, C).argmax(-1).numpy(), fx["latents_idx"])
    for got, key in ((h, "hiddens"), (a, "actions"), (r, "rewards"), (c, "continues"), (mu, "mus"), (sg, "sigmas")):
        assert torch.equal(got.detach(), _t(fx[key])), key
    ts = O.train_step(z, h, r, c, a, mu, sg, P2, float(fx["S0"]), ap, cp)
    assert torch.equal(ts["loss_actor"], _t(fx["loss_actor"])) and torch.equal(ts["loss_critic"], _t(fx["loss_critic"]))
    assert torch.equal(ts["R"], _t(fx["R"]))
    assert float(ts["S"]) == float(fx["S_after"]) and float(fx["S_after"]) > 1.0  # normaliser max(S, 1) > 1
    st_ = int(fx["sample_stride"])
    for keys, grads in ((O.ACTOR_KEYS, ts["grad_actor_clipped"]), (O.CRITIC_KEYS, ts["grad_critic_clipped"])):
        for k, g in zip(keys, grads):
            flat = g.reshape(-1)
            ref = _t(fx["gradc_agent." + k])
            got = flat if flat.numel() < int(fx["small_tensor"]) else flat[::st_]
            assert torch.equal(got, ref), k
