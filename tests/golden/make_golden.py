"""Generate golden fixtures by running the REFERENCE implementation.

Run in the survey/build container only (``/root/reference`` does not exist on
the GPU box):  ``python tests/golden/make_golden.py``.

For each configuration it builds the reference ``Dreamer``, fills its replay
``Buffer``, seeds numpy/torch, and steps through ``train_Agent``'s unit of work
(sample_sequences -> warm_start_generator -> dream_episodes -> train_step)
exactly as Dreamer.py:264-287 does.  The random draws the reference took from
torch's global generator are then replayed in the same order (``exponential_``
for each Categorical sample, ``normal_`` for each actor rsample) and stored as
explicit noise, together with the reference's inputs and outputs.  Finally it
checks the oracle (``oracle/dreamer_oracle.py``) reproduces every output from
that noise, so the committed fixtures pin the oracle.

Only data (inputs, noise, outputs, and for the reduced config its weights) is
written; no reference source is copied.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
sys.path.insert(0, "/root/reference")

from formula import FULL, SMALL, formula_state_dict, replay_data  # noqa: E402
from oracle import dreamer_oracle as O  # noqa: E402


def build_reference(cfg, weights):
    from Dreamer import Dreamer  # reference
    torch.manual_seed(0)
    d = Dreamer(dict(cfg), torch.device("cpu"))
    if weights == "formula":
        sd = formula_state_dict({k: tuple(v.shape) for k, v in d.state_dict().items()})
        d.load_state_dict(sd)
    return d


def run_case(cfg, weights, n_fill, np_seed, torch_seed, S0=1.0):
    d = build_reference(cfg, weights)
    sd0 = {k: v.detach().clone() for k, v in d.state_dict().items()}
    hw = tuple(cfg["observation_dims"])
    A = cfg["action_dims"]
    frames, acts, rews, conts = replay_data(n_fill, hw, A, seed=0)
    for i in range(n_fill):
        d.buffer.add_to_buffer(frames[i], acts[i], rews[i], conts[i])
    B, S, H = cfg["batch_size"], cfg["sequence_length"], cfg["horizon"]
    R_, C_ = cfg["latent_state_dims"]

    rec = {}
    ag = d.agent
    oa, oc = ag.actor_optimiser.step, ag.critic_optimiser.step

    def step_a(*a, **k):
        rec["ga"] = [p.grad.detach().clone() for p in ag.actor.parameters()]
        return oa(*a, **k)

    def step_c(*a, **k):
        rec["gc"] = [p.grad.detach().clone() for p in ag.critic.parameters()]
        return oc(*a, **k)

    ag.actor_optimiser.step = step_a
    ag.critic_optimiser.step = step_c

    np.random.seed(np_seed)
    torch.manual_seed(torch_seed)
    obs, act, rew, cont, seq = d.buffer.sample_sequences(batch_size=B)
    z0, h0 = d.warm_start_generator(obs, act, seq)
    outs = d.dream_episodes(z0, h0)
    lat, hid, acts_d, rews_d, conts_d, mus, sigs = outs
    with torch.no_grad():
        R = ag.compute_batched_R_lambda_returns(hid, lat, rews_d, conts_d, conts_d.shape[1])
    ag.S = S0  # return-range normaliser state before the update (Agent.py:60, 78-88)
    la, lc = ag.train_step(lat, hid, rews_d, conts_d, acts_d, mus, sigs)
    S_after = float(ag.S)
    sd1 = {k: v.detach().clone() for k, v in d.state_dict().items()}

    # replay the reference's draws in order
    torch.manual_seed(torch_seed)
    q_warm = torch.stack([torch.empty(B * R_, C_).exponential_() for _ in range(S // 2)])
    eps, q = [], []
    for _ in range(H):
        eps.append(torch.empty(B, 1, A).normal_())
        q.append(torch.empty(B * R_, C_).exponential_())
    eps, q = torch.stack(eps), torch.stack(q)
    np.random.seed(np_seed)
    starts = O.replay_starts(d.buffer.size, d.buffer.capacity, d.buffer.next_idx, S, B)

    # ---- check the oracle against the reference on the replayed noise ----
    P = {k: v.clone() for k, v in sd0.items()}
    idx = (starts[:, None] + np.arange(S)[None, :]) % d.buffer.capacity
    obs_o = torch.tensor(d.buffer.observation_buffer[idx], dtype=torch.float32)
    assert torch.equal(obs_o, obs), "replay gather mismatch"
    zo, ho = O.warm_start(obs_o, act, S, P, q_warm, R_, C_)
    assert torch.equal(zo, z0) and torch.equal(ho, h0), "warm start mismatch"
    ao = [p.detach().clone().requires_grad_(True) for p in (P["agent." + k] for k in O.ACTOR_KEYS)]
    co = [p.detach().clone().requires_grad_(True) for p in (P["agent." + k] for k in O.CRITIC_KEYS)]
    P2 = dict(P)
    for k, t in zip(O.ACTOR_KEYS, ao):
        P2["agent." + k] = t
    for k, t in zip(O.CRITIC_KEYS, co):
        P2["agent." + k] = t
    d_o = O.dream(z0.detach(), h0.detach(), P2, eps, q, H, R_, C_)
    for a_, b_ in zip(d_o, outs):
        assert torch.equal(a_, b_), "dream mismatch"
    zz, hh, aa, rr, cc, mm, ss = d_o
    ts = O.train_step(zz, hh, rr, cc, aa, mm, ss, P2, S0, ao, co)
    assert torch.equal(ts["loss_actor"], la.detach()) and torch.equal(ts["loss_critic"], lc.detach())
    assert torch.equal(ts["R"], R)
    maxd = max(float((g1 - g2).abs().max()) for g1, g2 in zip(ts["grad_actor_clipped"], rec["ga"]))
    maxc = max(float((g1 - g2).abs().max()) for g1, g2 in zip(ts["grad_critic_clipped"], rec["gc"]))
    print(f"  oracle vs reference: grads actor max|d|={maxd:.3g} critic max|d|={maxc:.3g}; S={S_after}")

    out = {
        "cfg_B": B, "cfg_S": S, "cfg_H": H, "cfg_rows": R_, "cfg_cols": C_, "cfg_A": A,
        "buf_frames": d.buffer.observation_buffer, "buf_actions": d.buffer.action_buffer,
        "buf_rewards": d.buffer.reward_buffer, "buf_continues": d.buffer.continue_buffer,
        "buf_size": d.buffer.size, "buf_next_idx": d.buffer.next_idx, "buf_capacity": d.buffer.capacity,
        "np_seed": np_seed, "starts": starts.astype(np.int64),
        "q_warm": q_warm.numpy(), "eps": eps.numpy(), "q": q.numpy(),
        "z0": z0.detach().numpy(), "h0": h0.detach().numpy(),
        "latents": lat.detach().numpy(), "hiddens": hid.detach().numpy(),
        "actions": acts_d.detach().numpy(), "rewards": rews_d.detach().numpy(),
        "continues": conts_d.detach().numpy(), "mus": mus.detach().numpy(),
        "sigmas": sigs.detach().numpy(), "R": R.numpy(),
        "loss_actor": la.detach().numpy(), "loss_critic": lc.detach().numpy(), "S_after": np.float32(S_after),
    }
    for k, g in zip(O.ACTOR_KEYS, rec["ga"]):
        out["gradc_agent." + k] = g.numpy()
    for k, g in zip(O.CRITIC_KEYS, rec["gc"]):
        out["gradc_agent." + k] = g.numpy()
    for k in list(sd1):
        if k.startswith("agent."):
            out["post_" + k] = sd1[k].numpy()
    if weights != "formula":
        for k, v in sd0.items():
            out["param_" + k] = v.numpy()
    return out


def blocks_case(cfg, weights, seed=5):
    """Per-block fixtures on the reference modules (teacher-forced inputs)."""
    d = build_reference(cfg, weights)
    wm, ag = d.world_model, d.agent
    B, A = 3, cfg["action_dims"]
    R_, C_ = cfg["latent_state_dims"]
    Hd = cfg["hidden_state_dims"]
    hw = tuple(cfg["observation_dims"])
    g = torch.Generator().manual_seed(seed)
    h = torch.randn(B, 1, Hd, generator=g)
    lg = torch.randn(B, 1, R_, C_, generator=g) * 2
    z = torch.nn.functional.one_hot(lg.argmax(-1), C_).float()
    a = torch.rand(B, 1, A, generator=g) * 2 - 1
    obs = torch.randint(0, 256, (B, 1, 3) + hw, generator=g).float() / 255.0 - 0.5
    out = {"h": h.numpy(), "z": z.numpy(), "a": a.numpy(), "obs": obs.numpy()}
    with torch.no_grad():
        out["gru"] = wm.sequence_model(z, h, a).numpy()
        out["enc_logits"] = wm.encoder(h, obs).numpy()
        out["prior_logits"] = wm.dynamics_predictor(h).numpy()
        out["reward"] = wm.reward_predictor.predict(h, z).numpy()
        out["reward_logits"] = wm.reward_predictor(h, z).numpy()
        p, l = wm.continue_predictor(h, z)
        out["cont_prob"], out["cont_logit"] = p.numpy(), l.numpy()
        mu, sg = ag.actor(h, z)
        out["actor_mu"], out["actor_sigma"] = mu.numpy(), sg.numpy()
        out["critic_value"] = ag.critic.value(h, z).numpy()
        out["critic_logits"] = ag.critic(h, z).numpy()
        # encoder.encode / prior.predict with recorded noise
        torch.manual_seed(seed + 1)
        ze, le = wm.encoder.encode(h, obs)
        zp, lp = wm.dynamics_predictor.predict(h)
        torch.manual_seed(seed + 1)
        out["q_enc"] = torch.empty(B * R_, C_).exponential_().numpy()
        out["q_prior"] = torch.empty(B * R_, C_).exponential_().numpy()
        out["enc_z"], out["prior_z"] = ze.numpy(), zp.numpy()
    # DreamerUtils
    from DreamerUtils import symexp, symlog, to_twohot
    v = torch.cat([torch.linspace(-30, 30, 41), torch.tensor([0.0, -20.0, 20.0, 1e-7, -1e-7, 3.0])]).view(-1, 1)
    out["u_v"] = v.numpy()
    out["u_symlog"] = symlog(v).numpy()
    out["u_symexp"] = symexp(v).numpy()
    out["u_twohot"] = to_twohot(symlog(v), torch.linspace(-20, 20, 255)).numpy()
    return out


def main():
    torch.set_num_threads(8)
    print("small config (reference default init, torch.manual_seed(0))")
    np.savez_compressed(os.path.join(HERE, "small_epoch.npz"), **run_case(SMALL, "init", 74, 1, 2))
    np.savez_compressed(os.path.join(HERE, "small_blocks.npz"), **blocks_case(SMALL, "init"))
    print("full width (formula weights)")
    np.savez_compressed(os.path.join(HERE, "full_epoch.npz"), **run_case(FULL, "formula", 40, 3, 4))
    np.savez_compressed(os.path.join(HERE, "full_blocks.npz"), **blocks_case(FULL, "formula"))
    # the reference's state_dict layout (names, shapes, order) for both configs
    import json
    lay = {}
    for name, cfg in (("small", SMALL), ("full", FULL)):
        d = build_reference(cfg, "init")
        lay[name] = [[k, list(v.shape)] for k, v in d.state_dict().items()]
    with open(os.path.join(HERE, "state_layout.json"), "w") as f:
        json.dump(lay, f)
    print("done")


if __name__ == "__main__":
    main()
