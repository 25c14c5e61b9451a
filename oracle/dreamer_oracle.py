"""CPU oracle for the Dreamer imagination hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline.  The product path (``dreamer_amd``) never
imports it and fails loudly when its HIP library is missing.

This is a functional restatement (plain PyTorch on the CPU, fp32) of the
reference's hot path with the randomness made explicit: every draw the
reference takes from torch's global generator is an argument here
(``eps`` for the actor's reparameterised Normal sample, ``q`` for the
Exp(1) variates ``torch.multinomial`` uses to sample a Categorical).  Each
function cites the reference file:line it follows.  Parity is pinned: the
fixtures in ``tests/golden`` were produced by running the reference itself
(``tests/golden/make_golden.py``) and ``tests/test_oracle_golden.py`` checks
this module against them bit-for-bit.

Parameters are passed as a flat dict keyed by the reference's own
``state_dict`` names (``world_model.sequence_model.GRU.weight_ih`` ...).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

WM = "world_model."
AG = "agent."


# ----------------------------------------------------------------------------
# DreamerUtils.py
# ----------------------------------------------------------------------------
def symlog(x):  # DreamerUtils.py:29-30
    return torch.sign(x) * torch.log(1.0 + torch.abs(x))


def symexp(x):  # DreamerUtils.py:35-37
    x = torch.clamp(x, -20.0, 20.0)
    return torch.sign(x) * (torch.exp(torch.abs(x).float()) - 1.0)


def twohot(value, buckets):  # DreamerUtils.py:39-50
    v = torch.clamp(value, min=buckets.min(), max=buckets.max())
    lo = torch.searchsorted(buckets, v, right=True) - 1
    lo = torch.clamp(lo, max=buckets.numel() - 2)
    b_lo = buckets[lo]
    b_hi = buckets[lo + 1]
    w = (v - b_lo) / (b_hi - b_lo + 1e-8)
    out = torch.zeros(value.shape[:-1] + (buckets.shape[0],), dtype=torch.float32)
    out = torch.scatter(out, -1, lo, 1.0 - w)
    out = torch.scatter(out, -1, lo + 1, w)
    return out


# ----------------------------------------------------------------------------
# building blocks
# ----------------------------------------------------------------------------
def _lin(x, P, name):
    return F.linear(x, P[name + ".weight"], P[name + ".bias"])


def _ln(x, P, name):
    w = P[name + ".weight"]
    return F.layer_norm(x, (w.shape[0],), w, P[name + ".bias"], 1e-5)


def mlp3(x, P, pre):
    """Linear-LN-SiLU-Linear-LN-SiLU-Linear with Sequential indices 0,1,3,4,6.

    DynamicsPredictors.py:15-23 / 52-60 / 85-93, Agent.py:219-227."""
    x = F.silu(_ln(_lin(x, P, pre + ".0"), P, pre + ".1"))
    x = F.silu(_ln(_lin(x, P, pre + ".3"), P, pre + ".4"))
    return _lin(x, P, pre + ".6")


def sample_onehot(logits, q, cols):
    """softmax -> 1% unimix -> Categorical(probs).sample() -> one-hot + STE.

    VariationalAutoEncoder.py:88-98 and DynamicsPredictors.py:33-39.
    ``Categorical(probs)`` normalises p by its sum and ``multinomial(n=1)``
    draws ``argmax(p_hat / q)`` with q ~ Exp(1) of shape (rows, cols).
    Returns (latent (…,R,C) with STE, idx (…,R), probs (…,R,C))."""
    probs = torch.softmax(logits.float(), dim=-1)
    probs = 0.99 * probs + 0.01 * (1.0 / cols)
    p_hat = probs / probs.sum(-1, keepdim=True)
    flat = p_hat.reshape(-1, cols)
    idx = torch.argmax(flat / q.reshape(-1, cols), dim=-1).reshape(probs.shape[:-1])
    onehot = F.one_hot(idx, num_classes=cols).float()
    return onehot + probs - probs.detach(), idx, probs


# ----------------------------------------------------------------------------
# world model blocks
# ----------------------------------------------------------------------------
def gru(z, h, a, P):
    """SequenceModel.forward (SequenceModel.py:19-24): x = cat(flatten(z), a)."""
    x = torch.cat((z.flatten(2), a), dim=-1).squeeze(1)
    hn = torch.gru_cell(x, h.squeeze(1), P[WM + "sequence_model.GRU.weight_ih"],
                        P[WM + "sequence_model.GRU.weight_hh"],
                        P[WM + "sequence_model.GRU.bias_ih"],
                        P[WM + "sequence_model.GRU.bias_hh"])
    return hn.unsqueeze(1)


def gru_manual(x, h, w_ih, w_hh, b_ih, b_hh):
    """torch.nn.GRUCell semantics spelled out (gate order r, z, n)."""
    gi = F.linear(x, w_ih, b_ih)
    gh = F.linear(h, w_hh, b_hh)
    i_r, i_z, i_n = gi.chunk(3, -1)
    h_r, h_z, h_n = gh.chunk(3, -1)
    r = torch.sigmoid(i_r + h_r)
    u = torch.sigmoid(i_z + h_z)
    n = torch.tanh(i_n + r * h_n)
    return (1 - u) * n + u * h


def encoder_logits(h, obs, P):
    """Encoder.forward (VariationalAutoEncoder.py:57-75). obs already normalised.
    obs (B, S, D): the vector-observation stand-in of BASELINE configs[4]
    (Linear-SiLU x2; NOT in the reference -- parity of that mode is pinned
    only against this restatement of the framework's own definition,
    include/dreamer_hip.h dr_dims.obs_dim)."""
    if obs.dim() == 3:
        x = obs
        for i in (0, 2):
            x = F.silu(_lin(x, P, WM + f"encoder.feature_extractor.{i}"))
        feat = x
        inp = torch.cat((feat, h), dim=-1)
        y = F.silu(_ln(_lin(inp, P, WM + "encoder.latent_mapper.0"), P, WM + "encoder.latent_mapper.1"))
        return _lin(y, P, WM + "encoder.latent_mapper.3")
    B, S, C, Hh, Ww = obs.shape
    x = obs.reshape(B * S, C, Hh, Ww)
    # 4 convs (VAE.py:33-42), or 5 for BASELINE configs[3]'s "deeper VAE" (the framework's
    # encoder_depth key: one more k4 s2 p1 conv + SiLU; no reference definition -- parity of
    # that depth is pinned only against this restatement)
    i = 0
    while WM + f"encoder.feature_extractor.{i}.weight" in P:
        x = F.silu(F.conv2d(x, P[WM + f"encoder.feature_extractor.{i}.weight"],
                            P[WM + f"encoder.feature_extractor.{i}.bias"], stride=2, padding=1))
        i += 2
    feat = x.reshape(B, S, -1)
    inp = torch.cat((feat, h), dim=-1)
    y = F.silu(_ln(_lin(inp, P, WM + "encoder.latent_mapper.0"), P, WM + "encoder.latent_mapper.1"))
    return _lin(y, P, WM + "encoder.latent_mapper.3")


def encode(h, obs, P, q, rows, cols):
    """Encoder.encode (VariationalAutoEncoder.py:77-99). Returns (z, logits)."""
    B, S, _ = h.shape
    logits = encoder_logits(h, obs, P).view(B, S, rows, cols)
    z, _, _ = sample_onehot(logits, q, cols)
    return z, logits


def prior_logits(h, P, rows, cols):  # DynamicsPredictors.py:25-29
    lg = mlp3(h, P, WM + "dynamics_predictor.logit_net")
    B, S, _ = lg.shape
    return lg.view(B, S, rows, cols)


def prior_predict(h, P, q, rows, cols):  # DynamicsPredictors.py:31-40
    lg = prior_logits(h, P, rows, cols)
    z, _, _ = sample_onehot(lg, q, cols)
    return z, lg


def reward_predict(h, z, P):  # DynamicsPredictors.py:64-74
    lg = mlp3(torch.cat([h, z.flatten(2)], -1), P, WM + "reward_predictor.logit_net")
    probs = F.softmax(lg, dim=-1)
    return symexp(torch.sum(probs * P[WM + "reward_predictor.buckets_rew"], dim=-1, keepdim=True))


def continue_forward(h, z, P):  # DynamicsPredictors.py:95-100
    lg = mlp3(torch.cat([h, z.flatten(2)], -1), P, WM + "continue_predictor.logit_generator")
    return torch.sigmoid(lg), lg


def imagine_step(h, z, a, P, q, rows, cols):  # WorldModel.py:72-77
    h2 = gru(z, h, a, P)
    z2, _ = prior_predict(h2, P, q, rows, cols)
    r = reward_predict(h2, z2, P)
    c, _ = continue_forward(h2, z2, P)
    return h2, z2, r, c


def observe_step(z, h, a, obs, P, q, rows, cols):  # WorldModel.py:79-82
    h2 = gru(z, h, a, P)
    z2, lg = encode(h2, obs, P, q, rows, cols)
    return z2, h2, lg


# ----------------------------------------------------------------------------
# actor / critic (Agent.py)
# ----------------------------------------------------------------------------
def actor_forward(h, z, P):  # Agent.py:191-200
    st = torch.cat([h, z.flatten(2)], dim=-1)
    x = F.silu(_ln(_lin(st, P, AG + "actor.base_net.0"), P, AG + "actor.base_net.1"))
    x = F.silu(_ln(_lin(x, P, AG + "actor.base_net.3"), P, AG + "actor.base_net.4"))
    mu = _lin(x, P, AG + "actor.mu_head")
    ls = torch.clamp(_lin(x, P, AG + "actor.log_sig_head"), -5.0, 2.0)
    sigma = F.softplus(ls) + 1e-3
    return mu, sigma


def actor_act(h, z, P, eps=None):
    """Agent.py:202-210. rsample of TanhTransform(Normal) == tanh(mu + eps*sigma)."""
    mu, sigma = actor_forward(h, z, P)
    if eps is None:
        return torch.tanh(mu), mu, sigma
    return torch.tanh(mu + eps * sigma), mu, sigma


def critic_logits(h, z, P, which="critic"):  # Agent.py:231-235
    return mlp3(torch.cat([h, z.flatten(2)], dim=-1), P, AG + which + ".value_net")


def critic_value(h, z, P, which="critic"):  # Agent.py:237-241
    probs = F.softmax(critic_logits(h, z, P, which), dim=-1)
    return symexp(torch.sum(probs * P[AG + which + ".buckets_crit"], dim=-1, keepdim=True))


def lambda_returns(V, r, c, gamma=0.99, lam=0.95):
    """Agent.compute_batched_R_lambda_returns (Agent.py:156-172) given V (B,H+1,1)."""
    H = c.shape[1]
    nxt = r[:, -1] + gamma * c[:, -1] * V[:, -1]
    seq = [nxt]
    for t in reversed(range(H - 1)):
        R = r[:, t] + gamma * c[:, t] * ((1 - lam) * V[:, t + 1] + lam * nxt)
        seq.insert(0, R)
        nxt = R
    return torch.stack(seq, dim=1)


def update_S(S, R):
    """Agent.update_S (Agent.py:78-88). S is a python float or 0-d tensor."""
    if torch.isnan(R).any() or torch.isinf(R).any():
        return S
    flat = R.detach().flatten()
    rng = torch.max(torch.quantile(flat, 0.95) - torch.quantile(flat, 0.05),
                    torch.tensor(1.0, dtype=torch.float32))
    alpha = 1.0 - 0.99
    return (1.0 - alpha) * S + alpha * rng


def tanh_normal_logprob(a, mu, sigma):
    """TransformedDistribution(Normal(mu,sigma),[TanhTransform()]).log_prob(clamp(a))
    summed over the action dim (Agent.py:110-115)."""
    y = torch.clamp(a.detach(), -1.0 + 1e-6, 1.0 - 1e-6)
    x = torch.atanh(y)  # TanhTransform._inverse (torch 2.10)
    var = sigma ** 2
    lp = -((x - mu) ** 2) / (2 * var) - sigma.log() - math.log(math.sqrt(2 * math.pi))
    ladj = 2.0 * (math.log(2.0) - x - F.softplus(-2.0 * x))
    return (lp - ladj).sum(dim=-1)


# ----------------------------------------------------------------------------
# composite paths (Dreamer.py)
# ----------------------------------------------------------------------------
def normalise_obs(obs):  # Dreamer.py:251, WorldModel.py:156
    return (obs.float() / 255.0) - 0.5


def warm_start(obs, act, S, P, q_warm, rows, cols, batch_size=None):
    """Dreamer.warm_start_generator (Dreamer.py:244-262).

    obs (B,S,3,H,W) holding 0..255, act (B,S,A), q_warm (S//2, B*rows, cols).
    obs (B,S,D): vector observations, used as given (encoder_logits' note)."""
    obs = obs if obs.dim() == 3 else normalise_obs(obs)
    B = obs.shape[0] if batch_size is None else batch_size
    hidden = P[WM + "sequence_model.GRU.weight_hh"].shape[1]
    h = torch.zeros(B, 1, hidden, dtype=torch.float32)
    z, _ = encode(h, obs[:, 0:1], P, q_warm[0], rows, cols)
    for t in range(1, S // 2):
        z, h, _ = observe_step(z, h, act[:, t - 1:t], obs[:, t:t + 1], P, q_warm[t], rows, cols)
    return z, h


def dream(z0, h0, P, eps, q, horizon, rows, cols):
    """Dreamer.dream_episodes (Dreamer.py:143-175). eps (H,B,1,A), q (H,B*rows,cols)."""
    h, z = h0, z0
    hs, zs, rs, acts, cs, mus, sigs = [], [], [], [], [], [], []
    for t in range(horizon):
        a, mu, sg = actor_act(h, z, P, eps[t])
        h2, z2, r, c = imagine_step(h, z, a, P, q[t], rows, cols)
        hs.append(h); zs.append(z); rs.append(r); acts.append(a); cs.append(c)
        mus.append(mu); sigs.append(sg)
        h, z = h2, z2
    hs.append(h); zs.append(z)
    cat = lambda xs: torch.cat(xs, dim=1)
    return cat(zs), cat(hs), cat(acts), cat(rs), cat(cs), cat(mus), cat(sigs)


def ac_losses(z, h, r, c, a, mu, sigma, P, S, nu=3e-4, lam=0.95, gamma=0.99):
    """Agent.train_step loss construction (Agent.py:96-135). Returns
    (loss_actor, loss_critic, R, new_S)."""
    V_t = critic_value(h, z, P, "target_critic")
    R = lambda_returns(V_t, r, c, gamma, lam)
    base = critic_value(h.detach(), z.detach(), P, "critic")[:, :-1]
    adv = (R - base).detach().squeeze(-1)
    logp = tanh_normal_logprob(a, mu, sigma)
    S_new = update_S(S, R)
    norm = torch.max(torch.as_tensor(S_new, dtype=torch.float32), torch.tensor(1.0)).detach()
    loss_actor = torch.mean(-(logp * (adv / norm)) - (nu * (-logp)))
    lg = critic_logits(h.detach(), z.detach(), P, "critic")[:, :-1]
    th = twohot(symlog(R.detach()), P[AG + "critic.buckets_crit"])
    loss_critic = torch.mean(-torch.sum(th * F.log_softmax(lg, dim=-1), dim=-1))
    return loss_actor, loss_critic, R, S_new


def clip_grad_norm(grads, max_norm=100.0):
    """torch.nn.utils.clip_grad_norm_ semantics on a list of grads (Agent.py:147-148)."""
    total = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g, 2) for g in grads]), 2)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    return [g * coef for g in grads], total


def adamw_step(p, g, m, v, step, lr, betas=(0.9, 0.999), eps=1e-5, wd=1e-6):
    """torch.optim.AdamW single-tensor update (the CPU path the reference's
    optimisers take, Agent.py:63-76) for one parameter; returns new (p, m, v)."""
    b1, b2 = betas
    p = p.mul(1 - lr * wd)
    m = m.lerp(g, 1 - b1)
    v = v.mul(b2).addcmul(g, g, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = (v.sqrt() / (bc2 ** 0.5)).add(eps)
    return p.addcdiv(m, denom, value=-(lr / bc1)), m, v


ACTOR_KEYS = ["actor.base_net.0.weight", "actor.base_net.0.bias", "actor.base_net.1.weight",
              "actor.base_net.1.bias", "actor.base_net.3.weight", "actor.base_net.3.bias",
              "actor.base_net.4.weight", "actor.base_net.4.bias", "actor.mu_head.weight",
              "actor.mu_head.bias", "actor.log_sig_head.weight", "actor.log_sig_head.bias"]
CRITIC_KEYS = ["critic.value_net.0.weight", "critic.value_net.0.bias", "critic.value_net.1.weight",
               "critic.value_net.1.bias", "critic.value_net.3.weight", "critic.value_net.3.bias",
               "critic.value_net.4.weight", "critic.value_net.4.bias", "critic.value_net.6.weight",
               "critic.value_net.6.bias"]


def train_step(z, h, r, c, a, mu, sigma, P, S, actor_params, critic_params,
               nu=3e-4, lam=0.95, gamma=0.99):
    """Loss + gradients of Agent.train_step (Agent.py:96-148), pre-optimiser.

    ``actor_params``/``critic_params`` are the leaf tensors (requires_grad)
    that ``mu``/``sigma`` and the critic were built from.  Returns a dict with
    losses, R, new S, raw grads and clipped grads (lists in *_KEYS order)."""
    la, lc, R, S_new = ac_losses(z, h, r, c, a, mu, sigma, P, S, nu, lam, gamma)
    gc = torch.autograd.grad(lc, critic_params, allow_unused=True)
    ga = torch.autograd.grad(la, actor_params, allow_unused=True)
    gc = [torch.zeros_like(p) if g is None else g for g, p in zip(gc, critic_params)]
    ga = [torch.zeros_like(p) if g is None else g for g, p in zip(ga, actor_params)]
    gc_c, nc = clip_grad_norm(gc)
    ga_c, na = clip_grad_norm(ga)
    return dict(loss_actor=la.detach(), loss_critic=lc.detach(), R=R.detach(), S=S_new,
                grad_actor=[g.detach() for g in ga], grad_critic=[g.detach() for g in gc],
                grad_actor_clipped=[g.detach() for g in ga_c],
                grad_critic_clipped=[g.detach() for g in gc_c],
                norm_actor=na.detach(), norm_critic=nc.detach())


def replay_starts(size, capacity, next_idx, seq_len, batch, rng=None):
    """Buffer.sample_sequences start-index logic (Buffer.py:36-48) on numpy's
    legacy global RNG (or the given RandomState)."""
    import numpy as np
    r = np.random if rng is None else rng
    valid = size - seq_len + 1
    starts = r.randint(0, valid, size=batch)
    if size == capacity:
        out = []
        for s in starts:
            if s < next_idx < s + seq_len:
                out.append(r.randint(0, valid))
            else:
                out.append(s)
        starts = np.array(out)
    return starts


# ----------------------------------------------------------------------------
# world-model training step (WorldModel.py:84-202, VariationalAutoEncoder.py:139-161)
# ----------------------------------------------------------------------------
def decoder_forward(h, z, P, img_hw):
    """Decoder.forward (VariationalAutoEncoder.py:139-161): cat(h, flatten z) ->
    Linear-LN-SiLU-Linear-SiLU -> view (C0, H/16, W/16) -> 4x ConvTranspose2d
    (k4 s2 p1) with SiLU between and Tanh at the end (the deeper VAE of
    configs[3]: H/32, 5 transposed convs -- encoder_logits' note)."""
    B, S, Hd = h.shape
    x = torch.cat((h.reshape(B * S, Hd), z.reshape(B * S, -1)), dim=-1)
    D = WM + "decoder."
    x = F.silu(_ln(_lin(x, P, D + "upscaler.0"), P, D + "upscaler.1"))
    x = F.silu(_lin(x, P, D + "upscaler.3"))
    if D + "image_builder.4.weight" not in P:  # vector-observation stand-in (encoder_logits' note)
        x = F.silu(_lin(x, P, D + "image_builder.0"))
        return _lin(x, P, D + "image_builder.2").view(B, S, -1)
    c0 = P[D + "image_builder.0.weight"].shape[0]
    depth = sum(1 for k in P if k.startswith(D + "image_builder.") and k.endswith(".weight"))  # 4, or 5 (configs[3])
    x = x.view(-1, c0, img_hw[0] // 2 ** depth, img_hw[1] // 2 ** depth)
    for j in range(depth):
        i = 2 * j
        x = F.conv_transpose2d(x, P[D + f"image_builder.{i}.weight"], P[D + f"image_builder.{i}.bias"],
                               stride=2, padding=1)
        x = torch.tanh(x) if j == depth - 1 else F.silu(x)
    _, C, Hh, Ww = x.shape
    return x.view(B, S, C, Hh, Ww)


def wm_unroll(obs, act, rew, cont, P, q, rows, cols, horizon):
    """WorldModel.unroll_model (WorldModel.py:84-146); obs normalised.
    q: (horizon, B*rows, cols) Exp(1) draws of the posterior samples."""
    B = cont.shape[0]
    Hd = P[WM + "sequence_model.GRU.weight_hh"].shape[1]
    A = act.shape[-1]
    h = torch.zeros(B, 1, Hd, dtype=torch.float32)
    z = torch.zeros(B, 1, rows, cols, dtype=torch.float32)
    zs, hs, lgs = [], [], []
    for t in range(horizon):
        a = act[:, t - 1:t] if t > 0 else torch.zeros(B, 1, A)
        z, h, lg = observe_step(z, h, a, obs[:, t:t + 1], P, q[t], rows, cols)
        zs.append(z); hs.append(h); lgs.append(lg)
    post_logits, hid, lat = torch.cat(lgs, 1), torch.cat(hs, 1), torch.cat(zs, 1)
    prior = prior_logits(hid, P, rows, cols)
    dec_mu = decoder_forward(hid, lat, P, tuple(obs.shape[-2:]))
    rin = torch.cat([hid[:, 1:], lat[:, 1:].flatten(2)], -1)
    rew_logits = mlp3(rin, P, WM + "reward_predictor.logit_net")
    cont_logits = mlp3(rin, P, WM + "continue_predictor.logit_generator")
    obs_t, rew_t, cont_t = obs[:, :horizon], rew[:, :horizon - 1], cont[:, :horizon - 1]
    th = twohot(rew_t, P[WM + "reward_predictor.buckets_rew"])
    obs_ll = -(dec_mu.float() - obs_t.float()).pow(2).sum(dim=[-1] if obs.dim() == 3 else [-3, -2, -1])
    cont_ll = F.binary_cross_entropy_with_logits(cont_logits, cont_t, reduction="none")
    rew_ll = torch.sum(th * F.log_softmax(rew_logits, dim=-1), dim=-1, keepdim=True)
    return dict(prior=prior[:, 1:], post=post_logits[:, 1:], obs_ll=obs_ll[:, 1:], rew_ll=rew_ll,
                cont_ll=cont_ll, hiddens=hid, latents=lat, post_logits=post_logits, dec_mu=dec_mu)


def _cat_kl(p_logits, q_logits):
    """kl_divergence(Categorical(logits=p), Categorical(logits=q)) over the last
    dim (torch.distributions.kl._kl_categorical_categorical)."""
    lp = p_logits - p_logits.logsumexp(-1, keepdim=True)
    lq = q_logits - q_logits.logsumexp(-1, keepdim=True)
    t = lp.exp() * (lp - lq)
    return t.sum(-1)


def wm_losses(obs_u8, act, rew, cont, P, q, rows, cols, horizon, betas=(1.0, 0.5, 0.1)):
    """WorldModel.training_step loss construction (WorldModel.py:148-189) with
    autocast disabled (fp32).  Returns a dict of losses (0-d tensors) and the
    unroll outputs."""
    obs = obs_u8 if obs_u8.dim() == 3 else normalise_obs(obs_u8)  # vector observations: as given
    H = horizon
    u = wm_unroll(obs[:, :H], act[:, :H], rew[:, :H], cont[:, :H], P, q, rows, cols, H)
    mask = cont[:, :H - 1]
    obs_ll = u["obs_ll"] * mask.squeeze(-1)
    rew_ll = u["rew_ll"] * mask
    cont_ll = u["cont_ll"] * mask
    prior, post = u["prior"].float(), u["post"].float()
    kl_dyn = _cat_kl(post.detach(), prior).sum(dim=-1)
    kl_rep = _cat_kl(post, prior.detach()).sum(dim=-1)
    kl_dyn = torch.mean(kl_dyn * mask.squeeze(-1))
    kl_rep = torch.mean(kl_rep * mask.squeeze(-1))
    denom = mask.sum() + 1e-5
    loss_pred = (-obs_ll.sum() - rew_ll.sum() + cont_ll.sum()) / denom
    one = torch.tensor(1.0)
    loss_dyn, loss_rep = torch.max(one, kl_dyn), torch.max(one, kl_rep)
    total = betas[0] * loss_pred + betas[1] * loss_dyn + betas[2] * loss_rep
    return dict(total=total, loss_pred=loss_pred, kl_dyn=kl_dyn, kl_rep=kl_rep, loss_dyn=loss_dyn,
                loss_rep=loss_rep, **u)


def wm_train_step(obs_u8, act, rew, cont, P, q, rows, cols, horizon, wm_keys, betas=(1.0, 0.5, 0.1)):
    """Loss + gradients of WorldModel.training_step (WorldModel.py:148-198),
    pre-optimiser.  ``wm_keys`` are the world-model parameter names in
    ``WorldModel.parameters()`` order; P must hold leaf tensors for them with
    requires_grad.  Returns losses, raw and clipped grads (clip 100, as
    clip_grad_norm_ at WorldModel.py:198) and the total norm."""
    out = wm_losses(obs_u8, act, rew, cont, P, q, rows, cols, horizon, betas)
    params = [P[k] for k in wm_keys]
    g = torch.autograd.grad(out["total"], params, allow_unused=True)
    g = [torch.zeros_like(p) if gi is None else gi for gi, p in zip(g, params)]
    gc, norm = clip_grad_norm(g)
    out.update(grads=[x.detach() for x in g], grads_clipped=[x.detach() for x in gc], norm=norm.detach())
    return out
