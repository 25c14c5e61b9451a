"""Inputs of the BASELINE-shape parity cases, regenerated deterministically
(test infrastructure).

* ``regen_fixture(fx)``: the replay frames and the reference's noise draws of
  ``tests/golden/baseline_b16.npz`` (see make_golden_baseline.py), checked
  against the digests the generator recorded from the reference run.
* ``oracle_epoch(...)``: one train_Agent epoch on the CPU oracle with
  tie-guarded noise (below), returning everything the GPU tests compare.

Tie guard.  A categorical draw is argmax_c(p_hat_c / q_c).  When the top two
scores of a group are within a relative 1e-4 the fp32 GPU and the CPU can
legitimately pick different classes (summation order), and one flip then
changes that row's whole trajectory.  The guard runs the oracle once and, for
every such group, scales the Exp(1) variate of every runner-up within that
margin up by (1 + 4e-4) before the draw (TieGuard(rel, scale) widens the
margin further for the bf16-mode tests).  The oracle's own choice (and so every oracle output) is
unchanged; the guarded noise then leaves every group a margin of at least
~3e-4, far above fp32 error, so the GPU must reproduce every index exactly.
The number of guarded groups is reported.
"""
import hashlib

import numpy as np
import torch

from formula import formula_state_dict, replay_data
from oracle import dreamer_oracle as O

TIE_REL = 1e-4
TIE_SCALE = 1.0 + 4e-4


def digest(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()[:8], dtype=np.int64)[0]


def reference_noise(torch_seed, B, S, H, R, C, A):
    """The reference's draws in order (make_golden.run_case)."""
    torch.manual_seed(torch_seed)
    q_warm = torch.stack([torch.empty(B * R, C).exponential_() for _ in range(S // 2)])
    eps, q = [], []
    for _ in range(H):
        eps.append(torch.empty(B, 1, A).normal_())
        q.append(torch.empty(B * R, C).exponential_())
    return q_warm, torch.stack(eps), torch.stack(q)


def regen_fixture(fx, shapes):
    """(P, frames, q_warm, eps, q) for baseline_b16.npz; asserts the digests."""
    B, S, H, R, C, A = (int(fx[k]) for k in ("cfg_B", "cfg_S", "cfg_H", "cfg_rows", "cfg_cols", "cfg_A"))
    n, cap = int(fx["n_fill"]), int(fx["buf_capacity"])
    fr, _, _, _ = replay_data(n, (64, 64), A, seed=0)
    frames = np.zeros((cap, 3, 64, 64), dtype=np.uint8)
    frames[:n] = fr
    assert digest(frames) == int(fx["frames_digest"]), "replay frames regeneration drifted"
    q_warm, eps, q = reference_noise(int(fx["torch_seed"]), B, S, H, R, C, A)
    for k, t in (("q_warm", q_warm), ("eps", eps), ("q", q)):
        assert digest(t.numpy()) == int(fx[k + "_digest"]), f"{k} regeneration drifted"
    return formula_state_dict(shapes), frames, q_warm, eps, q


class TieGuard:
    """Context manager: O.sample_onehot widens near-tie margins in the q it is
    given (in place) without changing its own argmax."""

    def __init__(self, rel=TIE_REL, scale=TIE_SCALE):
        self.rel, self.scale = rel, scale
        self.guarded = 0
        self.draws = 0

    def __enter__(self):
        self._orig = O.sample_onehot
        guard = self

        def sample(logits, q, cols):
            probs = torch.softmax(logits.float(), dim=-1)
            probs = 0.99 * probs + 0.01 * (1.0 / cols)
            p_hat = (probs / probs.sum(-1, keepdim=True)).reshape(-1, cols)
            qf = q.reshape(-1, cols)
            score = p_hat / qf
            top = score.max(dim=-1, keepdim=True)
            # every runner-up within a relative `rel` of the top score is pushed
            # down by `scale` (the top class, and so the oracle's draw, unchanged)
            near = (score > top.values * (1.0 - guard.rel)) & \
                (torch.arange(cols).view(1, -1) != top.indices)
            qf[near] = qf[near] * guard.scale  # in place: the caller's noise tensor
            near = near.any(dim=-1).nonzero().flatten()
            guard.guarded += int(len(near))
            guard.draws += int(qf.shape[0])
            return guard._orig(logits, q, cols)

        O.sample_onehot = sample
        return self

    def __exit__(self, *exc):
        O.sample_onehot = self._orig
        return False


def oracle_epoch(P, obs_u8, act, S, H, R, C, q_warm, eps, q, S0, guard=None):
    """CPU oracle train_Agent epoch (Dreamer.py:264-287) with the tie guard:
    warm start, dream, train_step, clip, AdamW (step 1), soft target."""
    with (guard or TieGuard()) as tg:
        z0, h0 = O.warm_start(obs_u8, act, S, P, q_warm, R, C)
        ap = [P["agent." + k].clone().requires_grad_(True) for k in O.ACTOR_KEYS]
        cp = [P["agent." + k].clone().requires_grad_(True) for k in O.CRITIC_KEYS]
        P2 = dict(P)
        P2.update({"agent." + k: t for k, t in zip(O.ACTOR_KEYS, ap)})
        P2.update({"agent." + k: t for k, t in zip(O.CRITIC_KEYS, cp)})
        d = O.dream(z0.detach(), h0.detach(), P2, eps, q, H, R, C)
    ts = O.train_step(*(d[i] for i in (0, 1, 3, 4, 2, 5, 6)), P2, S0, ap, cp)
    post = {}
    for keys, grads, lr in ((O.ACTOR_KEYS, ts["grad_actor_clipped"], 8e-5), (O.CRITIC_KEYS, ts["grad_critic_clipped"], 1e-4)):
        for k, g in zip(keys, grads):
            p = P["agent." + k]
            pn, _, _ = O.adamw_step(p, g, torch.zeros_like(p), torch.zeros_like(p), 1, lr)
            post["agent." + k] = pn
    for k in O.CRITIC_KEYS:
        post["agent.target_" + k] = P["agent.target_" + k] * 0.98 + 0.02 * post["agent." + k]
    return dict(z0=z0.detach(), h0=h0.detach(), dream=[t.detach() for t in d], ts=ts, post=post,
                guarded=tg.guarded, draws=tg.draws)
