"""Index flips on NATURAL noise (no tie guard): one train_Agent epoch at the
north-star batch (B = 256, S = 64, H = 15) in fp32 parity mode and in bf16
perf mode against the fp32 CPU oracle on the same replay windows, weights and
explicit noise.  Run on the MI355X box: pytest -m gpu.

The guarded parity tests (test_gpu_baseline.py, test_gpu_bf16.py) push every
near-tie of the oracle's categorical draws apart before the run, so every
index must match.  Here nothing is pushed: a draw whose top two p_hat / q
scores are closer than the GPU's rounding error may pick the other class, and
that row's trajectory then diverges from the oracle's.  The test reports:

* the flip fraction of every draw of the epoch (31 warm-start steps' final z0
  and the 15 imagined steps);
* the fraction of batch rows whose trajectory diverged (any flipped index, or
  an h0 / hidden-state error above 1e-3 of the row's norm -- a flip inside the
  warm start that left z0 unchanged still shows in h0);
* losses, S, and the clipped gradients (normwise) against the oracle, with
  a yardstick: the same oracle epoch with the noise of the diverged rows
  re-drawn (what re-sampling those rows alone moves the gradients by).

The mu head is given non-zero weights (the reference's default init zeroes it,
Agent.py:188-189, which made every mus comparison vacuous).

Bounds: clipped gradients normwise <= 2 x yardstick + 1e-3 (fp32) / 2e-2
(bf16); fp32 -- at most 2 % of the rows diverge, losses within 1e-3
relative (first run, round 4: 0 flips, 0 rows diverged, mus 3.0e-7 and
hiddens 1.6e-7 normwise); bf16 -- at most 50 % of the rows diverge, losses
within 2e-2 relative (first run: flip fractions 5.2e-3 warm / 8.3e-3 dream,
88 of 256 rows diverged -- one flip in a row's 1,472 draws is enough; losses
6e-3 / 3e-4 relative).  These are statistical statements about natural noise,
not parity bounds; the parity bounds are the guarded tests'."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _nw(a, b):
    a, b = a.detach().float().cpu().reshape(-1), b.detach().float().cpu().reshape(-1)
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


class _NoGuard:
    """TieGuard-compatible context that changes nothing (natural noise)."""
    guarded = 0
    draws = 0

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_unguarded_flip_rate_B256(precision, gpu):
    import bench
    from baseline_case import oracle_epoch
    from test_gpu_baseline import CAR, run_gpu_epoch
    from dreamer_amd import Dreamer
    from oracle import dreamer_oracle as O
    B, S, H, R, C, A = 256, 64, 15, 32, 32, 3
    cfg = dict(CAR)
    cfg.update(batch_size=B, sequence_length=S, horizon=H, precision=precision)
    torch.manual_seed(0)
    d = Dreamer(cfg, gpu)
    g = torch.Generator().manual_seed(901)
    with torch.no_grad():
        d.agent.actor.mu_head.weight.copy_(torch.randn(d.agent.actor.mu_head.weight.shape, generator=g) * 0.05)
        d.agent.actor.mu_head.bias.copy_(torch.randn(d.agent.actor.mu_head.bias.shape, generator=g) * 0.1)
    P = {k: v.detach().cpu().clone() for k, v in d.state_dict().items()}
    n = 4096
    frames, acts, rews, conts = bench.synthetic_replay(n, (64, 64), A, seed=0)
    starts = np.random.RandomState(910).randint(0, n - S + 1, size=B)
    q_warm = torch.empty(S // 2, B * R, C).exponential_(generator=g)
    eps = torch.randn(H, B, 1, A, generator=g)
    q = torch.empty(H, B * R, C).exponential_(generator=g)
    idx = starts[:, None] + np.arange(S)[None, :]
    obs = torch.tensor(frames[idx], dtype=torch.float32)
    act = torch.tensor(acts[idx])
    S0 = 3.0
    torch.set_num_threads(16)
    ref = oracle_epoch(P, obs, act, S, H, R, C, q_warm.clone(), eps, q.clone(), S0, guard=_NoGuard())
    eng, pre = run_gpu_epoch(d, frames, acts, rews, conts, n, 0, starts, q_warm, eps, q, S0)
    lat, hid, act_r, rew, cont, mu, sg = ref["dream"]
    fw = eng.z0.cpu().reshape(B, R, C).argmax(-1) != ref["z0"].reshape(B, R, C).argmax(-1)
    fd = eng.latents.cpu().reshape(B, H + 1, R, C).argmax(-1) != lat.reshape(B, H + 1, R, C).argmax(-1)
    h0e = (eng.h0.cpu() - ref["h0"].reshape(B, -1)).norm(dim=-1) / ref["h0"].reshape(B, -1).norm(dim=-1)
    hde = (eng.hiddens.cpu().reshape(B, -1) - hid.reshape(B, -1)).norm(dim=-1) / hid.reshape(B, -1).norm(dim=-1)
    div = fw.any(-1) | fd.reshape(B, -1).any(-1) | (h0e > 1e-3) | (hde > 1e-3)
    ok = ~div
    m = dict(flip_warm_z0=float(fw.float().mean()), flip_dream=float(fd.float().mean()),
             rows_diverged=float(div.float().mean()), n_rows_diverged=int(div.sum()))
    # on the rows that followed the oracle's trajectory, the element-wise agreement
    if bool(ok.any()):
        m["mus_ok_rows"] = _nw(eng.mus.cpu()[ok], mu.reshape(B, H, A)[ok])
        m["hiddens_ok_rows"] = _nw(eng.hiddens.cpu()[ok], hid.reshape(B, H + 1, -1)[ok])
    la_ref, lc_ref = float(ref["ts"]["loss_actor"]), float(ref["ts"]["loss_critic"])
    m["loss_actor"] = (pre["la"], la_ref)
    m["loss_critic"] = (pre["lc"], lc_ref)
    m["S"] = (pre["S"], float(ref["ts"]["S"]))
    ag = d.agent
    for f, keys, grads, name in ((ag.fa, O.ACTOR_KEYS, ref["ts"]["grad_actor_clipped"], "grad_actor"),
                                 (ag.fc, O.CRITIC_KEYS, ref["ts"]["grad_critic_clipped"], "grad_critic")):
        want = torch.cat([gr.reshape(-1) for gr in grads])
        got = torch.cat([f.grad[f.offsets[k.split(".", 1)[1]]:f.offsets[k.split(".", 1)[1]] + gr.numel()].cpu()
                         for k, gr in zip(keys, grads)])
        m[name] = _nw(got, want)
    # Yardstick for the gradients: a diverged row is a different sample of the
    # same policy / world model.  Re-draw the noise of exactly those rows and
    # run the oracle again; the gradient distance between the two oracle
    # epochs is what the divergence alone moves the gradients by.
    yard = {"grad_actor": 0.0, "grad_critic": 0.0}
    if bool(div.any()):
        g2 = torch.Generator().manual_seed(977)
        rows = torch.nonzero(div).reshape(-1)
        q_warm2, eps2, q2 = q_warm.clone(), eps.clone(), q.clone()
        for b in rows.tolist():
            q_warm2[:, b * R:(b + 1) * R] = torch.empty(S // 2, R, C).exponential_(generator=g2)
            q2[:, b * R:(b + 1) * R] = torch.empty(H, R, C).exponential_(generator=g2)
            eps2[:, b] = torch.randn(H, 1, A, generator=g2)
        ref2 = oracle_epoch(P, obs, act, S, H, R, C, q_warm2, eps2, q2, S0, guard=_NoGuard())
        for grads, grads2, name in ((ref["ts"]["grad_actor_clipped"], ref2["ts"]["grad_actor_clipped"], "grad_actor"),
                                    (ref["ts"]["grad_critic_clipped"], ref2["ts"]["grad_critic_clipped"],
                                     "grad_critic")):
            yard[name] = _nw(torch.cat([x.reshape(-1) for x in grads2]), torch.cat([x.reshape(-1) for x in grads]))
    m["yardstick"] = yard
    print(f"{precision} epoch B=256 on NATURAL noise vs the fp32 oracle: {m}")
    assert float(mu.abs().max()) > 1e-3, "the mu head must be live for the mus comparison"
    # clipped gradients, normwise: at most twice what re-sampling the diverged
    # rows moves them by, plus the rounding floor of the mode
    floor = 1e-3 if precision == "fp32" else 2e-2
    for name in ("grad_actor", "grad_critic"):
        assert m[name] <= 2.0 * yard[name] + floor, (name, m)
    if precision == "fp32":
        assert m["rows_diverged"] <= 0.02, m
        rel = 1e-3
        if bool(ok.any()):
            assert m["mus_ok_rows"] <= 1e-4 and m["hiddens_ok_rows"] <= 1e-4, m
    else:
        # one flip anywhere in a row's 1,472 draws diverges the row; at the
        # measured per-draw flip rates (5e-3 warm / 8e-3 dream, round 4) about
        # a third of the rows diverge.  The bound is 50 % with the gradient
        # yardstick above as the check that the divergence is benign.
        assert m["rows_diverged"] <= 0.5, m
        rel = 2e-2
    assert abs(pre["lc"] - lc_ref) <= rel * abs(lc_ref), m
    assert abs(pre["la"] - la_ref) <= rel * max(abs(la_ref), 0.1), m
