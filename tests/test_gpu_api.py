"""The reference's public API on the HIP path (drop-in contract),
called exactly as train_car_racer.py / Dreamer.train_dreamer call it, against
the CPU oracle on the same inputs.  One-off calls draw their noise from the
ad-hoc generator; ``hip.noise_override`` feeds them the oracle's explicit
variates (parity mode).  Run on the MI355X box: pytest -m gpu.

Tolerances as test_gpu_baseline.py: |d| <= 1e-5 + 1e-4 |ref| on hidden
states, logits and heads; categorical indices exact (inputs are tie-guarded)."""
import os

import numpy as np
import pytest
import torch

from baseline_case import TieGuard
from conftest import state_layout
from formula import FULL, formula_state_dict, replay_data
from gpu_helpers import close, cpu
from oracle import dreamer_oracle as O

pytestmark = pytest.mark.gpu
R, C, A, HD = 32, 32, 3, 600


def _dreamer(dev, formula=True, **over):
    """CarRacing widths; formula weights (or the default init for other widths)."""
    from dreamer_amd import Dreamer
    cfg = dict(FULL)
    cfg.update(over)
    torch.manual_seed(0)
    d = Dreamer(cfg, dev)
    if not formula:
        return d, None
    P = formula_state_dict(dict(state_layout("full")))
    d.load_state_dict({k: v.to(dev) for k, v in P.items()})
    return d, P


def _inputs(B, seed=3):
    g = torch.Generator().manual_seed(seed)
    h = torch.randn(B, 1, HD, generator=g)
    lg = torch.randn(B, 1, R, C, generator=g) * 2
    z = torch.nn.functional.one_hot(lg.argmax(-1), C).float()
    a = torch.rand(B, 1, A, generator=g) * 2 - 1
    obs = torch.randint(0, 256, (B, 1, 3, 64, 64), generator=g).float() / 255.0 - 0.5
    q = torch.empty(1, B * R, C).exponential_(generator=g)
    eps = torch.randn(1, B, A, generator=g)
    return h, z, a, obs, q, eps


def _idx(z):
    return cpu(z).reshape(-1, C).argmax(-1)


def test_warm_start_generator_api(gpu):
    """Dreamer.warm_start_generator(obs 0..255, act, S) (Dreamer.py:244-262)."""
    from dreamer_amd import hip
    B, S = 4, 16
    d, P = _dreamer(gpu, batch_size=B, sequence_length=S)
    fr, ac, _, _ = replay_data(64, (64, 64), A, seed=5)
    idx = np.arange(S)[None, :] + np.array([0, 7, 21, 40])[:, None]
    obs = torch.tensor(fr[idx], dtype=torch.float32)
    act = torch.tensor(ac[idx])
    q = torch.empty(S // 2, B * R, C).exponential_(generator=torch.Generator().manual_seed(9))
    with TieGuard():
        z_ref, h_ref = O.warm_start(obs, act, S, P, q, R, C)
    with hip.noise_override(q=q.to(gpu)):
        z, h = d.warm_start_generator(obs.to(gpu), act.to(gpu), S)
    assert torch.equal(_idx(z), _idx(z_ref))
    close(h, h_ref, 1e-4, 1e-5, "warm_start_generator h")
    close(z, z_ref, 0, 1.2e-7, "warm_start_generator z (straight-through value)")


@pytest.mark.parametrize("soft", [False, True])
def test_observe_step_and_encode_api(soft, gpu):
    """WorldModel.observe_step (WorldModel.py:79-82) and Encoder.encode
    (VAE.py:77-99); soft=True feeds a non-one-hot latent (dense GRU groups)."""
    from dreamer_amd import hip
    B = 3
    d, P = _dreamer(gpu)
    h, z, a, obs, q, _ = _inputs(B)
    if soft:
        z = torch.softmax(torch.randn(B, 1, R, C, generator=torch.Generator().manual_seed(4)), -1)
    with TieGuard():
        z_ref, h_ref, lg_ref = O.observe_step(z, h, a, obs, P, q[0], R, C)
        ze_ref, le_ref = O.encode(h, obs, P, q[0], R, C)
    wm = d.world_model
    with torch.no_grad(), hip.noise_override(q=q.to(gpu)):
        z2, h2, lg = wm.observe_step(z.to(gpu), h.to(gpu), a.to(gpu), obs.to(gpu))
        ze, le = wm.encoder.encode(h.to(gpu), obs.to(gpu))
    close(h2, h_ref, 1e-4, 1e-5, "observe_step h")
    close(lg, lg_ref, 1e-4, 1e-5, "observe_step logits")
    assert torch.equal(_idx(z2), _idx(z_ref))
    close(le, le_ref, 1e-4, 1e-5, "encode logits")
    assert torch.equal(_idx(ze), _idx(ze_ref))


@pytest.mark.parametrize("soft", [False, True])
def test_imagine_step_api(soft, gpu):
    """WorldModel.imagine_step (WorldModel.py:72-77) and SequenceModel."""
    from dreamer_amd import hip
    B = 3
    d, P = _dreamer(gpu)
    h, z, a, _, q, _ = _inputs(B, seed=6)
    if soft:
        z = torch.softmax(torch.randn(B, 1, R, C, generator=torch.Generator().manual_seed(5)), -1)
    with TieGuard():
        h_ref, z_ref, r_ref, c_ref = O.imagine_step(h, z, a, P, q[0], R, C)
    wm = d.world_model
    with torch.no_grad(), hip.noise_override(q=q.to(gpu)):
        h2, z2, r, c = wm.imagine_step(h.to(gpu), z.to(gpu), a.to(gpu))
        hs = wm.sequence_model(z.to(gpu), h.to(gpu), a.to(gpu))
    close(hs, O.gru(z, h, a, P), 1e-4, 1e-5, "SequenceModel")
    close(h2, h_ref, 1e-4, 1e-5, "imagine_step h")
    assert torch.equal(_idx(z2), _idx(z_ref))
    close(r, r_ref, 1e-4, 1e-5, "imagine_step reward")
    close(c, c_ref, 1e-4, 1e-6, "imagine_step continue")


@pytest.mark.parametrize("widths", [(200, 200), (64, 256)])
def test_actor_act_batch1(widths, gpu):
    """Actor.act at B = 1 (rollout_policy / evaluate_agent / Run) with the
    CarRacing widths and with actor_h2 > actor_h1 (workspace)."""
    from dreamer_amd import hip
    d, _ = _dreamer(gpu, formula=widths == (200, 200), hidden_layer_actor_1_size=widths[0],
                    hidden_layer_actor_2_size=widths[1])
    P = {k: v.detach().cpu() for k, v in d.state_dict().items()}
    h, z, _, _, _, eps = _inputs(1, seed=8)
    mu_ref, sg_ref = O.actor_forward(h, z, P)
    with torch.no_grad():
        a, mu, sg = d.agent.actor.act(h.to(gpu), z.to(gpu), deterministic=True)
        close(mu, mu_ref, 1e-4, 1e-5, "act mu")
        close(sg, sg_ref, 1e-4, 1e-6, "act sigma")
        close(a, torch.tanh(mu_ref), 1e-4, 1e-6, "act deterministic")
        with hip.noise_override(eps=eps.to(gpu)):
            a2, _, _ = d.agent.actor.act(h.to(gpu), z.to(gpu), deterministic=False)
    close(a2, torch.tanh(mu_ref + eps.view(1, 1, A) * sg_ref), 1e-4, 1e-6, "act sample")


@pytest.mark.parametrize("B", [4, 16])
def test_dream_episodes_from_soft_latent(B, gpu):
    """Dreamer.dream_episodes (Dreamer.py:143-175) from a non-one-hot z0 (B = 16:
    the persistent unroll's dense-group path, dream.hip)."""
    H = 5
    d, P = _dreamer(gpu, batch_size=B, horizon=H)
    g = torch.Generator().manual_seed(12)
    h0 = torch.randn(B, 1, HD, generator=g)
    z0 = torch.softmax(torch.randn(B, 1, R, C, generator=g), -1)
    eps = torch.randn(H, B, 1, A, generator=g)
    q = torch.empty(H, B * R, C).exponential_(generator=g)
    with TieGuard():
        ref = O.dream(z0, h0, P, eps, q, H, R, C)
    out = d._imagine_raw(z0.to(gpu), h0.to(gpu), eps=eps.to(gpu), q=q.to(gpu))[0]
    close(out[1], ref[1], 1e-4, 1e-5, "dream hiddens (soft z0)")
    assert torch.equal(_idx(out[0][:, 1:]), _idx(ref[0][:, 1:]))
    close(out[3], ref[3], 1e-4, 1e-5, "dream rewards (soft z0)")


def test_train_world_model_api(gpu):
    """Dreamer.train_world_model (Dreamer.py:228-242): the losses it returns
    equal the oracle's WorldModel.training_step loss on the same windows."""
    from dreamer_amd import hip
    B, S, H = 4, 16, 6
    d, P = _dreamer(gpu, batch_size=B, sequence_length=S, horizon=H, buffer_size=64)
    fr, ac, rw, ct = replay_data(64, (64, 64), A, seed=7)
    rws = O.symlog(torch.tensor(rw)).numpy()
    d.buffer.load_arrays(fr, ac, rws, ct)
    np.random.seed(3)
    starts = d.buffer.sample_start_indices(B)
    q = torch.empty(H, B * R, C).exponential_(generator=torch.Generator().manual_seed(13))
    idx = starts[:, None] + np.arange(S)[None, :]
    with TieGuard():
        ref = O.wm_losses(torch.tensor(fr[idx], dtype=torch.float32), torch.tensor(ac[idx]),
                          torch.tensor(rws[idx]).unsqueeze(-1), torch.tensor(ct[idx]).unsqueeze(-1), P, q, R, C, H)
    np.random.seed(3)
    with hip.noise_override(q=q.to(gpu)):
        losses = d.train_world_model()
    assert len(losses) == 1 and losses[0].dim() == 0
    assert abs(float(losses[0]) - float(ref["total"])) <= 1e-4 * abs(float(ref["total"])), \
        (float(losses[0]), float(ref["total"]))


def test_train_agent_api_matches_engine(gpu):
    """Dreamer.train_Agent() (Dreamer.py:264-287) with AC_epochs = 1 and 2 is
    the engine's epoch(s) on the same np.random window draws, bit for bit."""
    from dreamer_amd.engine import ImaginationEngine
    B, S, H = 8, 16, 5
    res = []
    for mode in ("api", "engine"):
        d, _ = _dreamer(gpu, batch_size=B, sequence_length=S, horizon=H, buffer_size=128, AC_epochs=2)
        fr, ac, rw, ct = replay_data(128, (64, 64), A, seed=2)
        d.buffer.load_arrays(fr, ac, O.symlog(torch.tensor(rw)).numpy(), ct)
        d._engine = ImaginationEngine(d)
        d._engine.rng.reseed(77)
        np.random.seed(21)
        if mode == "api":
            la, lc = d.train_Agent()
            la, lc = float(la), float(lc)
        else:
            ls = []
            for _ in range(2):
                a, c = d._engine.run(d.buffer.sample_start_indices(B))  # views of the loss slots
                ls.append((float(a), float(c)))
            la, lc = np.mean([x[0] for x in ls], dtype=np.float32), np.mean([x[1] for x in ls], dtype=np.float32)
        torch.cuda.synchronize()
        res.append((la, lc, cpu(d.agent.fa.flat), cpu(d.agent.fc.flat)))
    (a1, c1, fa1, fc1), (a2, c2, fa2, fc2) = res
    assert abs(a1 - a2) <= 1e-6 * max(1.0, abs(a2)) and abs(c1 - c2) <= 1e-6 * abs(c2)
    assert torch.equal(fa1, fa2) and torch.equal(fc1, fc2)


class _Space:
    def __init__(self, rng):
        self.rng = rng

    def sample(self):
        return self.rng.uniform(-1, 1, size=3).astype(np.float32)


class FakeCarRacing:
    """gymnasium-shaped env (reset / step / action_space.sample) with 64x64x3
    u8 frames, ending an episode every `length` steps."""

    def __init__(self, length=9, seed=0):
        self.rng = np.random.default_rng(seed)
        self.action_space = _Space(self.rng)
        self.length = length
        self.t = 0

    def _obs(self):
        return self.rng.integers(0, 256, size=(64, 64, 3), dtype=np.uint8)

    def reset(self, seed=None):
        self.t = 0
        return self._obs(), {}

    def step(self, action):
        a = np.asarray(action, dtype=np.float32)
        assert a.shape == (3,) and np.all(np.isfinite(a)) and np.all(np.abs(a) <= 1.0)
        self.t += 1
        return self._obs(), float(np.tanh(a.sum())), self.t >= self.length, False, {}

    def render(self):
        pass


@pytest.mark.parametrize("formula", [True, False])
def test_train_dreamer_with_fake_env(formula, gpu, tmp_path, monkeypatch):
    """Dreamer.train_dreamer(env, eval_env) end to end (train_car_racer.py:38):
    random kick-start, world-model and agent training iterations, evaluation,
    checkpoint + training-log files; then Run() and a reference-format reload."""
    monkeypatch.chdir(tmp_path)
    # the closed-form parity weights (formula=True) and the default init: in
    # rounds 2-3 the formula-weight run went non-finite on some Philox draws;
    # on the round-4 tree both run finite (profiles/r04o_fake_env_tests.txt)
    # and the failing draws no longer occur, so no single change is pinned
    # as the fix
    d, _ = _dreamer(gpu, formula=formula, batch_size=4, sequence_length=16, horizon=5, buffer_size=256,
                    random_iterations=2, training_iterations=2, AC_epochs=2)
    env, eval_env = FakeCarRacing(seed=1), FakeCarRacing(seed=2)
    wm, al, cl, ev = d.train_dreamer(env, eval_env)
    assert len(wm) == 2 + 2 and len(al) == 2 and len(cl) == 2 and len(ev) == 1 + 1 + 1
    for x in [v for row in wm for v in row] + al + cl + ev:
        assert np.isfinite(x)
    assert d.buffer.size == (2 + 2) * 16
    assert os.path.exists("models/agent_latest.pth") and os.path.exists("models/agent_checkpoint_0.pth")
    with np.load("models/training_logs.npz", allow_pickle=False) as f:
        assert set(f.files) == {"world_model_loss", "actor_loss", "critic_loss", "rewards"}
    total = d.Run(FakeCarRacing(seed=3), env_seed=0, render=True)
    assert np.isfinite(total)
    sd = torch.load("models/agent_latest.pth", weights_only=True)
    d2, _ = _dreamer(gpu, batch_size=4, sequence_length=16, horizon=5)
    d2.load_pretrained_dreamer("models/agent_latest.pth")
    assert all(torch.equal(v.cpu(), sd[k].cpu()) for k, v in d2.state_dict().items())


def test_training_state_resume(gpu, tmp_path):
    """save_training_state / load_training_state (true resume: weights, the
    three AdamW states, S, Philox / numpy / torch generators, replay ring):
    a resumed run repeats the uninterrupted run's next iteration bit for bit
    (the reference saves weights only, Dreamer.py:289-293)."""
    from formula import replay_data
    kw = dict(batch_size=8, sequence_length=16, horizon=5, buffer_size=256, AC_epochs=1, WM_epochs=1)
    d, _ = _dreamer(gpu, formula=False, **kw)
    fr, ac, rw, ct = replay_data(256, (64, 64), A, seed=11)
    d.buffer.load_arrays(fr, ac, rw, ct)
    np.random.seed(1)
    d.train_world_model()
    d.train_Agent()
    path = tmp_path / "state.pt"
    d.save_training_state(path)

    def iteration(dr):
        wm = float(dr.train_world_model()[0])
        la, lc = dr.train_Agent()
        torch.cuda.synchronize()
        return wm, float(la), float(lc), {k: v.detach().cpu().clone() for k, v in dr.state_dict().items()}

    ref = iteration(d)
    torch.manual_seed(123)  # a different process state before the resume
    np.random.seed(99)
    d2, _ = _dreamer(gpu, formula=False, **kw)
    d2.load_training_state(path)
    got = iteration(d2)
    assert got[:3] == ref[:3], (got[:3], ref[:3])
    for k in ref[3]:
        assert torch.equal(got[3][k], ref[3][k]), k
    # the file is plain tensors / scalars: loads with weights_only=True
    st = torch.load(path, weights_only=True)
    assert st["format"] == "dreamer_amd.training_state.v1" and len(st["model"]) == len(ref[3])


def test_act_step_matches_oracle(gpu):
    """dr_act_step (the one-launch env step) against the CPU oracle directly:
    O.encode at an episode start (h = 0, Dreamer.py:186-187), then
    O.observe_step (WorldModel.py:79-82) and O.actor_act (Agent.py:202-210)
    for 5 further env steps on the same frames and explicit noise (fresh
    tie-guarded q / eps per step).  Latent indices exact; h, z values, action,
    mu, sigma at |d| <= 1e-6 + 1e-4 |ref|; the status word stays 0."""
    from dreamer_amd import hip
    d, P = _dreamer(gpu)
    g = torch.Generator().manual_seed(33)
    n_steps = 6
    frames = [torch.randint(0, 256, (64, 64, 3), generator=g, dtype=torch.uint8).numpy() for _ in range(n_steps)]
    z_o = h_o = a_o = None
    z_f = h_f = a_f = None
    guarded = 0
    with torch.no_grad():
        for k in range(n_steps):
            obs = torch.tensor(frames[k].transpose(2, 0, 1), dtype=torch.float32).view(1, 1, 3, 64, 64) / 255.0 - 0.5
            q = torch.empty(1, R, C).exponential_(generator=g)
            eps = torch.randn(1, 1, A, generator=g)
            with TieGuard() as tg:  # widens near-tie margins in q (in place) without changing the oracle's draw
                if k == 0:
                    h_o = torch.zeros(1, 1, HD)
                    z_o, _ = O.encode(h_o, obs, P, q[0], R, C)
                else:
                    z_o, h_o, _ = O.observe_step(z_o, h_o, a_o, obs, P, q[0], R, C)
            guarded += tg.guarded
            a_o, mu_o, sg_o = O.actor_act(h_o, z_o, P, eps.view(1, 1, A))
            with hip.noise_override(q=q.to(gpu), eps=eps.to(gpu)):
                if k == 0:
                    a_f, mu_f, sg_f, z_f, h_f = d.act_step(frames[k])
                else:
                    a_f, mu_f, sg_f, z_f, h_f = d.act_step(frames[k], z_f, h_f, a_f)
                d.act_check()
            zi_f, zi_o = _idx(z_f), z_o.reshape(-1, C).argmax(-1)
            assert torch.equal(zi_f, zi_o), f"step {k}: {int((zi_f != zi_o).sum())} latent groups differ"
            close(h_f, h_o, 1e-4, 1e-6, f"h' step {k}")
            close(z_f, z_o.reshape(z_f.shape), 0, 1e-6, f"straight-through latent values step {k}")
            close(mu_f, mu_o, 1e-4, 1e-6, f"mu step {k}")
            close(sg_f, sg_o, 1e-4, 1e-6, f"sigma step {k}")
            close(a_f, a_o, 1e-4, 1e-6, f"action step {k}")
    assert int(d._act_bufs["status"].item()) == 0
    print(f"act_step vs oracle: {n_steps} env steps, {guarded} tie-guarded groups")


def test_act_step_matches_unfused(gpu):
    """dr_act_step (one launch per env step, grid barriers inside) == the unfused API
    path it replaces in rollout_policy / evaluate_agent / Run: Encoder.encode
    or WorldModel.observe_step, then Actor.act (Dreamer.py:177-226, 295-322),
    same explicit noise.  Indices exact; h, action, mu, sigma at 1e-5.
    Prints the per-env-step device time of both paths."""
    import time
    from dreamer_amd import hip
    d, P = _dreamer(gpu)
    g = torch.Generator().manual_seed(21)
    frames = [torch.randint(0, 256, (64, 64, 3), generator=g, dtype=torch.uint8).numpy() for _ in range(4)]
    q = torch.empty(1, R, C).exponential_(generator=g).to(gpu)
    eps = torch.randn(1, 1, A, generator=g).to(gpu)
    wm, actor = d.world_model, d.agent.actor
    with torch.no_grad(), hip.noise_override(q=q, eps=eps):
        _, ot = d._obs_tensor(frames[0])
        z_u, _ = wm.encoder.encode(torch.zeros(1, 1, HD, device=gpu), ot)
        h_u = torch.zeros(1, 1, HD, device=gpu)
        a_u, mu_u, sg_u = actor.act(h_u, z_u, deterministic=False)
        a_f, mu_f, sg_f, z_f, h_f = d.act_step(frames[0])
        for k in range(1, 4):
            close(h_f, h_u, 1e-5, 1e-6, f"h step {k - 1}")  # step 0: both exactly 0
            zi_f, zi_u = z_f.reshape(R, C).argmax(-1).cpu(), z_u.reshape(R, C).argmax(-1).cpu()
            assert torch.equal(zi_f, zi_u), f"step {k - 1}: {int((zi_f != zi_u).sum())} latent groups differ"
            close(z_f, z_u, 0, 1e-6, f"straight-through latent values step {k - 1}")
            close(a_f, a_u, 1e-5, 1e-6, "action")
            close(mu_f, mu_u, 1e-5, 1e-6, "mu")
            close(sg_f, sg_u, 1e-5, 1e-6, "sigma")
            _, ot = d._obs_tensor(frames[k])
            z_u, h_u, _ = wm.observe_step(z_u, h_u, a_u, ot)
            a_u, mu_u, sg_u = actor.act(h_u, z_u, deterministic=False)
            a_f, mu_f, sg_f, z_f, h_f = d.act_step(frames[k], z_f, h_f, a_f)
            close(h_f, h_u, 1e-5, 1e-6, f"h step {k}")
    torch.cuda.synchronize()

    def per_step(fn, n=50):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e6

    z, h, a = z_f, h_f, a_f
    with torch.no_grad():
        def unfused():
            _, ot = d._obs_tensor(frames[1])
            z2, h2, _ = wm.observe_step(z, h, a, ot)
            actor.act(h2, z2, deterministic=True)

        t_u = per_step(unfused)
        t_f = per_step(lambda: d.act_step(frames[1], z, h, a, deterministic=True))
    print(f"batch-1 env step (device work + H2D of the frame): unfused {t_u:.1f} us, fused dr_act_step {t_f:.1f} us")
    ts = d._act_bufs["ws"][0:128].view(torch.int64).cpu()  # workgroup 0's stage clock (10 ns ticks)
    marks = [0, 1, 2, 3, 4, 5, 6, 7, 15]
    print("dr_act_step stage ends (us after kernel start):",
          [round(float(ts[m] - ts[0]) / 100.0, 2) for m in marks[1:]])


def test_act_step_failure_paths(gpu, monkeypatch):
    """dr_act_step's failure paths, forced through its test hook
    (include/dreamer_hip.h: DREAMER_ACT_FORCE).  =timeout: every grid barrier
    gives up at once -> the status word is raised, act_check() raises, the
    outputs are NaN, and the next step runs normally.  =nonresident: the
    co-residency check fails -> DR_E_UNSUPPORTED -> Dreamer.act_step runs the
    unfused launches, which match the CPU oracle (O.encode at an episode start,
    O.actor_act; tie-guarded explicit noise, indices exact)."""
    from dreamer_amd import hip
    d, P = _dreamer(gpu)
    g = torch.Generator().manual_seed(44)
    frame = torch.randint(0, 256, (64, 64, 3), generator=g, dtype=torch.uint8).numpy()
    with torch.no_grad():
        monkeypatch.setenv("DREAMER_ACT_FORCE", "timeout")
        a, mu, sg, z, h = d.act_step(frame)
        with pytest.raises(RuntimeError, match="grid barrier timed out"):
            d.act_check()
        for t, name in ((a, "a"), (mu, "mu"), (sg, "sigma"), (z, "z"), (h, "h")):
            assert bool(torch.isnan(t).all()), f"{name} must be NaN after a barrier timeout"
        monkeypatch.delenv("DREAMER_ACT_FORCE")
        a, mu, sg, z, h = d.act_step(frame)
        d.act_check()
        assert all(bool(torch.isfinite(t).all()) for t in (a, mu, sg, z, h))
        assert int(d._act_bufs["status"].item()) == 0
        assert not getattr(d, "_act_unfused", False)
        # co-residency check failing: the unfused path, against the oracle
        monkeypatch.setenv("DREAMER_ACT_FORCE", "nonresident")
        obs = torch.tensor(frame.transpose(2, 0, 1), dtype=torch.float32).view(1, 1, 3, 64, 64) / 255.0 - 0.5
        q = torch.empty(1, R, C).exponential_(generator=g)
        eps = torch.randn(1, 1, A, generator=g)
        with TieGuard():
            h_o = torch.zeros(1, 1, HD)
            z_o, _ = O.encode(h_o, obs, P, q[0], R, C)
        a_o, mu_o, sg_o = O.actor_act(h_o, z_o, P, eps.view(1, 1, A))
        with hip.noise_override(q=q.to(gpu), eps=eps.to(gpu)):
            a_f, mu_f, sg_f, z_f, h_f = d.act_step(frame)
        assert getattr(d, "_act_unfused", False), "DR_E_UNSUPPORTED must switch Dreamer to the unfused path"
        assert torch.equal(_idx(z_f), z_o.reshape(-1, C).argmax(-1))
        close(h_f, h_o, 0, 0, "h' at an episode start")
        close(mu_f, mu_o, 1e-4, 1e-6, "mu (unfused fallback)")
        close(sg_f, sg_o, 1e-4, 1e-6, "sigma (unfused fallback)")
        close(a_f, a_o, 1e-4, 1e-6, "action (unfused fallback)")
