"""HIP path (libdreamer_hip via dreamer_amd) vs the CPU oracle / the
reference's golden outputs.  Run on the MI355X box: pytest -m gpu.

Tolerances (fp32 parity mode): GEMMs differ from the CPU only in summation
order, so single blocks match to ~1e-6 relative; recurrences (S/2 posterior
steps, H imagination steps, BPTT) are checked at rtol 2e-4 / atol 2e-5.
Categorical indices must match exactly except at near-ties, where the oracle's
top-2 p_hat/q scores are within 1e-4 relative (reported and bounded)."""
import numpy as np
import pytest
import torch

from conftest import load_fixture
from gpu_helpers import build, close, cpu, flip_report
from oracle import dreamer_oracle as O

pytestmark = pytest.mark.gpu
WHICH = ["small", "full"]


def _t(a, dev=None):
    t = torch.from_numpy(np.asarray(a).copy())
    return t if dev is None else t.to(dev)


@pytest.mark.parametrize("which", WHICH)
def test_blocks_teacher_forced(which, gpu):
    fx = load_fixture(which + "_blocks")
    d, P = build(which, gpu)
    wm, ag = d.world_model, d.agent
    h, z, a, obs = (_t(fx[k], gpu) for k in ("h", "z", "a", "obs"))
    R, C = z.shape[-2:]
    with torch.no_grad():
        close(wm.sequence_model(z, h, a), _t(fx["gru"]), 1e-4, 1e-5, "GRU cell")
        close(wm.dynamics_predictor(h), _t(fx["prior_logits"]), 1e-4, 1e-5, "prior logits")
        close(wm.reward_predictor(h, z), _t(fx["reward_logits"]), 1e-4, 1e-5, "reward logits")
        close(wm.reward_predictor.predict(h, z), _t(fx["reward"]), 1e-4, 1e-5, "reward value")
        p, lg = wm.continue_predictor(h, z)
        close(lg, _t(fx["cont_logit"]), 1e-4, 1e-5, "continue logit")
        close(p, _t(fx["cont_prob"]), 1e-4, 1e-6, "continue prob")
        act, mu, sg = ag.actor.act(h, z, deterministic=True)
        close(mu, _t(fx["actor_mu"]), 1e-4, 1e-5, "actor mu")
        close(sg, _t(fx["actor_sigma"]), 1e-4, 1e-6, "actor sigma")
        close(act, torch.tanh(_t(fx["actor_mu"])), 1e-4, 1e-6, "actor deterministic action")
        close(ag.critic(h, z), _t(fx["critic_logits"]), 1e-4, 1e-5, "critic logits")
        close(ag.critic.value(h, z), _t(fx["critic_value"]), 1e-4, 1e-5, "critic value")
        close(wm.encoder(h, obs), _t(fx["enc_logits"]), 1e-4, 1e-5, "encoder logits")


@pytest.mark.parametrize("which", WHICH)
def test_categorical_sampler_exact(which, gpu):
    from dreamer_amd import hip
    from dreamer_amd.networks import sample_latent
    fx = load_fixture(which + "_blocks")
    for lg_key, q_key, z_key in (("enc_logits", "q_enc", "enc_z"), ("prior_logits", "q_prior", "prior_z")):
        lg = _t(fx[lg_key])
        R, C = fx[z_key].shape[-2:]
        lg = lg.reshape(*fx[z_key].shape)
        q = _t(fx[q_key], gpu)
        z = sample_latent(lg.to(gpu), R, C, noise=hip.explicit_noise(q=q, device=gpu))
        assert torch.equal(cpu(z).argmax(-1), _t(fx[z_key]).argmax(-1)), lg_key
        # straight-through value: exactly 0 off the sample, (1+p)-p on it
        zz = cpu(z)
        assert torch.equal((zz != 0).float(), _t(fx[z_key]).ne(0).float())
        close(zz, _t(fx[z_key]), 0, 1.2e-7, "STE value")


def _engine_case(which, gpu):
    from dreamer_amd.engine import ImaginationEngine
    fx = load_fixture(which + "_epoch")
    d, P = build(which, gpu, fx)
    buf = d.buffer
    buf.load_arrays(fx["buf_frames"], fx["buf_actions"], fx["buf_rewards"], fx["buf_continues"])
    buf.size, buf.next_idx = int(fx["buf_size"]), int(fx["buf_next_idx"])
    eng = ImaginationEngine(d, use_graph=False)
    eng.starts.copy_(_t(fx["starts"]))
    return fx, d, P, eng


@pytest.mark.parametrize("which", WHICH)
def test_replay_gather_exact(which, gpu):
    fx = load_fixture(which + "_epoch")
    d, _ = build(which, gpu, fx)
    buf = d.buffer
    buf.load_arrays(fx["buf_frames"], fx["buf_actions"], fx["buf_rewards"], fx["buf_continues"])
    buf.size, buf.next_idx = int(fx["buf_size"]), int(fx["buf_next_idx"])
    np.random.seed(int(fx["np_seed"]))
    obs, act, rew, cont, S = buf.sample_sequences(int(fx["cfg_B"]))
    idx = (fx["starts"][:, None] + np.arange(S)[None, :]) % int(fx["buf_capacity"])
    assert torch.equal(cpu(obs), torch.tensor(fx["buf_frames"][idx], dtype=torch.float32))
    assert torch.equal(cpu(act), torch.tensor(fx["buf_actions"][idx]))
    assert torch.equal(cpu(rew), torch.tensor(fx["buf_rewards"][idx]))
    assert torch.equal(cpu(cont), torch.tensor(fx["buf_continues"][idx]))


@pytest.mark.parametrize("which", WHICH)
def test_warm_start_from_ring(which, gpu):
    fx, d, P, eng = _engine_case(which, gpu)
    d.buffer.gather_actions(eng.starts, eng.act_win)
    eng.encode_and_warm(d.buffer.frames_struct(eng.starts), noise_q=_t(fx["q_warm"], gpu))
    torch.cuda.synchronize()
    C = int(fx["cfg_cols"])
    za, zb = cpu(eng.z0).reshape(-1, C).argmax(-1), _t(fx["z0"]).reshape(-1, C).argmax(-1)
    assert torch.equal(za, zb), f"warm-start latent flips: {int((za != zb).sum())}"
    close(eng.h0, _t(fx["h0"]).reshape(eng.h0.shape), 2e-4, 2e-5, "warm-start h0")
    close(eng.z0, _t(fx["z0"]).reshape(eng.z0.shape), 0, 1.2e-7, "warm-start z0")


@pytest.mark.parametrize("which", WHICH)
def test_imagine_unroll(which, gpu):
    fx, d, P, eng = _engine_case(which, gpu)
    eng.z0.copy_(_t(fx["z0"]).reshape(eng.z0.shape))
    eng.h0.copy_(_t(fx["h0"]).reshape(eng.h0.shape))
    eng.imagine(eps=_t(fx["eps"], gpu), q=_t(fx["q"], gpu))
    torch.cuda.synchronize()
    C = int(fx["cfg_cols"])
    la, lb = cpu(eng.latents).reshape(-1, C).argmax(-1), _t(fx["latents"]).reshape(-1, C).argmax(-1)
    assert torch.equal(la, lb), f"imagined latent flips: {int((la != lb).sum())}"
    shp = lambda k, ref: _t(fx[k]).reshape(ref.shape)
    close(eng.hiddens, shp("hiddens", eng.hiddens), 2e-4, 2e-5, "hiddens")
    close(eng.actions, shp("actions", eng.actions), 2e-4, 2e-5, "actions")
    close(eng.mus, shp("mus", eng.mus), 2e-4, 2e-5, "mus")
    close(eng.sigmas, shp("sigmas", eng.sigmas), 2e-4, 2e-5, "sigmas")
    close(eng.rewards, shp("rewards", eng.rewards), 2e-4, 2e-5, "rewards")
    close(eng.continues, shp("continues", eng.continues), 2e-4, 2e-5, "continues")


@pytest.mark.parametrize("which", WHICH)
def test_actor_critic_update(which, gpu):
    """returns, update_S, losses, BPTT actor grads, critic grads, AdamW, EMA."""
    fx, d, P, eng = _engine_case(which, gpu)
    eng.z0.copy_(_t(fx["z0"]).reshape(eng.z0.shape))
    eng.h0.copy_(_t(fx["h0"]).reshape(eng.h0.shape))
    eng.imagine(eps=_t(fx["eps"], gpu), q=_t(fx["q"], gpu))
    eng.returns()
    eng.losses_and_grads()
    ag = d.agent
    torch.cuda.synchronize()
    close(eng.R, _t(fx["R"]).reshape(eng.R.shape), 2e-4, 2e-5, "lambda returns")
    close(ag.loss_buffer[0:1], _t(fx["loss_actor"]).reshape(1), 2e-4, 2e-6, "actor loss")
    close(ag.loss_buffer[1:2], _t(fx["loss_critic"]).reshape(1), 2e-4, 2e-6, "critic loss")
    assert abs(float(ag.S_dev) - float(fx["S_after"])) < 1e-5
    eng.optimise()  # clip_grad_norm_ scales the grads in place, as the reference's do
    torch.cuda.synchronize()
    for f, keys in ((ag.fa, O.ACTOR_KEYS), (ag.fc, O.CRITIC_KEYS)):
        for k in keys:
            name = k.split(".", 1)[1]
            o = f.offsets[name]
            ref = _t(fx["gradc_agent." + k])
            got = f.grad[o:o + ref.numel()].view(ref.shape)
            scale = float(ref.abs().max()) + 1e-12
            close(got, ref, 2e-3, 2e-4 * scale, "grad " + k)
    sd = d.state_dict()
    for k in O.ACTOR_KEYS + O.CRITIC_KEYS:
        close(sd["agent." + k], _t(fx["post_agent." + k]), 0, 2 * 1e-4 + 1e-7, "post-step " + k)
        if k.startswith("critic"):
            tk = "agent.target_" + k
            close(sd[tk], _t(fx["post_" + tk]), 0, 2 * 0.02 * 1e-4 + 1e-7, "target " + k)


@pytest.mark.parametrize("which", WHICH)
def test_api_dream_and_train_step(which, gpu):
    """Dreamer.dream_episodes (autograd node over the HIP unroll) + Agent.train_step."""
    fx = load_fixture(which + "_epoch")
    d, P = build(which, gpu, fx)
    z0, h0 = _t(fx["z0"], gpu), _t(fx["h0"], gpu)
    out = d._imagine_raw(z0, h0, eps=_t(fx["eps"], gpu), q=_t(fx["q"], gpu))[0]
    close(out[1], _t(fx["hiddens"]), 2e-4, 2e-5, "api hiddens")
    from dreamer_amd.dreamer import _DreamFn
    from dreamer_amd import hip
    orig = d._imagine_raw
    d._imagine_raw = lambda z, h: orig(z, h, eps=_t(fx["eps"], gpu), q=_t(fx["q"], gpu))
    outs = d.dream_episodes(z0, h0)
    d._imagine_raw = orig
    lat, hid, act, rew, cont, mu, sg = outs
    assert mu.requires_grad and mu.grad_fn is not None
    la, lc = d.agent.train_step(lat, hid, rew, cont, act, mu, sg)
    close(la.reshape(1), _t(fx["loss_actor"]).reshape(1), 2e-4, 2e-6, "api actor loss")
    close(lc.reshape(1), _t(fx["loss_critic"]).reshape(1), 2e-4, 2e-6, "api critic loss")
    sd = d.state_dict()
    for k in O.ACTOR_KEYS + O.CRITIC_KEYS:
        close(sd["agent." + k], _t(fx["post_agent." + k]), 0, 2 * 1e-4 + 1e-7, "api post-step " + k)


def test_graph_replay_matches_eager(gpu):
    """The captured HIP graph of a whole epoch == the eager launch sequence."""
    from dreamer_amd.engine import ImaginationEngine
    from formula import replay_data
    fx = load_fixture("small_epoch")
    res = []
    for use_graph in (False, True):
        d, P = build("small", gpu, fx, B=8, S=8, H=5)
        fr, ac, rw, ct = replay_data(64, (32, 32), 3, seed=3)
        d.buffer.load_arrays(fr, ac, O.symlog(torch.tensor(rw)).numpy(), ct)
        eng = ImaginationEngine(d, use_graph=use_graph)
        eng.rng.reseed(1234)
        np.random.seed(7)
        for _ in range(3):
            la, lc = eng.run(d.buffer.sample_start_indices(8))
        torch.cuda.synchronize()
        res.append((cpu(la), cpu(lc), cpu(d.agent.fa.flat), cpu(d.agent.fc.flat), cpu(d.agent.ft.flat)))
    for a, b in zip(*res):
        assert torch.isfinite(a).all()
        assert torch.equal(a, b)


@pytest.mark.parametrize("which,sched", [("small", None), ("full", None), ("full", "1.0:0:1"), ("full", "0.875:0:1"),
                                         ("full", "0.875:-1:0")])
def test_pipelined_epochs_match_sequential(which, sched, gpu, monkeypatch):
    """run_many (warm start of epoch e+1 on a second stream beside epoch e's
    actor-critic chain) == the same epochs run one after another, bit for
    bit: losses of every epoch, actor / critic / target parameters, S.
    sched "f:p:w": the warm stream restricted to a share f of the CUs
    (dr_stream_create_cumask; 1.0 = an unfenced plain stream), the chain on a
    stream of priority p, w = DREAMER_WARM0_MAIN (1: a call's first warm start
    on the chain's stream; 0: every warm start on the warm stream).  The
    default (None) is "0.875:-1:1".  The pipelined warm starts run the launch
    form (dr_dims.launch_form: their graphs replay on a CU-masked stream), so
    the sequential epochs here do too (DREAMER_PERSISTENT=0); the persistent
    scan is pinned against the oracle by test_gpu_baseline.py."""
    from dreamer_amd.engine import ImaginationEngine
    from formula import replay_data
    monkeypatch.setenv("DREAMER_PERSISTENT", "0")
    if sched:
        frac, prio, w0 = sched.split(":")
        monkeypatch.setenv("DREAMER_WARM_CUS", frac)
        monkeypatch.setenv("DREAMER_CHAIN_PRIORITY", prio)
        monkeypatch.setenv("DREAMER_WARM0_MAIN", w0)
    fx = load_fixture("small_epoch")
    hw = (32, 32) if which == "small" else (64, 64)
    B, S, H, K = (8, 8, 5, 5) if which == "small" else (16, 16, 6, 4)
    res = []
    for pipe in (False, True):
        d, P = build(which, gpu, fx if which == "small" else None, B=B, S=S, H=H)
        fr, ac, rw, ct = replay_data(64, hw, 3, seed=3)
        d.buffer.load_arrays(fr, ac, O.symlog(torch.tensor(rw)).numpy(), ct)
        eng = ImaginationEngine(d)
        eng.rng.reseed(4321)
        np.random.seed(5)
        starts = [d.buffer.sample_start_indices(B) for _ in range(K)]
        if pipe:
            losses = eng.run_many(starts).cpu()
        else:
            ls = []
            for st in starts:
                la, lc = eng.run(st)
                ls.append(torch.cat([la, lc]).clone())
            losses = torch.stack(ls).cpu()
        torch.cuda.synchronize()
        res.append((losses, cpu(d.agent.fa.flat), cpu(d.agent.fc.flat), cpu(d.agent.ft.flat), cpu(d.agent.S_dev),
                    cpu(eng.rng.state)))
    for a, b in zip(*res):
        assert torch.isfinite(a.float()).all()
        assert torch.equal(a, b)


@pytest.mark.parametrize("n", [3840, 16384, 16385, 30720, 262144])
def test_update_S_quantile_exact(n, gpu):
    """Agent.update_S (Agent.py:78-88) on n returns: bitonic LDS sort up to
    16384 values, exact radix select above (8 ranks x 256 rows x H 15 =
    30720 under DP).  torch.quantile's two order statistics and its linear
    interpolation are reproduced bit-exactly; ties and signed zeros are
    included; a NaN leaves S unchanged."""
    from dreamer_amd import _lib as L
    g = torch.Generator().manual_seed(n)
    R = (torch.randn(n, generator=g) * 7.0).round(decimals=2)  # many ties
    R[: n // 50] = 0.0
    R[n // 50: n // 25] = -0.0
    for S0 in (1.0, 3.5):
        Sd = torch.tensor([S0], device=gpu)
        norm = torch.zeros(1, device=gpu)
        Rd = R.to(gpu)
        L.call("dr_update_S", n, L.ptr(Rd), L.ptr(Sd), L.ptr(norm), None, 0, 0)
        torch.cuda.synchronize()
        ref = O.update_S(torch.tensor(S0), R)
        assert float(Sd) == float(ref), (n, float(Sd), float(ref))
        assert float(norm) == max(float(ref), 1.0)
    Rn = R.clone()
    Rn[n // 3] = float("nan")
    Sd = torch.tensor([2.0], device=gpu)
    L.call("dr_update_S", n, L.ptr(Rn.to(gpu)), L.ptr(Sd), None, None, 0, 0)
    torch.cuda.synchronize()
    assert float(Sd) == 2.0


def test_pipelined_engine_dropped_then_new_capture(gpu):
    """Regression test of the round-5 r05a abort: a
    segfault in the first pipelined test after f76c296 made every engine
    destroy its CU-masked warm stream when it was collected.  torch's caching
    allocator still held blocks allocated on that stream (the window starts
    and Philox copies run_many stages on it), and the next allocation that
    reused them touched the destroyed stream.  Since b2e3f22 one masked stream
    per (device, mask) lives for the process (engine._CU_STREAMS).  Here: an
    engine with pipelined graphs is built, run and dropped, the collector runs
    and the cache is emptied; a second engine then captures and runs both its
    pipelined and its sequential graphs, finite, on the same masked stream."""
    import gc
    from dreamer_amd import engine as E
    from formula import replay_data
    fx = load_fixture("small_epoch")
    B, S, H, K = 8, 8, 5, 3
    handles = []
    for rep in range(2):
        d, P = build("small", gpu, fx, B=B, S=S, H=H)
        fr, ac, rw, ct = replay_data(64, (32, 32), 3, seed=3)
        d.buffer.load_arrays(fr, ac, O.symlog(torch.tensor(rw)).numpy(), ct)
        eng = E.ImaginationEngine(d)
        np.random.seed(5 + rep)
        losses = eng.run_many([d.buffer.sample_start_indices(B) for _ in range(K)])
        la, lc = eng.run(d.buffer.sample_start_indices(B))
        torch.cuda.synchronize()
        assert torch.isfinite(losses).all() and bool(torch.isfinite(la).all()) and bool(torch.isfinite(lc).all())
        handles.append(eng._pipe["stream"].cuda_stream)
        eng.check_faults()
        del d, P, eng, losses, la, lc
        gc.collect()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        # new allocations reuse the blocks the dropped engine used on the masked stream
        junk = [torch.empty(1 << 20, device=gpu) for _ in range(8)]
        del junk
    assert handles[0] == handles[1], "the masked warm stream must be shared for the process"
    assert handles[0] in [h.value for h in E._CU_STREAMS.values()]
