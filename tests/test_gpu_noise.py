"""The Philox noise path that Dreamer.train_Agent() and bench.py actually run
(every parity test elsewhere feeds explicit noise).  Run on the MI355X box:
pytest -m gpu.

What the reference draws: a categorical sample per latent
group, argmax(p_hat / q) with q ~ Exp(1) (torch ``exponential_``;
VariationalAutoEncoder.py:95, DynamicsPredictors.py:36), and the actor's
rsample tanh(mu + eps * sigma), eps ~ N(0, 1) (Agent.py:202-210).  Here the
variates come from Philox4x32-10 keyed by (seed, offset, stream, global row,
element) (dreamer_amd/csrc/common.h).  The tests check, through the C ABI and
through train_Agent() itself:

* the sampler head (k_ln_gemm_sample, Philox mode) draws each class with
  probability p_hat = normalise(0.99 softmax + 0.01 / C): chi-square of class
  counts over identical rows, and a randomised probability-integral transform
  (PIT) over rows with different logits, against U(0, 1) (Kolmogorov-Smirnov);
* the warm-start posterior and the dream's prior draws of a real train_Agent
  epoch pass the same PIT test (p_hat recomputed in float64 from the epoch's
  own hidden states by the CPU oracle);
* the actor's rsample noise eps = (atanh(a) - mu) / sigma of that epoch is
  N(0, 1) (KS, mean, variance), and the draws of different steps, rows,
  action dimensions and streams (warm start / dream sampler / actor) are
  uncorrelated (|r| < 5 / sqrt(n));
* the noise is keyed by the global row: a B = 128 call with row0 = 128 draws
  exactly the second half of the B = 256 call (data-parallel shards and
  batch lanes reproduce the single-GPU draws);
* every Exp(1) variate is > 0 (dr_u01 maps to [2^-24, 1 - 2^-24]: a zero
  variate would make p_hat / q infinite).

The Philox seed is fixed per test (Rng.reseed), so the p-values are
deterministic; the threshold 1e-4 would reject a correct sampler only with
that probability."""
import numpy as np
import pytest
import torch
from scipy import stats

from oracle import dreamer_oracle as O

pytestmark = pytest.mark.gpu
R, C, A, HD = 32, 32, 3, 600
P_MIN = 1e-4


def _phat(logits):
    p = torch.softmax(logits.double().reshape(-1, C), -1)
    pu = 0.99 * p + 0.01 / C
    return pu / pu.sum(-1, keepdim=True)


def _pit(phat, idx, seed):
    """Randomised PIT of categorical draws: F(c - 1) + V p(c), V ~ U(0, 1)."""
    cdf = phat.cumsum(-1)
    idx = idx.reshape(-1, 1).long()
    lo = torch.where(idx > 0, cdf.gather(1, (idx - 1).clamp(min=0)), torch.zeros_like(cdf[:, :1]))
    pc = phat.gather(1, idx)
    v = torch.rand(len(idx), 1, generator=torch.Generator().manual_seed(seed), dtype=torch.float64)
    return (lo + v * pc).flatten().numpy()


def _corr(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    return float(np.corrcoef(a, b)[0, 1]), len(a)


def _bench_dreamer(gpu, B):
    import bench
    from dreamer_amd import hip
    _, d = bench.make_dreamer(bench.CAR_RACER, gpu, B, 64, 15, 64, 1, 1, 0, None, "fp32")
    hip.rng(gpu).reseed(0x1234ABCD)
    return d


def _scan_t1(d, gpu, feat, stream):
    """dr_observe_scan with T = 1 and no initial state: the encode step's
    sampler head (k_ln_gemm_sample) on latent_mapper(feat, h = 0) in Philox
    mode.  Returns (logits, one-hot z)."""
    from dreamer_amd import _lib as L
    from dreamer_amd import hip
    B = feat.shape[0]
    dd = d.world_model.dims(d.agent)
    z = torch.empty(B, R * C, device=gpu)
    h = torch.empty(B, HD, device=gpu)
    lg = torch.empty(B, R * C, device=gpu)
    ws = torch.empty(L.query("dr_observe_workspace_bytes", dd, B), dtype=torch.uint8, device=gpu)
    nz = L.dr_noise(None, None, hip.rng(gpu).state.data_ptr(), 0, stream)
    L.call("dr_observe_scan", dd, d.world_model.packed(), B, 1, L.ptr(feat), None, 0, 0, None, None, nz,
           L.ptr(z), L.ptr(h), L.ptr(lg), L.ptr(ws), ws.numel(), hip.stream())
    torch.cuda.synchronize()
    return lg.cpu(), z.cpu()


def test_sampler_head_class_frequencies(gpu):
    """Identical rows: per-group class counts of 16384 Philox draws against
    n p_hat (chi-square, cells with expected < 5 pooled), and the PIT of
    8192 rows with different logits (KS)."""
    d = _bench_dreamer(gpu, 64)
    with torch.no_grad():
        d.world_model.encoder.latent_mapper[3].weight.mul_(6.0)  # peaked p_hat: a wide range of probabilities
    n = 16384
    g = torch.Generator().manual_seed(5)
    row = torch.randn(1, 200, generator=g)
    lg, z = _scan_t1(d, gpu, row.expand(n, 200).contiguous().to(gpu), 77 << 17)
    assert torch.equal(lg[0:1].expand(n, -1), lg), "identical rows must give identical logits"
    ph = _phat(lg[0])  # [R][C]
    counts = z.reshape(n, R, C).argmax(-1)
    chi, dof = 0.0, 0
    for r in range(R):
        obs = torch.bincount(counts[:, r], minlength=C).double()
        exp = ph[r] * n
        small = exp < 5
        o = torch.cat([obs[~small], obs[small].sum().view(1)]) if small.any() else obs
        e = torch.cat([exp[~small], exp[small].sum().view(1)]) if small.any() else exp
        chi += float(((o - e) ** 2 / e).sum())
        dof += len(o) - 1
    p_chi = float(stats.chi2.sf(chi, dof))
    assert float(ph.max()) > 0.3 and float(ph.min()) < 1e-3, "the check needs a wide range of probabilities"
    # rows with different logits: randomised PIT against U(0, 1)
    feat = torch.randn(8192, 200, generator=g).to(gpu)
    lg2, z2 = _scan_t1(d, gpu, feat, 78 << 17)
    u = _pit(_phat(lg2), z2.reshape(-1, C).argmax(-1), seed=11)
    p_ks = float(stats.kstest(u, "uniform").pvalue)
    print(f"sampler head: chi2 {chi:.1f} on {dof} dof (p = {p_chi:.3g}); PIT KS p = {p_ks:.3g} over {len(u)} draws")
    assert p_chi > P_MIN, (chi, dof)
    assert p_ks > P_MIN


def test_sampler_row_keyed(gpu):
    """Noise keyed by the global row: M = 128 rows with row0 = 128 draw
    exactly the second half of the M = 256 call (dr_categorical_sample and the
    scan's sampler head)."""
    from dreamer_amd import _lib as L
    from dreamer_amd import hip
    d = _bench_dreamer(gpu, 64)
    st = hip.rng(gpu).state.data_ptr()
    lg = torch.randn(256, R * C, device=gpu) * 3
    outs = []
    for M, row0, off in ((256, 0, 0), (128, 128, 128)):
        z = torch.empty(M, R * C, device=gpu)
        idx = torch.empty(M, R, dtype=torch.int32, device=gpu)
        L.call("dr_categorical_sample", M, R, C, L.ptr(lg[off:]), L.dr_noise(None, None, st, row0, 99 << 17),
               L.ptr(z), L.ptr(idx), None, hip.stream())
        outs.append(idx)
    torch.cuda.synchronize()
    assert torch.equal(outs[0][128:], outs[1])
    assert not torch.equal(outs[0][:128], outs[1])


@pytest.fixture(scope="module")
def philox_epoch(gpu):
    """One Dreamer.train_Agent() epoch (Philox noise, the benchmarked path) at
    B = 1024, S = 64, H = 15; returns the engine's epoch outputs on the CPU."""
    B = 1024
    d = _bench_dreamer(gpu, B)
    d.train_Agent()
    torch.cuda.synchronize()
    e = d._engine
    P = {k: v.detach().cpu() for k, v in d.world_model.state_dict().items()}
    P = {"world_model." + k: v for k, v in P.items()}
    out = dict(B=B, T=e.T, z0=e.z0.cpu(), h0=e.h0.cpu(), feat_last=e.feat.view(e.T, B, -1)[-1].cpu(),
               lat=e.latents.cpu(), hid=e.hiddens.cpu(), act=e.actions.cpu(), mu=e.mus.cpu(), sig=e.sigmas.cpu(),
               P=P)
    return out


def _eps(ep):
    a = ep["act"].double()
    keep = a.abs() < 0.999  # atanh stays accurate (drops |mu + eps sigma| > 3.8: ~1e-7 of draws)
    x = torch.atanh(a.clamp(-0.999999, 0.999999))
    eps = (x - ep["mu"].double()) / ep["sig"].double()
    return eps, keep


def test_actor_rsample_noise_is_standard_normal(philox_epoch):
    """eps = (atanh(a) - mu) / sigma over the epoch's B x H x A actions."""
    eps, keep = _eps(philox_epoch)
    e = eps[keep].numpy()
    n = len(e)
    assert n > 0.999 * eps.numel()
    p_ks = float(stats.kstest(e, "norm").pvalue)
    m, v = float(e.mean()), float(e.var())
    print(f"actor eps: n {n}, mean {m:.4f}, var {v:.4f}, KS p {p_ks:.3g}")
    assert abs(m) < 5 / np.sqrt(n)
    assert abs(v - 1) < 5 * np.sqrt(2 / n)
    assert p_ks > P_MIN
    # independence: consecutive steps, neighbouring rows, action dimensions
    E = eps.numpy()
    for name, (x, y) in {"step t / t+1": (E[:, :-1], E[:, 1:]), "row b / b+1": (E[:-1], E[1:]),
                         "dim 0 / 1": (E[..., 0], E[..., 1]), "dim 1 / 2": (E[..., 1], E[..., 2])}.items():
        r, k = _corr(x, y)
        print(f"  corr {name}: {r:+.4f} (n {k})")
        assert abs(r) < 5 / np.sqrt(k), (name, r)


def _dream_pit(ep):
    """PIT of the dream's prior draws z_{t+1} given h_{t+1} (float64 oracle
    prior logits) -> [B][H][R]."""
    B, H = ep["B"], ep["act"].shape[1]
    P = {k: v.double() for k, v in ep["P"].items()}
    h = ep["hid"][:, 1:].double()
    lg = O.prior_logits(h, P, R, C)  # [B][H][R][C]
    idx = ep["lat"][:, 1:].reshape(-1, C).argmax(-1)
    return _pit(_phat(lg), idx, seed=21).reshape(B, H, R)


def _warm_pit(ep):
    """PIT of the warm start's last posterior draw z0 given (features, h0)."""
    P = {k: v.double() for k, v in ep["P"].items()}
    wm = "world_model.encoder.latent_mapper."
    W0 = P[wm + "0.weight"]
    F = W0.shape[1] - HD
    pre = ep["feat_last"].double() + ep["h0"].double() @ W0[:, F:].T
    y = torch.nn.functional.silu(torch.nn.functional.layer_norm(pre, (pre.shape[-1],), P[wm + "1.weight"],
                                                                P[wm + "1.bias"], 1e-5))
    lg = torch.nn.functional.linear(y, P[wm + "3.weight"], P[wm + "3.bias"])
    idx = ep["z0"].reshape(-1, C).argmax(-1)
    return _pit(_phat(lg), idx, seed=31).reshape(ep["B"], R)


def test_epoch_categorical_draws_follow_p_hat(philox_epoch):
    """The warm start's and the dream's categorical draws of the train_Agent
    epoch against p_hat from the epoch's own states (PIT, KS), and the three
    Philox streams (warm sampler, dream sampler, actor) uncorrelated."""
    ud = _dream_pit(philox_epoch)
    uw = _warm_pit(philox_epoch)
    for name, u in (("dream prior", ud), ("warm posterior", uw)):
        p = float(stats.kstest(u.ravel(), "uniform").pvalue)
        print(f"{name}: {u.size} draws, PIT KS p = {p:.3g}")
        assert p > P_MIN, name
    checks = {"dream step t / t+1": (ud[:, :-1], ud[:, 1:]), "dream group r / r+1": (ud[..., :-1], ud[..., 1:]),
              "dream row b / b+1": (ud[:-1], ud[1:]), "warm z0 / dream z1": (uw, ud[:, 0])}
    eps, _ = _eps(philox_epoch)
    checks["dream z_{t+1} / actor eps_t"] = (ud[:, :, 0], eps[..., 0].numpy())
    for name, (x, y) in checks.items():
        r, k = _corr(x, y)
        print(f"  corr {name}: {r:+.4f} (n {k})")
        assert abs(r) < 5 / np.sqrt(k), (name, r)
