"""bf16 perf mode (config key precision="bf16"; SURVEY.md section 5, BASELINE
configs[1]): the encoder's four convolutions and the latent_mapper.0 feature
projection (VariationalAutoEncoder.py:57-75) run on the bf16 MFMA with f32
accumulation.

Two checks, both through the C ABI (dr_encoder_features):
  * kernel exactness: against a torch emulation that rounds to bf16 at the
    same points (normalised frame, weights, every activation) and accumulates
    in f32 -- normwise relative error <= 2e-3 (differences are f32 summation
    order and the odd 1-ulp bf16 rounding flip they cause downstream);
  * precision cost: against the fp32 parity path -- normwise relative error
    <= 2e-2 (the stated bf16 tolerance of the features).
A full train_Agent epoch in bf16 mode at BASELINE configs[1] shape must give
finite losses, and its warm-start latents are compared with the fp32 mode's:
the flip fraction is reported (bf16 does not promise identical indices).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _bf(x):
    return x.to(torch.bfloat16).float()


def _emulate(frames_u8, P, pre=""):
    """bf16-rounded reference of Encoder.forward's conv stack + feature columns."""
    x = _bf(frames_u8.float() / 255.0 - 0.5)
    for i in range(4):
        w, b = P[f"{pre}feature_extractor.{2 * i}.weight"], P[f"{pre}feature_extractor.{2 * i}.bias"]
        x = F.conv2d(x, _bf(w), b.float(), stride=2, padding=1)
        x = _bf(F.silu(x))
    flat = x.flatten(1)
    W = P[f"{pre}latent_mapper.0.weight"][:, :flat.shape[1]]
    return flat @ _bf(W).t() + P[f"{pre}latent_mapper.0.bias"]


def _features(enc, d, frames_u8, dev):
    """dr_encoder_features over a (n, 3, H, W) u8 batch via a one-slot-per-frame ring."""
    from dreamer_amd import _lib as L
    from dreamer_amd import hip
    n = frames_u8.shape[0]
    ring = frames_u8.contiguous().to(dev)
    starts = torch.arange(n, dtype=torch.int64, device=dev)
    fr = L.dr_frames(L.ptr(ring), n, L.ptr(starts), None, 0, 0, 1, 0)
    feat = torch.empty(n, d.enc_hidden, device=dev)
    ws = torch.empty(L.query("dr_encoder_workspace_bytes", d, n), dtype=torch.uint8, device=dev)
    L.call("dr_encoder_features", d, enc, fr, n, 1, L.ptr(feat), L.ptr(ws), ws.numel(), hip.stream())
    torch.cuda.synchronize()
    return feat.cpu()


@pytest.mark.parametrize("res", [64, 128])
def test_encoder_bf16_matches_emulation(gpu, res):
    from dreamer_amd import Dreamer
    from formula import FULL
    cfg = dict(FULL)
    cfg.update(observation_dims=[res, res], precision="bf16")
    torch.manual_seed(0)
    d = Dreamer(cfg, gpu)
    wm = d.world_model
    g = torch.Generator().manual_seed(1)
    n = 40 if res == 64 else 12
    frames = torch.randint(0, 256, (n, 3, res, res), generator=g, dtype=torch.uint8)
    dims = wm.dims(d.agent)
    assert dims.precision == 1
    got = _features(wm.packed(), dims, frames, gpu)
    P = {k: v.detach().cpu() for k, v in wm.encoder.state_dict().items()}
    ref = _emulate(frames, P)
    err = float((got - ref).norm() / ref.norm())
    assert err <= 2e-3, f"bf16 encoder vs bf16 emulation: normwise rel err {err:.3g}"
    # the fp32 parity path on the same frames: the precision cost of bf16
    dims.precision = 0
    f32 = _features(wm.packed(), dims, frames, gpu)
    err32 = float((got - f32).norm() / f32.norm())
    print(f"res {res}: bf16 vs emulation {err:.2e}, bf16 vs fp32 {err32:.2e}")
    assert err32 <= 2e-2, f"bf16 encoder vs fp32: normwise rel err {err32:.3g}"


def test_train_agent_bf16_epoch(gpu):
    """One train_Agent epoch per precision at configs[1] (B=64 S=64 H=15) from
    the same replay, weights and noise: bf16 losses finite and near fp32."""
    from dreamer_amd import Dreamer
    from formula import FULL, replay_data
    out = {}
    for prec in ("fp32", "bf16"):
        cfg = dict(FULL)
        cfg.update(batch_size=64, sequence_length=64, horizon=15, buffer_size=1024, precision=prec)
        torch.manual_seed(0)
        d = Dreamer(cfg, gpu)
        fr, ac, rw, ct = replay_data(1024, (64, 64), 3, seed=3)
        d.buffer.load_arrays(fr, ac, rw, ct)
        d.engine.rng.reseed(77)
        np.random.seed(5)
        la, lc = d.train_Agent()
        torch.cuda.synchronize()
        out[prec] = (float(la), float(lc), d.engine.latents[:, 0].cpu().clone())
    (a32, c32, z32), (a16, c16, z16) = out["fp32"], out["bf16"]
    assert np.isfinite(a16) and np.isfinite(c16)
    flips = float((z32.reshape(-1, 32).argmax(-1) != z16.reshape(-1, 32).argmax(-1)).float().mean())
    print(f"fp32 losses ({a32:.5f}, {c32:.5f}), bf16 ({a16:.5f}, {c16:.5f}); warm-start index flips {flips:.3%}")
    assert abs(c16 - c32) <= 0.05 * abs(c32)


@pytest.mark.parametrize("res", [64, 128])
def test_encoder_fp32_from_frames_matches_torch(gpu, res):
    """fp32 parity mode: dr_encoder_features (first conv straight from the u8
    frames, k_conv1_frames; then the NHWC implicit GEMMs) against the plain
    torch fp32 conv stack on the same frames: normwise relative error <= 1e-5
    (f32 summation order only)."""
    from dreamer_amd import Dreamer
    from formula import FULL
    cfg = dict(FULL)
    cfg.update(observation_dims=[res, res])
    torch.manual_seed(0)
    d = Dreamer(cfg, gpu)
    wm = d.world_model
    g = torch.Generator().manual_seed(2)
    n = 40 if res == 64 else 12
    frames = torch.randint(0, 256, (n, 3, res, res), generator=g, dtype=torch.uint8)
    dims = wm.dims(d.agent)
    got = _features(wm.packed(), dims, frames, gpu)
    P = {k: v.detach().cpu() for k, v in wm.encoder.state_dict().items()}
    x = frames.float() / 255.0 - 0.5
    for i in range(4):
        x = F.silu(F.conv2d(x, P[f"feature_extractor.{2 * i}.weight"], P[f"feature_extractor.{2 * i}.bias"],
                            stride=2, padding=1))
    flat = x.flatten(1)
    ref = flat @ P["latent_mapper.0.weight"][:, :flat.shape[1]].t() + P["latent_mapper.0.bias"]
    err = float((got - ref).norm() / ref.norm())
    print(f"res {res}: fp32 encoder vs torch {err:.2e}")
    assert err <= 1e-5


def test_encoder_fp32_split_is_f32_accurate(gpu):
    """The fp32 encoder's conv2..4 run on the bf16 MFMA with a 3-term split
    (conv_split.hip): its error against a float64 conv stack must be of the
    order of torch's own float32 stack (<= 4x its normwise error), i.e. f32
    accuracy, not bf16 (which sits ~1e-3 away, test above)."""
    from dreamer_amd import Dreamer
    from formula import FULL
    torch.manual_seed(0)
    d = Dreamer(dict(FULL), gpu)
    wm = d.world_model
    g = torch.Generator().manual_seed(5)
    frames = torch.randint(0, 256, (64, 3, 64, 64), generator=g, dtype=torch.uint8)
    got = _features(wm.packed(), wm.dims(d.agent), frames, gpu).double()
    P = {k: v.detach().cpu() for k, v in wm.encoder.state_dict().items()}

    def stack(dt):
        x = (frames.float() / 255.0 - 0.5).to(dt)
        for i in range(4):
            x = F.silu(F.conv2d(x, P[f"feature_extractor.{2 * i}.weight"].to(dt),
                                P[f"feature_extractor.{2 * i}.bias"].to(dt), stride=2, padding=1))
        flat = x.flatten(1)
        return flat @ P["latent_mapper.0.weight"][:, :flat.shape[1]].to(dt).t() + P["latent_mapper.0.bias"].to(dt)

    ref64 = stack(torch.float64)
    err = float((got - ref64).norm() / ref64.norm())
    err32 = float((stack(torch.float32).double() - ref64).norm() / ref64.norm())
    print(f"fp32 encoder vs float64: {err:.2e}; torch float32 vs float64: {err32:.2e}")
    assert err <= 4 * err32 + 1e-7, (err, err32)


def test_critic_fwd_bf16_chain_gemm(gpu):
    """bf16 mode's chain GEMMs (k_gemm_tile_b16: NT tile-route products with
    operands rounded to bf16, f32 accumulation) through dr_critic_fwd at the
    headline row count M = 256 (ValueNetwork, ActorCriticNetworks.py critic
    MLP): first layer K = hidden + R*C takes the bf16 tile.  Against the fp32
    mode on the same inputs: normwise relative error of the bucket logits in
    (1e-6, 2e-2] -- non-zero proves the bf16 kernel ran, the bound is the
    stated bf16 tolerance."""
    from dreamer_amd import Dreamer
    from dreamer_amd import _lib as L
    from dreamer_amd import hip
    from formula import FULL
    torch.manual_seed(0)
    d = Dreamer(dict(FULL), gpu)
    crit = d.agent.critic
    M = 256
    g = torch.Generator().manual_seed(4)
    h = torch.randn(M, d.hidden_state_dims, generator=g).to(gpu)
    R, C = d.latent_state_dims
    z = torch.nn.functional.one_hot(torch.randint(0, C, (M, R), generator=g), C).float().reshape(M, -1).to(gpu)
    out = {}
    for prec in (0, 1):
        dm = L.dr_dims()
        dm.hidden, dm.rows, dm.cols = h.shape[1], z.shape[1], 1
        dm.critic_h1, dm.critic_h2 = crit.value_net[0].out_features, crit.value_net[3].out_features
        dm.buckets = crit.num_buckets
        dm.precision = prec
        lg = torch.empty(M, crit.num_buckets, device=gpu)
        v = torch.empty(M, device=gpu)
        ws = torch.empty(L.query("dr_critic_tape_bytes", dm, M), dtype=torch.uint8, device=gpu)
        L.call("dr_critic_fwd", dm, crit.struct(), M, L.ptr(h), h.shape[1], L.ptr(z), z.shape[1], L.ptr(lg),
               L.ptr(v), None, L.ptr(ws), ws.numel(), hip.stream())
        torch.cuda.synchronize()
        out[prec] = lg.cpu()
    err = float((out[1] - out[0]).norm() / out[0].norm())
    print(f"critic logits bf16 vs fp32: normwise rel err {err:.2e}")
    assert 1e-6 < err <= 2e-2
