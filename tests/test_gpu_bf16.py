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
A full train_Agent epoch in bf16 mode at configs[1] (B = 64) and the north-star
batch (B = 256) is bounded element-wise against the fp32 oracle on widely
tie-guarded noise (test_train_agent_bf16_epoch_vs_oracle states the bounds).
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


# bf16 mode does not promise the fp32 mode's categorical draws: a feature
# error of ~1e-3 flips any draw whose top-2 scores are that close, and one
# flip changes the row's whole trajectory.  The epoch test therefore widens
# every near-tie of the (fp32) oracle's draws to a margin far above bf16 error
# (TieGuard: runners-up within 3 % of the top score pushed down by 10 %), so
# bf16 and the oracle walk the same trajectories and every output can be
# bounded element-wise.
BF16_TIE_REL, BF16_TIE_SCALE = 3e-2, 1.10


def _nw(a, b):
    a, b = a.detach().float().cpu().reshape(-1), b.detach().float().cpu().reshape(-1)
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


@pytest.mark.parametrize("B", [64, 256])
def test_train_agent_bf16_epoch_vs_oracle(B, gpu):
    """One train_Agent epoch in bf16 perf mode (precision="bf16") at configs[1]
    (B = 64) and the north-star batch (B = 256; its chain tile GEMMs are bf16
    too), S = 64, H = 15, against the fp32 CPU oracle on the same replay
    windows, weights (default init) and widely tie-guarded noise (above).

    Bounds (the stated bf16 tolerances of the epoch):
      warm-start and imagined categorical indices: flip fraction <= 1e-3
        (measured 0 on the guarded noise);
      warm-start h0, imagined hiddens / mus / sigmas, lambda returns:
        normwise relative error <= 1e-2;
      critic loss: relative 1e-2; actor loss: |d| <= 1e-2 max(|ref|, 0.1);
      S: relative 1e-3;
      clipped actor and critic gradients: normwise relative 2e-2 per buffer.
    The measured values are printed (first GPU run: B = 256 h0 5.0e-4, R 2.2e-3,
    actor / critic gradients 2.9e-3 / 1.3e-3, no flips on 11,159 guarded of
    385,024 draws; B = 64 is fp32 past the encoder, so only the sampled indices
    could differ)."""
    import bench
    from baseline_case import TieGuard, oracle_epoch
    from test_gpu_baseline import CAR, run_gpu_epoch
    from dreamer_amd import Dreamer
    from oracle import dreamer_oracle as O
    S, H, R, C, A = 64, 15, 32, 32, 3
    cfg = dict(CAR)
    cfg.update(batch_size=B, sequence_length=S, horizon=H, precision="bf16")
    torch.manual_seed(0)
    d = Dreamer(cfg, gpu)
    P = {k: v.detach().cpu().clone() for k, v in d.state_dict().items()}
    n = 4096
    frames, acts, rews, conts = bench.synthetic_replay(n, (64, 64), A, seed=0)
    starts = np.random.RandomState(500 + B).randint(0, n - S + 1, size=B)
    g = torch.Generator().manual_seed(600 + B)
    q_warm = torch.empty(S // 2, B * R, C).exponential_(generator=g)
    eps = torch.randn(H, B, 1, A, generator=g)
    q = torch.empty(H, B * R, C).exponential_(generator=g)
    idx = starts[:, None] + np.arange(S)[None, :]
    obs = torch.tensor(frames[idx], dtype=torch.float32)
    act = torch.tensor(acts[idx])
    S0 = 3.0
    torch.set_num_threads(16)
    ref = oracle_epoch(P, obs, act, S, H, R, C, q_warm, eps, q, S0, guard=TieGuard(BF16_TIE_REL, BF16_TIE_SCALE))
    eng, pre = run_gpu_epoch(d, frames, acts, rews, conts, n, 0, starts, q_warm, eps, q, S0)
    from gpu_helpers import assert_persistent_ran
    assert_persistent_ran(eng)  # B = 64: scan, unroll and BPTT ran persistent, status 0
    ag = d.agent
    m = {}
    zw = (eng.z0.cpu().reshape(-1, C).argmax(-1) != ref["z0"].reshape(-1, C).argmax(-1)).float().mean()
    lat, hid, act_r, rew, cont, mu, sg = ref["dream"]
    zd = (eng.latents.cpu().reshape(-1, C).argmax(-1) != lat.reshape(-1, C).argmax(-1)).float().mean()
    m["flip_warm"], m["flip_dream"] = float(zw), float(zd)
    m["h0"] = _nw(eng.h0, ref["h0"])
    m["hiddens"] = _nw(eng.hiddens, hid)
    m["mus"] = _nw(eng.mus, mu)
    m["sigmas"] = _nw(eng.sigmas, sg)
    m["R"] = _nw(pre["R"], ref["ts"]["R"])
    la_ref, lc_ref = float(ref["ts"]["loss_actor"]), float(ref["ts"]["loss_critic"])
    m["loss_actor"] = (pre["la"], la_ref)
    m["loss_critic"] = (pre["lc"], lc_ref)
    m["S"] = (pre["S"], float(ref["ts"]["S"]))
    for f, keys, grads, name in ((ag.fa, O.ACTOR_KEYS, ref["ts"]["grad_actor_clipped"], "grad_actor"),
                                 (ag.fc, O.CRITIC_KEYS, ref["ts"]["grad_critic_clipped"], "grad_critic")):
        want = torch.cat([gr.reshape(-1) for gr in grads])
        got = torch.cat([f.grad[f.offsets[k.split(".", 1)[1]]:f.offsets[k.split(".", 1)[1]] + gr.numel()].cpu()
                         for k, gr in zip(keys, grads)])
        m[name] = _nw(got, want)
    print(f"bf16 epoch B={B} vs fp32 oracle (guarded {ref['guarded']}/{ref['draws']} draws): {m}")
    assert m["flip_warm"] <= 1e-3 and m["flip_dream"] <= 1e-3, m
    for k in ("h0", "hiddens", "mus", "sigmas", "R"):
        assert m[k] <= 1e-2, (k, m[k])
    assert abs(pre["lc"] - lc_ref) <= 1e-2 * abs(lc_ref), m["loss_critic"]
    assert abs(pre["la"] - la_ref) <= 1e-2 * max(abs(la_ref), 0.1), m["loss_actor"]
    assert abs(pre["S"] - float(ref["ts"]["S"])) <= 1e-3 * abs(float(ref["ts"]["S"])), m["S"]
    assert m["grad_actor"] <= 2e-2 and m["grad_critic"] <= 2e-2, m


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


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_encoder_persistent_tiles_match_reference(gpu, precision):
    """The persistent conv1 + conv2 kernels (k_enc12_split3: one workgroup per
    CU in fp32; the one-term form, two per CU, in bf16) walk several tiles per
    workgroup only when the frames outnumber the resident grid: 1536 frames =
    3072 half-frame tiles, against 256 / 512 resident workgroups.  Every frame
    is checked on its own (a wrong tile in a later loop iteration must not hide
    in a normwise average): fp32 against torch's f32 stack at 1e-5, bf16 against
    the bf16 emulation at 4e-3 per frame (2e-3 normwise).  Measured: fp32 worst
    frame 2.7e-7, bf16 worst frame 1.0e-3 (normwise 8.7e-4)."""
    from dreamer_amd import Dreamer
    from formula import FULL
    cfg = dict(FULL)
    cfg.update(precision=precision)
    torch.manual_seed(0)
    d = Dreamer(cfg, gpu)
    wm = d.world_model
    g = torch.Generator().manual_seed(7)
    frames = torch.randint(0, 256, (1536, 3, 64, 64), generator=g, dtype=torch.uint8)
    got = _features(wm.packed(), wm.dims(d.agent), frames, gpu)
    P = {k: v.detach().cpu() for k, v in wm.encoder.state_dict().items()}
    if precision == "bf16":
        ref = _emulate(frames, P)
        tol_frame, tol_all = 4e-3, 2e-3
    else:
        x = frames.float() / 255.0 - 0.5
        for i in range(4):
            x = F.silu(F.conv2d(x, P[f"feature_extractor.{2 * i}.weight"], P[f"feature_extractor.{2 * i}.bias"],
                                stride=2, padding=1))
        flat = x.flatten(1)
        ref = flat @ P["latent_mapper.0.weight"][:, :flat.shape[1]].t() + P["latent_mapper.0.bias"]
        tol_frame, tol_all = 1e-5, 1e-5
    per_frame = ((got - ref).norm(dim=1) / ref.norm(dim=1)).max().item()
    err = float((got - ref).norm() / ref.norm())
    print(f"{precision}: 1536 frames, normwise {err:.2e}, worst frame {per_frame:.2e}")
    assert err <= tol_all and per_frame <= tol_frame, (err, per_frame)


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
