"""Host-side checks that need no GPU: the C ABI library loads and exports
every entry point include/dreamer_hip.h declares, the modules reproduce the
reference's state_dict layout, the Buffer reproduces the reference's sampling
RNG consumption, and the reference module names import."""
import os
import re
import sys

import numpy as np
import pytest
import torch

from conftest import REPO, load_fixture, state_layout
from formula import FULL, SMALL
from oracle import dreamer_oracle as O


def _header_symbols():
    src = open(os.path.join(REPO, "include", "dreamer_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dr_[A-Za-z0-9_]+)\s*\(", src)))


def test_abi_exports_every_declared_symbol():
    from dreamer_amd import _lib
    lib = _lib.load()
    declared = _header_symbols()
    assert len(declared) > 20
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    assert set(declared) == set(_lib.EXPORTED), set(declared) ^ set(_lib.EXPORTED)
    assert lib.dr_version() == 1


def test_workspace_queries_need_no_gpu():
    from dreamer_amd import _lib as L
    from dreamer_amd import Dreamer
    d = Dreamer(dict(FULL), torch.device("cpu"))
    dims = d.world_model.dims(d.agent)
    assert dims.hidden == 600 and dims.rows == 32 and dims.enc_hidden == 200 and dims.critic_h2 == 200
    assert L.query("dr_imagine_tape_bytes", dims, 64, 15) > 64 * 15 * 600 * 4 * 4
    assert L.query("dr_encoder_workspace_bytes", dims, 2048) > 2048 * 32 * 32 * 32 * 4


@pytest.mark.parametrize("which,cfg", [("small", SMALL), ("full", FULL)])
def test_state_dict_layout_matches_reference(which, cfg):
    from dreamer_amd import Dreamer
    d = Dreamer(dict(cfg), torch.device("cpu"))
    assert [(k, tuple(v.shape)) for k, v in d.state_dict().items()] == state_layout(which)


def test_reference_checkpoint_round_trip(tmp_path):
    """A reference-format state_dict loads (weights_only) and flat views survive."""
    from dreamer_amd import Dreamer
    fx = load_fixture("small_epoch")
    d = Dreamer(dict(SMALL), torch.device("cpu"))
    sd = {k: torch.from_numpy(fx["param_" + k].copy()) for k, _ in state_layout("small")}
    torch.save(sd, tmp_path / "ref.pth")
    d.load_pretrained_dreamer(str(tmp_path / "ref.pth"))
    for k, v in d.state_dict().items():
        assert torch.equal(v, sd[k]), k
    assert d.agent.fa.intact() and d.agent.fc.intact() and d.agent.ft.intact()
    d.save_trained_Dreamer(str(tmp_path / "mine.pth"))
    back = torch.load(str(tmp_path / "mine.pth"), weights_only=True)
    assert all(torch.equal(back[k], sd[k]) for k in sd)


def test_buffer_sampling_semantics():
    """Buffer.sample_start_indices == reference Buffer.sample_sequences' starts
    (fixture recorded from the reference, including the straddle redraw)."""
    from dreamer_amd import Buffer
    for name in ("small_epoch", "full_epoch"):
        fx = load_fixture(name)
        cap = int(fx["buf_capacity"])
        b = Buffer(cap, int(fx["cfg_S"]), int(fx["cfg_A"]), fx["buf_frames"].shape[2:])
        b.load_arrays(fx["buf_frames"], fx["buf_actions"], fx["buf_rewards"], fx["buf_continues"])
        b.size, b.next_idx = int(fx["buf_size"]), int(fx["buf_next_idx"])
        np.random.seed(int(fx["np_seed"]))
        assert np.array_equal(b.sample_start_indices(int(fx["cfg_B"])), fx["starts"])
        # host sample_sequences on CPU returns the reference's windows
        np.random.seed(int(fx["np_seed"]))
        obs, act, rew, cont, S = b.sample_sequences(int(fx["cfg_B"]))
        idx = (fx["starts"][:, None] + np.arange(S)[None, :]) % cap
        assert torch.equal(obs, torch.tensor(fx["buf_frames"][idx], dtype=torch.float32))


def test_add_to_buffer_symlog_and_wrap():
    from dreamer_amd import Buffer
    b = Buffer(4, 2, 3, (16, 16))
    for i in range(6):
        b.add_to_buffer(np.full((3, 16, 16), i, np.uint8), np.ones(3) * i, float(i) - 2.5, 1 - (i == 3))
    assert b.size == 4 and b.next_idx == 2
    assert b.observation_buffer[0, 0, 0, 0] == 4 and b.observation_buffer[3, 0, 0, 0] == 3
    np.testing.assert_allclose(b.reward_buffer[1, 0], O.symlog(torch.tensor(5 - 2.5)).item(), rtol=1e-6)
    assert b.continue_buffer[3, 0] == 0.0


def test_reference_module_names_import():
    sys.path.insert(0, os.path.join(REPO, "dreamer_amd", "refapi"))
    try:
        import Adaptors, Agent, Buffer, Dreamer, DreamerUtils, DynamicsPredictors  # noqa: F401
        import SequenceModel, VariationalAutoEncoder, WorldModel  # noqa: F401
        assert Dreamer.Dreamer.__module__ == "dreamer_amd.dreamer"
        assert hasattr(DreamerUtils, "_sanitize_for_save")
        arr = DreamerUtils._sanitize_for_save([torch.tensor(1.5), torch.tensor(2.0), 4.0])
        assert arr.tolist() == [1.5, 2.0, 4.0]
        arr = DreamerUtils._sanitize_for_save([[torch.tensor(1.0), 2.0], [torch.tensor(3.0), 4.0]])
        assert arr.shape == (2, 2)
    finally:
        sys.path.remove(os.path.join(REPO, "dreamer_amd", "refapi"))


def test_hot_path_refuses_cpu_tensors():
    """No CPU fallback: hot-path calls on CPU tensors raise."""
    from dreamer_amd import Dreamer
    d = Dreamer(dict(SMALL), torch.device("cpu"))
    h = torch.zeros(2, 1, SMALL["hidden_state_dims"])
    z = torch.zeros(2, 1, 8, 8)
    a = torch.zeros(2, 1, 3)
    with torch.no_grad(), pytest.raises(RuntimeError, match="GPU"):
        d.world_model.imagine_step(h, z, a)
    with pytest.raises(RuntimeError, match="GPU"):
        d.dream_episodes(z, h)


def test_world_model_gradient_buckets_partition_the_flat_buffer():
    """The three DP all-reduce buckets (DR_WM_BWD_HEADS / _SCAN / _ENC, world_model._grad_buckets)
    are disjoint, contiguous, cover every parameter, and hold exactly the
    parameters each backward stage finalises (include/dreamer_hip.h)."""
    from dreamer_amd import Dreamer
    from dreamer_amd.agent import _Flat
    d = Dreamer(dict(FULL), torch.device("cpu"))
    wm = d.world_model
    f = _Flat(wm)
    (h0, h1), (s0, s1), (e0, e1) = wm._grad_buckets(f)
    assert e0 == 0 and e1 == s0 and s1 == h0 and h1 == f.numel
    for n in f.names:
        o = f.offsets[n]
        if n.startswith("encoder.feature_extractor."):
            assert e0 <= o < e1, n
        elif n.startswith(("encoder.latent_mapper.", "sequence_model.")):
            assert s0 <= o < s1, n
        else:
            assert h0 <= o < h1, n
    print(f"bucket MB: heads+decoder {(h1 - h0) * 4e-6:.1f}, scan {(s1 - s0) * 4e-6:.1f}, "
          f"encoder {(e1 - e0) * 4e-6:.1f}")


def test_vector_observation_mode_host_side():
    """configs[4] vector observations: module shapes, dims and every workspace
    query computed on the host without a GPU (a zero conv-plane size must not
    reach an integer division)."""
    from dreamer_amd import Dreamer
    from dreamer_amd import _lib as L
    cfg = dict(FULL)
    cfg.update(observation_dims=[24], batch_size=4, sequence_length=8, horizon=6)
    d = Dreamer(cfg, torch.device("cpu"))
    sd = d.state_dict()
    assert tuple(sd["world_model.encoder.feature_extractor.0.weight"].shape) == (256, 24)
    assert tuple(sd["world_model.decoder.image_builder.2.weight"].shape) == (24, 256)
    assert d.buffer.observation_buffer.dtype == np.float32
    dims = d.world_model.dims(d.agent)
    assert dims.obs_dim == 24 and dims.img_h == 0
    for name, args in (("dr_encoder_workspace_bytes", (100,)), ("dr_observe_workspace_bytes", (100,)),
                       ("dr_decoder_workspace_bytes", (100,)), ("dr_wm_train_workspace_bytes", (4, 6)),
                       ("dr_imagine_workspace_bytes", (4, 6))):
        assert L.query(name, dims, *args) > 0, name


def _trunc16(x):
    """f32 -> the f32 value of its bf16 head (low 16 bits cleared), as split3_pair."""
    return (np.asarray(x, np.float32).view(np.uint32) & np.uint32(0xFFFF0000)).view(np.float32)


def test_split3_numerics_bound():
    """Host restatement of the fp32-on-bf16 split (common.h split3_pair,
    conv_split.hip): x = h + m + l with h, m truncated bf16 heads and l the
    truncated remainder; the residual subtractions are exact in f32, every
    term is a bf16 value, |x - (h + m + l)| < 2^-23 |x|, and the six-term
    product h_a h_b + h_a m_b + m_a h_b + h_a l_b + m_a m_b + l_a h_b is within
    2^-21 |a b| of the exact product (the order of one f32 rounding)."""
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(200000) * np.exp(rng.uniform(-20, 20, 200000))).astype(np.float32)
    h = _trunc16(x)
    r1 = (x - h).astype(np.float32)
    m = _trunc16(r1)
    r2 = (r1 - m).astype(np.float32)
    l = _trunc16(r2)
    # the subtractions are exact: recomposition in float64 gives x back up to l's truncation
    assert np.array_equal(h.astype(np.float64) + r1.astype(np.float64), x.astype(np.float64))
    assert np.array_equal(m.astype(np.float64) + r2.astype(np.float64), r1.astype(np.float64))
    for t in (h, m, l):  # every term is exactly a bf16 value
        assert not np.any(t.view(np.uint32) & np.uint32(0xFFFF))
    xs = x.astype(np.float64)
    rec = h.astype(np.float64) + m.astype(np.float64) + l.astype(np.float64)
    assert np.all(np.abs(xs - rec) <= 2.0 ** -23 * np.abs(xs))
    a, b = xs[:100000], xs[100000:]
    ha, ma, la = (t.astype(np.float64)[:100000] for t in (h, m, l))
    hb, mb, lb = (t.astype(np.float64)[100000:] for t in (h, m, l))
    six = ha * hb + ha * mb + ma * hb + ha * lb + ma * mb + la * hb
    assert np.all(np.abs(six - a * b) <= 2.0 ** -21 * np.abs(a * b))


def test_deep_vae_state_layout():
    """BASELINE configs[3]'s deeper VAE (config key encoder_depth = 5, 128 x 128
    frames): five encoder convs 3 -> 32 -> 64 -> 128 -> 256 -> 256 and five
    decoder convTs 256 -> 256 -> 128 -> 64 -> 32 -> 3; latent_mapper.0 still
    reads 4096 features + h (4 x 4 x 256), as the reference's 64 x 64 encoder
    does (VariationalAutoEncoder.py:33-55).  The default (no key) is the
    reference's 4-layer layout."""
    from dreamer_amd import Dreamer
    cfg = dict(FULL)
    cfg.update(observation_dims=[128, 128], encoder_depth=5, device="cpu")
    torch.manual_seed(0)
    sd = Dreamer(cfg, torch.device("cpu")).state_dict()
    enc = [tuple(sd[f"world_model.encoder.feature_extractor.{i}.weight"].shape) for i in range(0, 10, 2)]
    assert enc == [(32, 3, 4, 4), (64, 32, 4, 4), (128, 64, 4, 4), (256, 128, 4, 4), (256, 256, 4, 4)]
    dec = [tuple(sd[f"world_model.decoder.image_builder.{i}.weight"].shape) for i in range(0, 10, 2)]
    assert dec == [(256, 256, 4, 4), (256, 128, 4, 4), (128, 64, 4, 4), (64, 32, 4, 4), (32, 3, 4, 4)]
    assert tuple(sd["world_model.encoder.latent_mapper.0.weight"].shape) == (200, 4096 + 600)
    assert tuple(sd["world_model.decoder.upscaler.3.weight"].shape) == (4096, 200)
    cfg4 = dict(FULL)
    cfg4.update(device="cpu")
    sd4 = Dreamer(cfg4, torch.device("cpu")).state_dict()
    assert "world_model.encoder.feature_extractor.8.weight" not in sd4
    # the oracle walks however many layers the state_dict holds
    P = {k: v.detach() for k, v in sd.items()}
    g = torch.Generator().manual_seed(0)
    h = torch.randn(1, 2, 600, generator=g)
    obs = torch.rand(1, 2, 3, 128, 128, generator=g) - 0.5
    assert tuple(O.encoder_logits(h, obs, P).shape) == (1, 2, 1024)
    z = torch.nn.functional.one_hot(torch.randint(0, 32, (1, 2, 32), generator=g), 32).float()
    assert tuple(O.decoder_forward(h, z, P, (128, 128)).shape) == (1, 2, 3, 128, 128)


def test_tn_split3_predicate_covers_its_limits():
    """tn_launch routes a TN weight-gradient problem to the split3 kernel only
    when op_gemm_tn_split3 accepts it: the 4736-wide encoder
    projection gradient at K = B*T rows beyond ~151k exceeds the 32-bit plane
    offsets and must fall back to the f32 tile GEMM instead of failing."""
    import ctypes
    from dreamer_amd import _lib
    f = _lib.load().dr_internal_tn_split3_supported
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_int] * 3
    assert f(200, 4736, 3840) == 1        # the WM step's projection gradient at B = 256, T = 15
    assert f(200, 4736, 16384) == 1
    assert f(200, 4736, 160000) == 0      # > 2^31 plane elements
    assert f(200, 1624, 61440) == 1       # the critic's first layer at B = 4096, H + 1 = 16 (configs[4])
    assert f(0, 10, 10) == 0 and f(10, 10, 0) == 0


def test_cu_mask_words():
    """The fenced warm stream's CU mask (engine.cu_mask_words): 7/8 of 256 CUs
    keeps CUs 0-223 (words 0-6 full, word 7 empty); a fraction never keeps zero
    CUs or more than the device has; a partial word sets its low bits."""
    from dreamer_amd.engine import cu_mask_words
    w = cu_mask_words(256, 0.875)
    assert len(w) == 8 and w[:7] == [0xFFFFFFFF] * 7 and w[7] == 0
    assert sum(bin(x).count("1") for x in cu_mask_words(256, 0.75)) == 192
    assert cu_mask_words(256, 0.0001) == [1] + [0] * 7
    assert sum(bin(x).count("1") for x in cu_mask_words(304, 1.5)) == 304
    w = cu_mask_words(40, 0.5)
    assert w == [0xFFFFF, 0]
