"""The persistent unroll (dream.hip) where it cannot run: on a stream whose
CUs cannot hold every workgroup, dr_imagine_fwd must detect it
(DR_E_UNSUPPORTED inside the library) and run the launch form instead, with
the oracle's results (Dreamer.dream_episodes, Dreamer.py:143-175).  The same
call on the full stream runs the persistent kernel (its GRU counter reaches
60 H), also with the oracle's results.  Tolerances as test_gpu_parity.py."""
import ctypes

import pytest
import torch

from baseline_case import TieGuard
from gpu_helpers import close
from oracle import dreamer_oracle as O

pytestmark = pytest.mark.gpu
R, C, A, HD = 32, 32, 3, 600


def _idx(z):
    return z.reshape(*z.shape[:-2], -1, z.shape[-1]).argmax(-1).cpu()


def _gru_counter(ws, d, B, H):
    """the unroll's GRU-stage counter of rows 0..15 (dream.hip counter block,
    which ends where the BPTT's block starts at the end of the workspace)"""
    from dreamer_amd import _lib as L
    total = L.query("dr_imagine_workspace_bytes", d, B, H)
    pb = (4 * B * H * (4 * 200 + 200 + 2 * 1800 + 600 + 1664 + 2 * 200 + 1024 + 600) + 8 * 8 * 32 * 4) if B <= 64 else 0
    o = (total - pb) - 7 * 16 * 32 * 4 + 2 * 16 * 32 * 4
    return int(ws.view(torch.uint8)[o:o + 4].view(torch.int32).item())


@pytest.mark.parametrize("narrow", [False, True])
def test_unroll_on_full_and_narrow_streams(narrow, gpu):
    from dreamer_amd import Dreamer, hip
    from dreamer_amd import _lib as L
    from dreamer_amd.engine import cu_mask_words
    from formula import FULL
    B, H = 16, 15
    cfg = dict(FULL)
    cfg.update(batch_size=B, horizon=H)
    torch.manual_seed(0)
    d = Dreamer(cfg, gpu)
    P = {k: v.detach().cpu().clone() for k, v in d.state_dict().items()}
    g = torch.Generator().manual_seed(21)
    h0 = torch.randn(B, 1, HD, generator=g)
    z0 = torch.nn.functional.one_hot(torch.randint(0, C, (B, 1, R), generator=g), C).float()
    eps = torch.randn(H, B, 1, A, generator=g)
    q = torch.empty(H, B * R, C).exponential_(generator=g)
    with TieGuard():
        ref = O.dream(z0, h0, P, eps, q, H, R, C)
    dims = d.world_model.dims(d.agent)
    ws = hip.workspace(gpu).get("im", L.query("dr_imagine_workspace_bytes", dims, B, H))
    ws.zero_()
    if narrow:
        # 20 % of the CUs: fewer than the unroll's 60 workgroups at B = 16
        n = ctypes.c_int(0)
        L.call("dr_device_cus", ctypes.byref(n))
        words = cu_mask_words(n.value, 0.2)
        assert sum(bin(w).count("1") for w in words) < 60
        mask = (ctypes.c_uint * len(words))(*words)
        h = ctypes.c_void_p()
        L.call("dr_stream_create_cumask", len(words), mask, ctypes.byref(h))
        stream = torch.cuda.ExternalStream(h.value, device=gpu)
    else:
        stream = torch.cuda.current_stream(gpu)
    stream.wait_stream(torch.cuda.current_stream(gpu))
    with torch.cuda.stream(stream):
        out = d._imagine_raw(z0.to(gpu), h0.to(gpu), eps=eps.to(gpu), q=q.to(gpu))[0]
    stream.synchronize()
    torch.cuda.current_stream(gpu).wait_stream(stream)
    assert _gru_counter(ws, dims, B, H) == (0 if narrow else 60 * H)
    close(out[1], ref[1], 2e-4, 2e-5, "dream hiddens")
    assert torch.equal(_idx(out[0][:, 1:]), _idx(ref[0][:, 1:]))
    close(out[2], ref[2], 2e-4, 2e-5, "dream actions")
    close(out[3], ref[3], 2e-4, 2e-5, "dream rewards")
    if narrow:
        torch.cuda.synchronize()
        L.call("dr_stream_destroy", h)


def _narrow_stream(gpu, frac):
    """A HIP stream restricted to round(frac * CUs) CUs (frac >= 1: the current
    stream); returns (stream, handle or None)."""
    from dreamer_amd import _lib as L
    from dreamer_amd.engine import cu_mask_words
    if frac >= 1.0:
        return torch.cuda.current_stream(gpu), None
    n = ctypes.c_int(0)
    L.call("dr_device_cus", ctypes.byref(n))
    words = cu_mask_words(n.value, frac)
    mask = (ctypes.c_uint * len(words))(*words)
    h = ctypes.c_void_p()
    L.call("dr_stream_create_cumask", len(words), mask, ctypes.byref(h))
    return torch.cuda.ExternalStream(h.value, device=gpu), h


@pytest.mark.parametrize("B,frac", [(16, 0.4), (64, 0.4), (64, 1.0)])
def test_bptt_on_narrow_stream_vs_oracle(B, frac, gpu):
    """The persistent BPTT (bptt.hip) on a CU-masked stream: its grid shrinks to
    the stream's CUs (96 workgroups at 40 %), so every stage walks several
    tiles per workgroup through its grid stride.  The actor
    gradient of L = sum(g_mu mu + g_sigma sigma) through the H-step unroll
    (Dreamer.dream_episodes' graph, Dreamer.py:143-175) against the oracle's
    autograd; the kernel's status word is 0, its Q7 counter of rows 0..15
    reached 51 H and every workgroup left through the exit ticket."""
    from dreamer_amd import Dreamer, hip
    from dreamer_amd import _lib as L
    from formula import FULL
    H = 15
    cfg = dict(FULL)
    cfg.update(batch_size=B, horizon=H)
    torch.manual_seed(0)
    d = Dreamer(cfg, gpu)
    P = {k: v.detach().cpu().clone() for k, v in d.state_dict().items()}
    g = torch.Generator().manual_seed(31 + B)
    h0 = torch.randn(B, 1, HD, generator=g)
    z0 = torch.nn.functional.one_hot(torch.randint(0, C, (B, 1, R), generator=g), C).float()
    eps = torch.randn(H, B, 1, A, generator=g)
    q = torch.empty(H, B * R, C).exponential_(generator=g)
    g_mu = torch.randn(B, H, A, generator=g)
    g_sg = torch.randn(B, H, A, generator=g)
    leaves = []
    for k in O.ACTOR_KEYS:
        P["agent." + k] = P["agent." + k].clone().requires_grad_(True)
        leaves.append(P["agent." + k])
    with TieGuard():
        ref = O.dream(z0, h0, P, eps, q, H, R, C)
    loss = (g_mu * ref[5]).sum() + (g_sg * ref[6]).sum()
    ref_g = torch.autograd.grad(loss, leaves)
    dims = d.world_model.dims(d.agent)
    assert L.query("dr_persistent_kernels", dims, B, 32, H) & 4
    out, tape = d._imagine_raw(z0.to(gpu), h0.to(gpu), eps=eps.to(gpu), q=q.to(gpu))
    ag = d.agent
    f = ag.fa
    grad_flat = torch.zeros_like(f.flat)
    gptr = lambda n: grad_flat.data_ptr() + 4 * f.offsets[n]
    gs = L.dr_actor(*(L.dr_linear(gptr(w), gptr(b)) for w, b in (
        ("base_net.0.weight", "base_net.0.bias"), ("base_net.1.weight", "base_net.1.bias"),
        ("base_net.3.weight", "base_net.3.bias"), ("base_net.4.weight", "base_net.4.bias"),
        ("mu_head.weight", "mu_head.bias"), ("log_sig_head.weight", "log_sig_head.bias"))))
    total = L.query("dr_imagine_workspace_bytes", dims, B, H)
    ws = torch.zeros(total, dtype=torch.uint8, device=gpu)
    gm, gsd = g_mu.to(gpu).contiguous(), g_sg.to(gpu).contiguous()
    stream, h = _narrow_stream(gpu, frac)
    stream.wait_stream(torch.cuda.current_stream(gpu))
    with torch.cuda.stream(stream):
        L.call("dr_imagine_bwd", dims, d.world_model.packed(), ag.actor_struct(), B, H, L.ptr(out[0]),
               L.ptr(out[1]), L.ptr(out[2]), L.ptr(gm), L.ptr(gsd), None, None, None, L.ptr(tape), gs, L.ptr(ws),
               ws.numel(), stream.cuda_stream)
    stream.synchronize()
    torch.cuda.current_stream(gpu).wait_stream(stream)
    if h is not None:
        L.call("dr_stream_destroy", h)
    pcnt = total - 8 * 8 * 32 * 4
    word = lambda o: int(ws[o:o + 4].view(torch.int32).item())
    n_cus = ctypes.c_int(0)
    L.call("dr_device_cus", ctypes.byref(n_cus))
    grid = min(max(1, int(round(n_cus.value * min(frac, 1.0)))), 256) & ~7
    assert word(pcnt + 7 * 8 * 32 * 4) == 0, "BPTT status word"
    assert word(pcnt + 6 * 8 * 32 * 4) == 51 * H, "BPTT Q7 counter (rows 0..15)"
    assert word(pcnt + (7 * 8 + 1) * 32 * 4) == grid, "BPTT exit ticket"
    for k, r_ in zip(O.ACTOR_KEYS, ref_g):
        name = k.split(".", 1)[1]
        got = grad_flat[f.offsets[name]:f.offsets[name] + r_.numel()].view(r_.shape)
        scale = float(r_.abs().max()) + 1e-12
        close(got, r_, 2e-3, 2e-4 * scale, f"B{B} narrow {frac}: grad {k}")


def _fault_case(gpu, B=64):
    """configs[1]'s shape (B = 64, S = 64, H = 15), full widths, the bench's
    synthetic replay: every part of the epoch runs persistent."""
    import bench
    from dreamer_amd import Dreamer
    from test_gpu_baseline import CAR
    cfg = dict(CAR)
    cfg.update(batch_size=B, sequence_length=64, horizon=15, AC_epochs=1, buffer_size=4096)
    torch.manual_seed(0)
    d = Dreamer(cfg, gpu)
    fr, ac, rw, ct = bench.synthetic_replay(4096, (64, 64), 3, seed=0)
    d.buffer.load_arrays(fr, ac, rw, ct)
    return d


@pytest.mark.parametrize("which", ["scan", "dream", "bptt", "timeout"])
def test_forced_timeout_skips_update_and_raises(which, gpu, monkeypatch):
    """a timed-out wait in a persistent kernel must never be
    consumed silently.  DREAMER_PERSIST_FORCE makes every wait of the named
    kernel (all three: "timeout") time out.  Then the kernel NaN-fills its
    outputs and the fault slot; the epoch's update is skipped like the
    reference's non-finite skip (Agent.py:137-139): actor, critic and target
    parameters unchanged; the host-mapped fault word is set and the next
    train_Agent() raises; after that the engine runs the launch form and
    updates again."""
    import numpy as np
    monkeypatch.setenv("DREAMER_PERSIST_FORCE", which)
    d = _fault_case(gpu)
    ag = d.agent
    assert d.engine.persistent_bptt()
    np.random.seed(5)
    before = [t.detach().clone() for t in (ag.fa.flat, ag.fc.flat, ag.ft.flat)]
    d.train_Agent()
    torch.cuda.synchronize()
    assert not torch.isfinite(ag.fault_slot()).all(), "fault slot not set"
    for a, b in zip(before, (ag.fa.flat, ag.fc.flat, ag.ft.flat)):
        assert torch.equal(a, b), "the faulted epoch's update was applied"
    assert int(ag.fault_host()[0][0]) == 1, "host-mapped fault word not set"
    with pytest.raises(RuntimeError, match="persistent kernel"):
        d.train_Agent()  # sees the fault of the finished epoch before queueing another
    assert not ag.persistent_ok and not d.engine.persistent_bptt()
    assert float(ag.fault_slot()) == 0.0 and int(ag.fault_host()[0][0]) == 0
    la, lc = d.train_Agent()
    torch.cuda.synchronize()
    d.engine.check_faults()
    assert np.isfinite(float(la)) and np.isfinite(float(lc))
    assert not torch.equal(before[0], ag.fa.flat) and not torch.equal(before[1], ag.fc.flat)
    assert all(bool(torch.isfinite(t).all()) for t in (ag.fa.flat, ag.fc.flat, ag.ft.flat))
