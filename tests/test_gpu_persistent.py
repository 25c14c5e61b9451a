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
