"""bitwise repeatability of the bf16 encoder (dr_encoder_features over one
epoch's 8192 frames) and the bf16 tile GEMM (dr_critic_fwd, M = 4096 and 256):
a kernel race shows as an occasional mismatch (GPU box)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for _p in ("tests", "tests/golden"):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), _p))
from test_gpu_bf16 import _features
from dreamer_amd import Dreamer, _lib as L, hip
from formula import FULL

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
dev = torch.device("cuda:0")
cfg = dict(FULL)
cfg.update(observation_dims=[64, 64], precision=prec)
torch.manual_seed(0)
d = Dreamer(cfg, dev)
wm = d.world_model
dims = wm.dims(d.agent)
g = torch.Generator().manual_seed(1)
frames = torch.randint(0, 256, (8192, 3, 64, 64), generator=g, dtype=torch.uint8)
ref = _features(wm.packed(), dims, frames, dev)
bad = 0
for r in range(reps):
    x = _features(wm.packed(), dims, frames, dev)
    if not torch.equal(x, ref):
        bad += 1
        diff = (x != ref)
        rows = diff.any(1).nonzero().flatten()
        print(f"encoder rep {r}: {int(diff.sum())} elems differ, rows {rows[:8].tolist()} nan {int(torch.isnan(x).sum())}",
              flush=True)
print(f"{prec} encoder mismatching reps {bad}/{reps}", flush=True)

crit = d.agent.critic
for M in (4096, 256):
    h = torch.randn(M, d.hidden_state_dims, generator=g).to(dev)
    R, C = d.latent_state_dims
    z = torch.nn.functional.one_hot(torch.randint(0, C, (M, R), generator=g), C).float().reshape(M, -1).to(dev)
    dm = L.dr_dims()
    dm.hidden, dm.rows, dm.cols = h.shape[1], z.shape[1], 1
    dm.critic_h1, dm.critic_h2 = crit.value_net[0].out_features, crit.value_net[3].out_features
    dm.buckets = crit.num_buckets
    dm.precision = 1 if prec == "bf16" else 0
    ws = torch.empty(L.query("dr_critic_tape_bytes", dm, M), dtype=torch.uint8, device=dev)

    def run():
        lg = torch.empty(M, crit.num_buckets, device=dev)
        v = torch.empty(M, device=dev)
        L.call("dr_critic_fwd", dm, crit.struct(), M, L.ptr(h), h.shape[1], L.ptr(z), z.shape[1], L.ptr(lg),
               L.ptr(v), None, L.ptr(ws), ws.numel(), hip.stream())
        return lg
    ref = run().clone()
    bad = 0
    for r in range(reps * 4):
        if not torch.equal(run(), ref):
            bad += 1
    torch.cuda.synchronize()
    print(f"{prec} critic M={M} mismatching reps {bad}/{reps * 4}", flush=True)
