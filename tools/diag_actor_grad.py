"""Actor / critic gradient norms of consecutive train_Agent epochs on the HIP
path (pre-clip: the flat gradient buffer after the update phase) and the
optimiser's effect (GPU box).
usage: diag_actor_grad.py B {synthetic|replay_data} {eager|graph}"""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench

B, data, mode = int(sys.argv[1]), sys.argv[2], sys.argv[3]
dev = torch.device("cuda:0")
np.random.seed(1000)
cfg, d = bench.make_dreamer(bench.CAR_RACER, dev, B, 64, 15, 64, 1, 1, 0, None, "fp32")
if data == "replay_data":  # the tests' fixture replay (raw N(0,1) rewards)
    for _p in ("tests", "tests/golden"):
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), _p))
    from formula import replay_data
    fr, ac, rw, ct = replay_data(4096, (64, 64), 3, seed=3)
    d.buffer.load_arrays(fr, ac, rw, ct)
    d.buffer._mirror()
e, ag = d._engine, d.agent
nA = sum(-(-p.numel() // 64) * 64 for p in ag.actor.parameters())
if mode == "graph":
    key = (ag.params_key(), d.world_model.params_key(), d.buffer.device_key())
    e._capture(key)
for ep in range(4):
    starts = d.buffer.sample_start_indices(e.B)
    e.starts.copy_(torch.as_tensor(np.asarray(starts, dtype=np.int64)))
    before = [p.detach().clone() for p in ag.actor.parameters()]
    wm_before = [p.detach().clone() for p in d.world_model.parameters()]
    for k, (name, body, _) in enumerate(e.phases()[:4]):
        if mode == "graph":
            e.graph[k].replay()
        else:
            body()
    torch.cuda.synchronize()
    g = ag.grad_buffer
    ga, gc = g[:nA].double(), g[nA:-2].double()
    print(f"epoch {ep}: |g_actor| {float(ga.norm()):.4g} |g_critic| {float(gc.norm()):.4g} "
          f"|h0| {float(e.h0.norm()):.5g} |hiddens| {float(e.hiddens.norm()):.5g} sig min {float(e.sigmas.min()):.3g} "
          f"|R| max {float(e.R.abs().max()):.3g} norm {float(e.norm):.4g}", flush=True)
    if mode == "graph":
        e.graph[4].replay()
    else:
        e.phases()[4][1]()
    torch.cuda.synchronize()
    moved = max(float((p.detach() - b).abs().max()) for p, b in zip(ag.actor.parameters(), before))
    wm_moved = max(float((p.detach() - b).abs().max()) for p, b in zip(d.world_model.parameters(), wm_before))
    print(f"   actor max |dp| {moved:.4g}  world-model max |dp| {wm_moved:.4g}", flush=True)
