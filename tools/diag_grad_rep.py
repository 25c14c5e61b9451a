"""Which gradients of the actor-critic update phase are not bitwise
repeatable: replays the captured update graph from a restored state and maps
differing elements of the flat [actor | critic] gradient buffer to parameter
names (GPU box).  usage: diag_grad_rep.py PREC REPS [phase]"""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for _p in ("tests", "tests/golden"):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), _p))
from formula import FULL, replay_data
from dreamer_amd import Dreamer

prec, reps = sys.argv[1], int(sys.argv[2])
phase = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # first phase replayed (through the update, 3)
dev = torch.device("cuda:0")
cfg = dict(FULL)
cfg.update(batch_size=256, sequence_length=64, horizon=15, buffer_size=2048, precision=prec)
torch.manual_seed(0)
d = Dreamer(cfg, dev)
fr, ac, rw, ct = replay_data(2048, (64, 64), 3, seed=3)
d.buffer.load_arrays(fr, ac, rw, ct)
np.random.seed(7)
d.train_Agent()
torch.cuda.synchronize()
e, ag = d.engine, d.agent
e.starts.copy_(torch.as_tensor(np.asarray(d.buffer.sample_start_indices(e.B), dtype=np.int64)))
e.rng.state.copy_(e.rng.state)
snap = (e.rng.state.clone(), ag.S_dev.clone(), ag.grad_buffer.clone())
for k in range(phase):
    e.graph[k].replay()
torch.cuda.synchronize()
names = []
off = 0
for mod, tag in ((ag.actor, "actor"), (ag.critic, "critic")):
    for n, p in mod.named_parameters():
        names.append((f"{tag}.{n}", off, p.numel()))
        off += -(-p.numel() // 64) * 64
ref = None
stats = {}
for r in range(reps):
    e.rng.state.copy_(snap[0]); ag.S_dev.copy_(snap[1]); ag.grad_buffer.copy_(snap[2])
    for k in range(phase, 4):
        e.graph[k].replay()
    torch.cuda.synchronize()
    g = ag.grad_buffer.clone()
    na = names[12][1] if len(names) > 12 else 0
    if r == 0:
        for n, o, c in names:
            x = g[o:o + c].double()
            print(f"   {n}: max|g| {float(x.abs().max()):.4g} rms {float(x.pow(2).mean().sqrt()):.4g} nonfinite {int((~torch.isfinite(x)).sum())}", flush=True)
        print(f"   g_mu max {float(e.g_mu.abs().max()):.4g} g_sig max {float(e.g_sig.abs().max()):.4g} sigmas min {float(e.sigmas.min()):.4g} max {float(e.sigmas.max()):.4g} |mus| max {float(e.mus.abs().max()):.4g} norm {float(e.norm):.4g}", flush=True)
    print(f"rep {r}: |g_actor| {float(g[:na].double().norm()):.6g} |g_critic| {float(g[na:-2].norm()):.6g} "
          f"losses {g[-2:].tolist()} |latents| {float(e.latents.norm()):.6g} |tape| {float(e.tape.view(torch.float32).nan_to_num().norm()):.6g}",
          flush=True)
    if ref is None:
        ref = g
        continue
    if torch.equal(g, ref):
        continue
    for n, o, c in names:
        a, b = g[o:o + c], ref[o:o + c]
        nd = int((a != b).sum())
        if nd:
            rel = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
            s = stats.setdefault(n, [0, 0, 0.0])
            s[0] += 1; s[1] = max(s[1], nd); s[2] = max(s[2], rel)
print(f"{prec} phase {phase}: differing parameters over {reps - 1} replays:", flush=True)
for n, (cnt, nd, rel) in stats.items():
    print(f"  {n}: {cnt} replays, up to {nd} elems, max rel {rel:.3g}", flush=True)
print("done", flush=True)
