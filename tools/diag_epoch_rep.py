"""Repeatability of one train_Agent epoch's phases at the headline shape: the
state the phases read (Philox state, S, gradient / loss buffers) is restored
before each replay of the captured phase graphs (encwarm, imagine, returns,
update); every output buffer is compared bitwise with the first replay, in
phase order (GPU box).  usage: diag_epoch_rep.py PREC REPS [eager]"""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench

prec = sys.argv[1]
reps = int(sys.argv[2])
eager = len(sys.argv) > 3 and sys.argv[3] == "eager"
dev = torch.device("cuda:0")
np.random.seed(1000)
cfg, d = bench.make_dreamer(bench.CAR_RACER, dev, 256, 64, 15, 64, 1, 1, 0, None, prec)
for _ in range(3):
    d.train_Agent()
torch.cuda.synchronize()
e, ag = d._engine, d.agent
starts = d.buffer.sample_start_indices(e.B)
e.starts.copy_(torch.as_tensor(np.asarray(starts, dtype=np.int64)))
snap = dict(rng=e.rng.state.clone(), S=ag.S_dev.clone(), gb=ag.grad_buffer.clone())
order = [("encwarm", ["feat", "z0", "h0"]),
         ("imagine", ["latents", "hiddens", "actions", "mus", "sigmas", "rewards", "continues", "tape"]),
         ("returns", ["V_t", "R"]),
         ("update", ["V_c", "norm", "loss_a", "g_mu", "g_sig", "ctape", "grad"])]
ref = None
prev = None
nbad = 0
for r in range(reps):
    e.rng.state.copy_(snap["rng"])
    ag.S_dev.copy_(snap["S"])
    ag.grad_buffer.copy_(snap["gb"])
    for k in range(4):
        if eager:
            e.phases()[k][1]()
        else:
            e.graph[k].replay()
    torch.cuda.synchronize()
    out = {}
    for ph, keys in order:
        for kk in keys:
            out[kk] = (ag.grad_buffer if kk == "grad" else getattr(e, kk)).clone()
    if ref is None:
        ref = out
        prev = out
        continue
    for ph, keys in order:
        diff = [kk for kk in keys if not torch.equal(out[kk].view(-1).view(torch.uint8), ref[kk].view(-1).view(torch.uint8))]
        if diff:
            nbad += 1
            kk = diff[0]
            a, b = out[kk].view(-1), ref[kk].view(-1)
            idx = (a.view(torch.uint8) != b.view(torch.uint8)).nonzero().flatten()
            rel = float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))
            prev_eq = torch.equal(out[kk], prev[kk]) if prev is not None else None
            if r < 12 or r % 50 == 0:
                print(f"rep {r}: first mismatch in phase {ph}: {diff} ({kk}: {idx.numel()} bytes differ, first byte "
                      f"{int(idx[0])}, max rel diff {rel:.3g}, equal to previous rep {prev_eq})", flush=True)
            break
    prev = out
print(f"{prec} {'eager' if eager else 'graph'}: {nbad}/{reps - 1} replays differ", flush=True)
