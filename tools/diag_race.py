"""bench-style epochs (no host sync between train_Agent calls) with toggles,
printing the last epoch's losses: a run-to-run difference is a race (GPU box).
usage: diag_race.py PREC MODE   MODE: default | sync | nograph"""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
prec, mode = sys.argv[1], sys.argv[2]
dev = torch.device("cuda:0")
np.random.seed(int(sys.argv[3]) if len(sys.argv) > 3 else 1000)
cfg, d = bench.make_dreamer(bench.CAR_RACER, dev, 256, 64, 15, 64, 1, 1, 0, None, prec)
if mode == "nograph":
    d._engine.use_graph = False
cpu = next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")), "?")
psum = sum(float(p.double().sum()) for p in d.parameters())
print("cpu", cpu, "param checksum", repr(psum), flush=True)
hist = []
for ep in range(23):
    la, lc = d.train_Agent()
    hist.append(la)
    if mode == "sync":
        torch.cuda.synchronize()
        if not np.isfinite(float(la)):
            print("non-finite actor loss at epoch", ep, flush=True)
            e = d._engine
            for k in ("mus", "sigmas", "actions", "rewards", "continues", "V_t", "V_c", "R", "norm", "latents",
                      "hiddens", "g_mu", "g_sig", "loss_a"):
                v = getattr(e, k)
                fin = torch.isfinite(v)
                print(f"  {k}: finite {bool(fin.all())} n_bad {int((~fin).sum())} absmax "
                      f"{float(v.nan_to_num(0, 0, 0).abs().max()):.4g} min {float(v.nan_to_num(0, 0, 0).min()):.4g}",
                      flush=True)
            break
torch.cuda.synchronize()
print(prec, mode, " ".join(f"{float(x):.7f}" for x in hist[-4:]), flush=True)
