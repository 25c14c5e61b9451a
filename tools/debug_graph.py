"""Diagnose eager vs graph-replay differences of the fused epoch."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "tests/golden"); sys.path.insert(0, ".")
import numpy as np, torch
from conftest import load_fixture
from gpu_helpers import build, cpu
from formula import replay_data
from oracle import dreamer_oracle as O
from dreamer_amd.engine import ImaginationEngine

dev = torch.device("cuda:0")
fx = load_fixture("small_epoch")
res = []
for mode in ("eager", "eager2", "graph"):
    d, P = build("small", dev, fx, B=8, S=8, H=5)
    fr, ac, rw, ct = replay_data(64, (32, 32), 3, seed=3)
    d.buffer.load_arrays(fr, ac, O.symlog(torch.tensor(rw)).numpy(), ct)
    eng = ImaginationEngine(d, use_graph=(mode == "graph"))
    eng.rng.reseed(1234)
    np.random.seed(7)
    snaps = []
    for e in range(3):
        la, lc = eng.run(d.buffer.sample_start_indices(8))
        torch.cuda.synchronize()
        snaps.append(dict(la=cpu(la), lc=cpu(lc), z0=cpu(eng.z0), h0=cpu(eng.h0), lat=cpu(eng.latents),
                          hid=cpu(eng.hiddens), R=cpu(eng.R), fa=cpu(d.agent.fa.flat), fc=cpu(d.agent.fc.flat),
                          ft=cpu(d.agent.ft.flat), S=cpu(d.agent.S_dev), rng=eng.rng.state.cpu().clone(),
                          starts=cpu(eng.starts)))
    res.append(snaps)
for other in (1, 2):
    print("== eager vs", ("eager2", "graph")[other - 1])
    for e in range(3):
        for k in res[0][e]:
            a, b = res[0][e][k].float(), res[other][e][k].float()
            if not torch.equal(a, b):
                print(f" epoch {e} {k}: max|d|={float((a-b).abs().max()):.3g}")
print("done")
