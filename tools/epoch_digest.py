"""Digest of the agent after a few train_Agent() epochs (bench.py's B = 256
setup, fixed seeds): sha256 of the actor / critic parameters and the last
losses.  Two library variants whose kernels should be bitwise the same
(DREAMER_LIB_VARIANT) must print the same digest.
python tools/epoch_digest.py [B] [fp32|bf16] [epochs] [wm]   (GPU box)
With `wm`: the same for WorldModel.training_step (bench.py's ring feed, fixed
window starts): sha256 of the world-model parameters and the last loss."""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    prec = sys.argv[2] if len(sys.argv) > 2 else "bf16"
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    np.random.seed(1000)
    _, d = bench.make_dreamer(bench.CAR_RACER, dev, B, 64, 15, 64, 1, 1, 0, None, prec)
    if len(sys.argv) > 4 and sys.argv[4] == "wm":
        wm = d.world_model
        for _ in range(n):
            wm.train_step_ring(d.buffer, d.buffer.sample_start_indices(B))
        torch.cuda.synchronize()
        h = hashlib.sha256()
        for p in wm.parameters():
            h.update(p.detach().float().cpu().numpy().tobytes())
        print(f"wm digest {prec} B={B} steps={n}: {h.hexdigest()[:16]} loss {float(wm.last_losses[0]):.9g}", flush=True)
        return
    for _ in range(n):
        la, lc = d.train_Agent()
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for t in (d.agent.fa.flat, d.agent.fc.flat):
        h.update(t.detach().cpu().numpy().tobytes())
    print(f"digest {prec} B={B} epochs={n}: {h.hexdigest()[:16]} losses {float(la):.9g} {float(lc):.9g}", flush=True)


if __name__ == "__main__":
    main()
