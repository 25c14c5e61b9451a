"""Digest of the agent after a few train_Agent() epochs (bench.py's B = 256
setup, fixed seeds): sha256 of the actor / critic parameters and the last
losses.  Two library variants whose kernels should be bitwise the same
(DREAMER_LIB_VARIANT) must print the same digest.
python tools/epoch_digest.py [B] [fp32|bf16] [epochs]   (GPU box)"""
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
    for _ in range(n):
        la, lc = d.train_Agent()
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for t in (d.agent.fa.flat, d.agent.fc.flat):
        h.update(t.detach().cpu().numpy().tobytes())
    print(f"digest {prec} B={B} epochs={n}: {h.hexdigest()[:16]} losses {float(la):.9g} {float(lc):.9g}", flush=True)


if __name__ == "__main__":
    main()
