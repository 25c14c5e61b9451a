"""Per-phase milliseconds of one graph-replayed train_Agent epoch (HIP events
between the engine's phase graphs) at several batch sizes: how the latency-
bound chain phases (posterior scan, dream, BPTT) scale with the rows per
launch.  python tools/phase_probe.py [B ...]  (GPU box)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    prec = os.environ.get("PRECISION", "fp32")
    Bs = [int(x) for x in sys.argv[1:]] or [64, 128, 256]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for B in Bs:
        np.random.seed(1)
        _, d = bench.make_dreamer(bench.CAR_RACER, dev, B, 64, 15, 64, 1, 1, 0, None, prec)
        eng = d._engine
        for _ in range(3):
            eng.run(d.buffer.sample_start_indices(B))
        torch.cuda.synchronize()
        rows = []
        for _ in range(10):
            eng.run(d.buffer.sample_start_indices(B), timing=True)
            torch.cuda.synchronize()
            rows.append(eng.phase_ms())
        med = {k: float(np.median([r[k] for r in rows])) for k in rows[0]}
        tot = sum(med.values())
        enc = eng.time_encoder(reps=5)
        print(f"{prec} B={B:4d} encoder {enc:6.3f} ms, epoch {tot:7.3f} ms | " + "  ".join(f"{k} {v:6.3f}" for k, v in med.items()), flush=True)
        del d, eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
