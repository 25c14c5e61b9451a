"""A few world-model training steps (B=64, T=15, CarRacing widths) from the
device replay ring, for rocprofv3 kernel traces of the WM step alone.
  rocprofv3 --kernel-trace --stats -d gpurun_out/wmprof -- python3 tools/wm_prof.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dreamer_amd import Dreamer  # noqa: E402


def main(steps=int(os.environ.get("WM_STEPS", "6")), B=int(os.environ.get("WM_B", "64"))):
    dev = torch.device("cuda", 0)
    cfg = dict(bench.CAR_RACER)
    cfg.update(batch_size=B, precision=os.environ.get("WM_PREC", "fp32"))
    torch.manual_seed(0)
    d = Dreamer(cfg, dev)
    fr, ac, rw, ct = bench.synthetic_replay(4096, cfg["observation_dims"], cfg["action_dims"], seed=0)
    d.buffer.load_arrays(fr, ac, rw, ct)
    np.random.seed(0)
    s, g, loss = bench.bench_wm(d, B, steps, 2)
    fl = bench.wm_step_flops(cfg, B, cfg["horizon"])
    print(f"WM step B={B} T={cfg['horizon']}: {s * 1e3:.3f} ms wall, {g * 1e3:.3f} ms GPU, "
          f"{fl / s / 1e12:.1f} TFLOP/s, loss {loss:.3f}, precision {cfg['precision']}")


if __name__ == "__main__":
    main()
