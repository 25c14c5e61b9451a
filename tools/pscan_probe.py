"""Stage timeline of the persistent posterior scan (scan.hip) on the GPU box.

Needs the DR_PSCAN_TS library variant (built by tools/build_pscan_ts.sh;
DREAMER_LIB_VARIANT=pscants): every workgroup stamps the 100 MHz wall clock at
each stage's entry, after its poll and after its signal.  Prints, per stage,
the median over workgroups of the wait (entry -> poll done) and the work
(poll done -> signal done), and the step period of stage S1.

  DREAMER_LIB_VARIANT=pscants python tools/pscan_probe.py [--batch 256] [--precision fp32]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--precision", default="fp32")
    a = ap.parse_args()
    import bench
    dev = torch.device("cuda:0")
    B, S, H = a.batch, 64, 15
    c, d = bench.make_dreamer(bench.CAR_RACER, dev, B, S, H, 64, 1, 1, 0, None, a.precision)
    eng = d._engine
    np.random.seed(0)
    for _ in range(3):
        eng.run(d.buffer.sample_start_indices(B))
    torch.cuda.synchronize()
    T = eng.T
    grid = {16: 60, 32: 120, 64: 240, 128: 256, 256: 256}[B]
    off = 4 * (2 * B * 600 + 2 * B * 200 + 4 * B * 32) + 6400 + 8 * B * 32  # scan.hip ring layout
    n = 64 * 24 * grid
    st = eng.ws_obs.view(torch.uint8)[off:off + 8 * n].view(torch.int64).cpu().numpy().reshape(64, 3, 8, grid)
    st = st[:T].astype(np.float64) / 100.0  # us
    t0 = st[st > 0].min()
    print(f"B={B} {a.precision}: T={T}, grid {grid}, kernel span of the stamps {st[st > 0].max() - t0:.1f} us")
    for t in list(range(0, 3)) + [T // 2, T - 1]:
        print(f"t={t:2d}")
        for sg in range(3):
            m = st[t, sg]
            live = m[7] > 0
            if not live.any():
                continue
            marks = [k for k in range(8) if (m[k][live] > 0).all()]
            seg = " ".join(f"{a}->{b} {np.median(m[b][live] - m[a][live]):6.2f}" for a, b in zip(marks, marks[1:]))
            print(f"   S{sg + 1}: entry {np.median(m[0][live]) - t0:8.1f}  {seg}  | last signal {np.max(m[7][live]) - t0:8.1f}")
    s1 = st[1:, 0, 7]
    per = np.diff(np.nanmedian(np.where(s1 > 0, s1, np.nan), axis=1))
    print("S1 step period (median signal time, us):", np.round(per, 2).tolist())


if __name__ == "__main__":
    main()
