"""Stage timeline of the persistent BPTT (bptt.hip) on the GPU box.

Needs the DR_PBPTT_TS library variant (tools/build_pbptt_ts.sh;
DREAMER_LIB_VARIANT=pbts): thread 0 of every workgroup stamps the 100 MHz wall
clock at marks of the first tile it runs in each stage (0 entry, 1 inputs
ready, 6 before the signal, 7 after it).  Prints, per stage, the medians over
workgroups of the mark-to-mark intervals and the step period.

  DREAMER_LIB_VARIANT=pbts python tools/pbptt_probe.py [--batch 64] [--precision bf16]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

STAGES = ["Q1 STE+W_p6", "Q2 LNb+W_p3", "Q3 LNb+W_p0+GRUb", "Q4 W_ih|W_hh", "Q5 heads bwd", "Q6 LNb+W_a3",
          "Q7 LNb+W_a0+totals"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--precision", default="bf16")
    a = ap.parse_args()
    import bench
    from dreamer_amd import _lib as L
    dev = torch.device("cuda:0")
    B, S, H = a.batch, 64, 15
    c, d = bench.make_dreamer(bench.CAR_RACER, dev, B, S, H, 64, 1, 1, 0, None, a.precision)
    eng = d._engine
    np.random.seed(0)
    for _ in range(3):
        eng.run(d.buffer.sample_start_indices(B))
    torch.cuda.synchronize()
    grid = 256
    nbytes = 16 * 7 * 8 * 256 * 8
    total = L.query("dr_imagine_workspace_bytes", eng.d, B, H)
    off = total - nbytes
    st = eng.ws_im.view(torch.uint8)[off:off + nbytes].view(torch.int64).cpu().numpy()
    st = st[:16 * 7 * 8 * grid].reshape(16, 7, 8, grid)[:H].astype(np.float64) / 100.0  # us
    pos = st[st > 0]
    t0 = pos.min()
    print(f"B={B} {a.precision}: H={H}, grid {grid}, kernel span of the stamps {pos.max() - t0:.1f} us "
          f"({(pos.max() - t0) / H:.1f} us per step)")
    for s in [0, 1, H // 2, H - 1]:
        print(f"s={s:2d}")
        for sg in range(7):
            m = st[s, sg]
            live = m[7] > 0
            if not live.any():
                continue
            marks = [k for k in range(8) if (m[k][live] > 0).all()]
            seg = " ".join(f"{x}->{y} {np.median(m[y][live] - m[x][live]):5.2f}" for x, y in zip(marks, marks[1:]))
            print(f"   {STAGES[sg]:22s} entry {np.median(m[0][live]) - t0:7.1f} {seg} | last signal "
                  f"{np.max(m[7][live]) - t0:7.1f}")
    dg = st[:, 6, 7]
    per = np.diff(np.nanmedian(np.where(dg > 0, dg, np.nan), axis=1))
    print("Q7 step period (median signal time, us):", np.round(per, 2).tolist())
    # the critical chain: last signal of each stage, step by step
    last = np.where(st[:, :, 7] > 0, st[:, :, 7], np.nan)
    lastmax = np.nanmax(np.where(st[:, :, 7, :] > 0, st[:, :, 7, :], np.nan), axis=2) - t0
    print("last signal per stage (us from the first stamp), steps 1..3:")
    for s in range(1, 4):
        print(f"   s={s}: " + " ".join(f"{v:7.1f}" for v in lastmax[s]))


if __name__ == "__main__":
    main()
