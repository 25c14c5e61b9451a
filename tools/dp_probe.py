"""Per-phase timing of a data-parallel train_Agent epoch (gloo rehearsal: all
ranks on the box's one GPU).  Run under torch.distributed.run with
DREAMER_DIST_BACKEND=gloo; rank 0 prints per-phase ms (HIP events around each
phase graph + its collective) and the wall ms of whole epochs."""
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    group = None
    if world > 1:
        dist.init_process_group("gloo")
        group = dist.group.WORLD
    _, d = bench.make_dreamer(bench.CAR_RACER, dev, B, 64, 15, 64, 1, world, rank, group, "fp32")
    eng = d._engine
    rng = np.random.RandomState(rank)
    for it in range(6):
        starts = d.buffer.sample_start_indices(B)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.run(starts, timing=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if rank == 0 and it >= 2:
            ph = eng.phase_ms()
            print(f"epoch {it}: wall {1e3 * (t1 - t0):.2f} ms  phases " +
                  " ".join(f"{k}={v:.2f}" for k, v in ph.items()), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
