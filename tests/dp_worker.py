"""Worker for the data-parallel tests (spawned; one process per rank)."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.dirname(HERE), HERE, os.path.join(HERE, "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def make_dreamer(dev, B, S=8, H=5, full=False):
    """small widths on 32x32 frames, or (full=True) the CarRacing widths on
    64x64 frames with S=64, H=15 (BASELINE configs[1] per rank)."""
    from formula import FULL, SMALL, replay_data
    from dreamer_amd import Dreamer
    cfg = dict(FULL if full else SMALL)
    n = 1024 if full else 64
    if full:
        S, H = 64, 15
    cfg.update(batch_size=B, sequence_length=S, horizon=H, buffer_size=n)
    torch.manual_seed(0)
    d = Dreamer(cfg, dev)
    fr, ac, rw, ct = replay_data(n, (64, 64) if full else (32, 32), 3, seed=3)
    rw = (np.sign(rw) * np.log1p(np.abs(rw))).astype(np.float32)
    d.buffer.load_arrays(fr, ac, rw, ct)
    return d


def run_epochs(d, eng, starts_list, seed=4321, pipelined=False):
    eng.rng.reseed(seed)
    out = []
    ag = d.agent
    grads, svals = [], []
    if pipelined:  # warm start of epoch e+1 beside epoch e's update (run_many)
        ls = eng.run_many(starts_list).cpu()
        out = [(float(a), float(c)) for a, c in ls]
    for st in ([] if pipelined else starts_list):
        la, lc = eng.run(st)
        torch.cuda.synchronize()
        out.append((float(la), float(lc)))
        # after each step the flat gradient buffer holds the clipped (global) gradients
        grads.append(ag.grad_buffer[:ag.fa.numel + ag.fc.numel].cpu())
        svals.append(float(ag.S_dev))
    return out, ag.fa.flat.cpu(), ag.fc.flat.cpu(), ag.ft.flat.cpu(), float(ag.S_dev), grads, svals


def worker(rank, world, port, B_global, starts_list, out_path, backend, pipelined=False, full=False):
    import torch.distributed as dist
    from dreamer_amd.engine import ImaginationEngine
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group(backend, rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    b = B_global // world
    d = make_dreamer(dev, b, full=full)
    eng = ImaginationEngine(d, B=b, world=(rank, world, dist.group.WORLD))
    mine = [st[rank * b:(rank + 1) * b] for st in starts_list]
    res = run_epochs(d, eng, mine, pipelined=pipelined)
    if rank == 0:
        torch.save(res, out_path)
    dist.barrier()
    dist.destroy_process_group()


def run_wm_steps(d, starts_list, seed=98765):
    """world-model training steps from the device ring; returns losses and the flat parameters"""
    from dreamer_amd import hip
    hip.adhoc(d.device).reseed(seed)  # the world-model step draws from the ad-hoc generator
    out = []
    for st in starts_list:
        loss = d.world_model.train_step_ring(d.buffer, st)
        torch.cuda.synchronize()
        out.append(float(loss))
    return out, d.world_model._flat.flat.cpu()


def wm_worker(rank, world, port, B_global, starts_list, out_path, backend):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group(backend, rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    b = B_global // world
    d = make_dreamer(dev, b)
    d.world_model.set_data_parallel(rank, world, dist.group.WORLD)
    mine = [st[rank * b:(rank + 1) * b] for st in starts_list]
    res = run_wm_steps(d, mine)
    if rank == 0:
        torch.save(res, out_path)
    dist.barrier()
    dist.destroy_process_group()
