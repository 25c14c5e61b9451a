"""CPU-baseline fidelity: wall time of the reference's own
Dreamer.train_Agent epoch (imported from /root/reference, build container
only) against bench.CpuEpoch -- the oracle's reference-faithful restatement
that bench.py times as `cpu_baseline` on the GPU box -- on identical inputs,
weights and noise, same thread count.  Also checks the first epoch's losses
agree bit for bit.  Writes profiles/r02_cpu_fidelity.json.

  python tools/cpu_fidelity.py [--threads 8]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import bench  # noqa: E402


def ref_dreamer(cfg, B, S, H, frames, acts, rews, conts):
    sys.path.insert(0, "/root/reference")
    from Dreamer import Dreamer as RefDreamer
    c = dict(cfg)
    c.update(device="cpu", batch_size=B, sequence_length=S, horizon=H, AC_epochs=1, buffer_size=len(frames))
    torch.manual_seed(0)
    d = RefDreamer(c, torch.device("cpu"))
    for i in range(len(frames)):
        d.buffer.add_to_buffer(frames[i], acts[i], float(np.sign(rews[i]) * np.expm1(abs(rews[i]))), conts[i])
    return d


def run(cfg, B, S, H, reps):
    from oracle import dreamer_oracle as O
    n = max(4096, 8 * S) if B > 16 else 512
    frames, acts, rews, conts = bench.synthetic_replay(n, cfg["observation_dims"], cfg["action_dims"], seed=0)
    ref = ref_dreamer(cfg, B, S, H, frames, acts, rews, conts)
    ce = bench.CpuEpoch(cfg, B, S, H)
    ce.P = {k: v.detach().clone().requires_grad_(v.dtype == torch.float32 and "buckets" not in k)
            for k, v in ref.state_dict().items()}
    ce.actor = [ce.P["agent." + k] for k in O.ACTOR_KEYS]
    ce.critic = [ce.P["agent." + k] for k in O.CRITIC_KEYS]
    ce.m = {id(p): (torch.zeros_like(p), torch.zeros_like(p)) for p in ce.actor + ce.critic}
    R, C, A = 32, 32, cfg["action_dims"]
    t_ref, t_port = [], []
    same = None
    for rep in range(reps + 1):
        np.random.seed(100 + rep)
        torch.manual_seed(200 + rep)
        t0 = time.perf_counter()
        la_r, lc_r = ref.train_Agent()
        t1 = time.perf_counter()
        # the same windows and the reference's draws in its order, for the port
        np.random.seed(100 + rep)
        st = O.replay_starts(ref.buffer.size, ref.buffer.capacity, ref.buffer.next_idx, S, B)
        idx = (st[:, None] + np.arange(S)[None, :]) % ref.buffer.capacity
        obs = torch.tensor(ref.buffer.observation_buffer[idx], dtype=torch.float32)
        act = torch.tensor(ref.buffer.action_buffer[idx])
        torch.manual_seed(200 + rep)
        qw = torch.stack([torch.empty(B * R, C).exponential_() for _ in range(S // 2)])
        eps, q = [], []
        for _ in range(H):
            eps.append(torch.empty(B, 1, A).normal_())
            q.append(torch.empty(B * R, C).exponential_())
        ce.set_inputs(obs, act, qw, torch.stack(eps), torch.stack(q))
        t2 = time.perf_counter()
        la_p, lc_p = ce.epoch()
        t3 = time.perf_counter()
        if rep == 0:
            same = (float(la_r) == la_p) and (float(lc_r) == lc_p)
            continue  # warm-up
        t_ref.append(t1 - t0)
        t_port.append(t3 - t2)
    return dict(B=B, S=S, H=H, ref_s=sorted(t_ref), port_s=sorted(t_port),
                ratio_min=min(t_port) / min(t_ref), ratio_median=float(np.median(t_port) / np.median(t_ref)),
                first_epoch_losses_bit_equal=same)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    model, phys, aff = bench.cpu_info()
    cfg = dict(bench.CAR_RACER)
    out = {"cpu_model": model, "threads": args.threads, "cases": []}
    for B, S, H in ((16, 50, 15), (64, 64, 15)):
        r = run(cfg, B, S, H, args.reps)
        print(json.dumps(r))
        out["cases"].append(r)
    out["note"] = ("ratio = port time / reference time per train_Agent epoch (min and median of the timed reps, "
                   "one warm-up epoch each); the port is bench.CpuEpoch (oracle reference-faithful mode)")
    json.dump(out, open(os.path.join(ROOT, "profiles", "r02_cpu_fidelity.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
