"""Benchmark: imagined latent-steps/sec (B x H) of Dreamer.train_Agent epochs
on MI355X (BASELINE.json metric), 64x64x3 CarRacing-shaped synthetic replay.

  python bench.py [--gpus N --steps K --warmup W --batch B --seq S --horizon H]

Multi-GPU: launched by torch.distributed.run, one process per GPU; weak
scaling (B rows per GPU), RCCL all-gather of lambda returns + one all-reduce
of the flat [actor|critic|loss] gradient buffer per epoch.  Rank 0 prints ONE
JSON line.  The CPU baseline (rank 0, N=1 only) times the oracle's
reference-faithful CPU restatement on a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "imagined latent-steps/sec (B×H) at 64×64 CarRacing, 1/2/4/8 MI355X"
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_16x16x4_f32 = f32 vector peak
HBM_PEAK_GBS = 8000.0
# HBM-side bytes of the encoder group per epoch, measured by tools/pmc_traffic.sh
# (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, gfx950 correction)
TRAFFIC_FILE = os.path.join(REPO, "profiles", "r01_traffic.json")
# SURVEY.md §8d figure of record: necessary dense FLOPs per imagined step at
# 64x64, S=64, H=15 (warm start 131.07 + dream 8.88 + update 11.17 MFLOP)
PATH_MFLOP_PER_STEP = {(64, 15, 64): 151.12, (50, 15, 64): 122.36, (64, 20, 128): 383.00}

CAR_RACER = dict(
    hidden_state_dims=600, latent_state_dims=[32, 32], action_dims=3, observation_dims=[64, 64],
    encoder_filter_num_1=32, encoder_filter_num_2=64, encoder_hidden_layer_nodes=200,
    decoder_filter_num_1=32, decoder_filter_num_2=64, decoder_hidden_layer_nodes=200,
    dyn_pred_hidden_num_nodes_1=200, dyn_pred_hidden_num_nodes_2=200,
    rew_pred_hidden_num_nodes_1=200, rew_pred_hidden_num_nodes_2=200,
    cont_pred_hidden_num_nodes_1=200, cont_pred_hidden_num_nodes_2=200,
    hidden_layer_actor_1_size=200, hidden_layer_actor_2_size=200,
    hidden_layer_critic_1_size=200, hidden_layer_critic_2_size=200, device="cuda",
    horizon=15, batch_size=64, nu=0.0003, lambda_=0.95, gamma=0.99, buffer_size=200000,
    sequence_length=64, seed=42, training_iterations=10000, random_iterations=500,
    actor_lr=0.00008, actor_betas=[0.9, 0.999], actor_eps=0.00001, critic_lr=0.0001,
    critic_betas=[0.9, 0.999], critic_eps=0.00001, AC_epochs=1, world_model_lr=0.0001,
    world_model_betas=[0.9, 0.999], world_model_eps=0.00001, WM_epochs=1,
    beta_prediction=1.0, beta_dynamics=0.5, beta_representation=0.1, critic_reward_buckets=255,
    env_id="CarRacing-v3",
)


def synthetic_replay(n, hw, A, seed=0):
    """u8 frames, U(-1,1) actions, N(0,1) rewards (symlog'ed as
    add_to_buffer does), continues 1 except every 1000th."""
    rng = np.random.default_rng(seed)
    frames = rng.integers(0, 256, size=(n, 3, hw[0], hw[1]), dtype=np.uint8)
    acts = rng.uniform(-1, 1, size=(n, A)).astype(np.float32)
    r = rng.standard_normal(size=(n,)).astype(np.float32)
    rews = (np.sign(r) * np.log(1.0 + np.abs(r))).astype(np.float32)
    conts = np.ones((n,), dtype=np.float32)
    conts[::1000] = 0.0
    return frames, acts, rews, conts


def encoder_flops_per_frame(c):
    """Algorithmic FLOPs of the conv stack + latent_mapper.0 feature columns
    for one 64x64 frame (dense conv FLOPs; SURVEY §8d counting)."""
    ch = [3, c["encoder_filter_num_1"], c["encoder_filter_num_2"], 2 * c["encoder_filter_num_2"],
          4 * c["encoder_filter_num_2"]]
    h, w = c["observation_dims"]
    fl = 0
    for i in range(4):
        h, w = h // 2, w // 2
        fl += 2 * h * w * ch[i + 1] * ch[i] * 16
    F = ch[4] * h * w
    return fl + 2 * F * c["encoder_hidden_layer_nodes"]


def wm_step_flops(c, B, T):
    """Algorithmic (dense) FLOPs of one WorldModel.training_step on B windows
    of T steps: encoder on all B*T frames, posterior scan, prior / reward /
    continue heads and decoder on the B*(T-1) rows the losses read
    (WorldModel.py:141-145), backward = 2x forward minus the first conv's
    (unneeded) input gradient."""
    Hd, (R, C), A = c["hidden_state_dims"], c["latent_state_dims"], c["action_dims"]
    L = R * C
    eh, dh = c["encoder_hidden_layer_nodes"], c["decoder_hidden_layer_nodes"]
    h, w = c["observation_dims"]
    M, M1 = B * T, B * (T - 1)
    f1, f2 = c["decoder_filter_num_1"], c["decoder_filter_num_2"]
    conv1 = 2 * (h // 2) * (w // 2) * c["encoder_filter_num_1"] * 3 * 16
    enc = encoder_flops_per_frame(c) * M
    scan = M * 2 * (3 * Hd * (L + A + Hd) + eh * Hd + L * eh)
    p1, p2 = c["dyn_pred_hidden_num_nodes_1"], c["dyn_pred_hidden_num_nodes_2"]
    r1, r2 = c["rew_pred_hidden_num_nodes_1"], c["rew_pred_hidden_num_nodes_2"]
    q1, q2 = c["cont_pred_hidden_num_nodes_1"], c["cont_pred_hidden_num_nodes_2"]
    nb = c["critic_reward_buckets"]
    Fd = 4 * f2 * (h // 16) * (w // 16)
    heads = 2 * (Hd * p1 + p1 * p2 + p2 * L + (Hd + L) * r1 + r1 * r2 + r2 * nb + (Hd + L) * q1 + q1 * q2 + q2
                 + (Hd + L) * dh + dh * Fd)
    chans = [4 * f2, 2 * f2, f2, f1, 3]
    dec = 0
    hh, ww = h // 16, w // 16
    for i in range(4):
        dec += 2 * hh * ww * chans[i] * chans[i + 1] * 16
        hh, ww = 2 * hh, 2 * ww
    fwd = enc + scan + M1 * (heads + dec)
    return 3 * fwd - conv1 * M


def bench_wm(d, B, steps, warmup):
    """WorldModel.training_step throughput (sequences/s) fed from the device
    replay ring (Dreamer.train_world_model's unit of work)."""
    wm = d.world_model
    for _ in range(warmup):
        wm.train_step_ring(d.buffer, d.buffer.sample_start_indices(B))
    torch.cuda.synchronize()
    st = [d.buffer.sample_start_indices(B) for _ in range(steps)]
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for s in st:
        wm.train_step_ring(d.buffer, s)
    ev1.record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return el / steps, ev0.elapsed_time(ev1) / 1e3 / steps, float(wm.last_losses[0])


def cpu_baseline(cfg, B, S, H, budget_s=15.0, threads=None):
    """Reference-faithful CPU epoch (oracle restatement of Dreamer.train_Agent:
    warm start with the un-detached graph, dream, train_step with backward into
    everything, AdamW, EMA) timed on the host cores."""
    from oracle import dreamer_oracle as O
    from dreamer_amd import Dreamer
    threads = threads or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    c = dict(cfg)
    c.update(device="cpu", batch_size=B, sequence_length=S, horizon=H)
    torch.manual_seed(0)
    d = Dreamer(c, torch.device("cpu"))
    P = {k: v.detach().clone().requires_grad_(v.dtype == torch.float32 and "buckets" not in k)
         for k, v in d.state_dict().items()}
    R, C = c["latent_state_dims"]
    A = c["action_dims"]
    frames, acts, rews, conts = synthetic_replay(max(4096, 8 * S), c["observation_dims"], A, seed=0)
    rng = np.random.default_rng(1)
    actor = [P["agent." + k] for k in O.ACTOR_KEYS]
    critic = [P["agent." + k] for k in O.CRITIC_KEYS]
    m = {id(p): (torch.zeros_like(p), torch.zeros_like(p)) for p in actor + critic}
    S_val = 1.0

    def epoch(step):
        nonlocal S_val
        st = rng.integers(0, len(frames) - S, size=B)
        idx = st[:, None] + np.arange(S)[None, :]
        obs = torch.tensor(frames[idx], dtype=torch.float32)
        act = torch.tensor(acts[idx])
        qw = torch.empty(S // 2, B * R, C).exponential_()
        z0, h0 = O.warm_start(obs, act, S, P, qw, R, C)
        eps = torch.randn(H, B, 1, A)
        q = torch.empty(H, B * R, C).exponential_()
        z, h, a, r, cc, mu, sg = O.dream(z0, h0, P, eps, q, H, R, C)
        la, lc, Rl, S_val = O.ac_losses(z, h, r, cc, a, mu, sg, P, S_val)
        for p in actor + critic:
            p.grad = None
        lc.backward()
        la.backward()  # traverses the dream AND the warm-start graph, as the reference does
        for ps, lr in ((critic, 1e-4), (actor, 8e-5)):
            gs, _ = O.clip_grad_norm([p.grad for p in ps])
            with torch.no_grad():
                for p, g in zip(ps, gs):
                    mm, vv = m[id(p)]
                    pn, mn, vn = O.adamw_step(p, g, mm, vv, step, lr)
                    p.copy_(pn); mm.copy_(mn); vv.copy_(vn)
        with torch.no_grad():
            for k in O.CRITIC_KEYS:
                t = P["agent.target_" + k]
                t.mul_(0.98).add_(0.02 * P["agent." + k])

    epoch(1)  # warm-up (not timed)
    n, t0 = 0, time.perf_counter()
    while True:
        epoch(2 + n)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 50:
            break
    return dict(value=B * H * n / el, unit="imagined latent-steps/s", cores=threads, kind="port",
                sample=f"{n} reference-faithful train_Agent epochs (oracle CPU restatement, fp32, warm-start "
                       f"backward included) at B={B} S={S} H={H} {c['observation_dims'][0]}x{c['observation_dims'][1]}x3, "
                       f"{el:.1f} s on {threads} threads")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64, help="imagination rows per GPU (configs[1]: 64)")
    ap.add_argument("--seq", type=int, default=64)
    ap.add_argument("--horizon", type=int, default=15)
    ap.add_argument("--res", type=int, default=64,
                    help="frame side (64: CarRacing configs[1]; 128: configs[3]'s frames with the reference's "
                         "4-conv encoder -- the 'deeper VAE' is not in the reference)")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--phases", action="store_true", help="print per-phase ms to stderr")
    ap.add_argument("--sequential", action="store_true",
                    help="report the epochs run one after another (no warm-start / update overlap)")
    ap.add_argument("--wm-steps", type=int, default=10, help="world-model training steps timed (0: skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("DREAMER_DIST_BACKEND") == "gloo":
        local %= max(1, torch.cuda.device_count())  # rehearsal: several ranks may share one GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    if world > 1:
        import torch.distributed as dist
        # nccl = RCCL over xGMI; DREAMER_DIST_BACKEND=gloo rehearses N ranks on one GPU
        backend = os.environ.get("DREAMER_DIST_BACKEND", "nccl")
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)
        group = dist.group.WORLD

    from dreamer_amd import Dreamer
    from dreamer_amd.engine import ImaginationEngine
    B, S, H = args.batch, args.seq, args.horizon
    cfg = dict(CAR_RACER)
    cfg.update(batch_size=B, sequence_length=S, horizon=H, observation_dims=[args.res, args.res])
    torch.manual_seed(0)
    d = Dreamer(cfg, dev)
    n_rep = max(4096, 8 * S)
    fr, ac, rw, ct = synthetic_replay(n_rep, cfg["observation_dims"], cfg["action_dims"], seed=0)
    d.buffer.load_arrays(fr, ac, rw, ct)
    d.buffer._mirror()
    eng = ImaginationEngine(d, B=B, world=(rank, world, group) if world > 1 else None)
    d._engine = eng
    if world > 1:
        d.world_model.set_data_parallel(rank, world, group)
    np.random.seed(1000 + rank)

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()

    def timed_epochs(pipelined):
        """K consecutive train_Agent epochs after W warm-up ones.  Pipelined:
        the warm start of epoch e+1 overlaps epoch e's actor-critic chain
        (ImaginationEngine.run_many; the pipeline fills and drains inside the
        timed region).  Sequential: one epoch after the other (engine.run)."""
        if pipelined:
            eng.run_many([d.buffer.sample_start_indices(B) for _ in range(args.warmup)])
        else:
            for _ in range(args.warmup):
                eng.run(d.buffer.sample_start_indices(B))
        starts = [d.buffer.sample_start_indices(B) for _ in range(args.steps)]
        barrier()
        t0 = time.perf_counter()
        phase_tot = {}
        if pipelined:
            eng.run_many(starts)
        else:
            for st in starts:
                eng.run(st, timing=True)
                if args.phases:
                    torch.cuda.current_stream().synchronize()
                    for k, v in eng.phase_ms().items():
                        phase_tot[k] = phase_tot.get(k, 0.0) + v
        barrier()
        el = time.perf_counter() - t0
        if world > 1:
            import torch.distributed as dist
            t = torch.tensor([el], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t)
        return el, phase_tot

    el_seq, phase_tot = timed_epochs(False)
    el = el_seq if args.sequential else timed_epochs(True)[0]
    la, lc = float(d.agent.loss_buffer[0]), float(d.agent.loss_buffer[1])
    # the world-model step all-reduces under DP: every rank runs it (max over ranks)
    wm = None
    if args.wm_steps > 0:
        wm_s, wm_gpu_s, wm_loss = bench_wm(d, B, args.wm_steps, 2)
        if world > 1:
            import torch.distributed as dist
            t = torch.tensor([wm_s, wm_gpu_s], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            wm_s, wm_gpu_s = (float(x) for x in t.cpu())
        wm = (wm_s, wm_gpu_s, wm_loss)
    if rank != 0:
        barrier()
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    value = world * B * H * args.steps / el
    frames = B * (S // 2)
    enc_flops = encoder_flops_per_frame(cfg) * frames
    # the dominant kernel group (conv encoder + feature projection, all time
    # chunks) timed live with HIP events on the engine's stream, back to back
    # without the overlapping scan, after the timed region
    enc_s = eng.time_encoder(reps=5) / 1e3
    achieved = enc_flops / enc_s / 1e12
    if args.phases:
        print(json.dumps({k: round(v / args.steps, 4) for k, v in phase_tot.items()}), file=sys.stderr)
    traffic, traffic_src = None, None
    if os.path.exists(TRAFFIC_FILE):
        t = json.load(open(TRAFFIC_FILE))
        traffic, traffic_src = t.get("encoder_bytes_per_epoch"), os.path.relpath(TRAFFIC_FILE, REPO)
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "imagined latent-steps/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"Dreamer.train_Agent epoch (replay sample + warm start S/2 + H-step imagination + "
                               f"actor-critic update), B={B}/GPU S={S} H={H} {args.res}x{args.res}x3"
                               + (" (BASELINE configs[1])" if (args.res, B, S, H) == (64, 64, 64, 15) else ""),
                   "global_batch": B * world, "seq_len": S, "horizon": H, "parallelism": f"dp{world}"},
        "roofline": {"bound": "mfma", "kernel": f"encoder conv stack + feature projection ({len(eng.chunks)} time chunks x 5 launches)",
                     "achieved": round(achieved, 2), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
                     "traffic_unit": "bytes per epoch (HBM side)", "traffic_source": traffic_src,
                     "algorithmic_flops_per_launch": enc_flops, "encoder_ms": round(enc_s * 1e3, 4)},
        "losses": {"actor": la, "critic": lc},
        "epochs": {"mode": "sequential" if args.sequential else "pipelined",
                   "pipelined_note": "warm start (encoder + posterior scan, world-model parameters only) of epoch "
                                     "e+1 runs on a second stream beside epoch e's imagination / actor-critic "
                                     "update; results equal the sequential epochs bit for bit "
                                     "(tests/test_gpu_parity.py::test_pipelined_epochs_match_sequential)",
                   "sequential_value": round(world * B * H * args.steps / el_seq, 1),
                   "sequential_ms_per_step": round(el_seq / args.steps * 1e3, 4)},
    }
    mf = PATH_MFLOP_PER_STEP.get((S, H, args.res))
    if mf is not None:
        tf = value * mf * 1e6 / 1e12
        out["path_roofline"] = {"bound": "mfma", "achieved": round(tf, 2), "peak": FP32_MFMA_PEAK_TFLOPS,
                                "unit": "TFLOP/s", "frac": round(tf / FP32_MFMA_PEAK_TFLOPS, 4),
                                "mflop_per_imagined_step": mf,
                                "note": "whole train_Agent epoch, SURVEY §8d necessary FLOPs x imagined steps/s"}
    if wm is not None:
        wm_s, wm_gpu_s, wm_loss = wm
        fl = wm_step_flops(cfg, B, H)
        ac_s = el / args.steps
        out["secondary"] = {
            "wm_step": {"value": round(world * B / wm_s, 1), "unit": "sequences/s", "ms_per_step": round(wm_s * 1e3, 3),
                        "gpu_ms_per_step": round(wm_gpu_s * 1e3, 3), "B_per_gpu": B, "T": H, "loss": wm_loss,
                        "mfma_tflops": round(fl / wm_s / 1e12, 2),
                        "mfma_frac": round(fl / wm_s / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4),
                        "algorithmic_gflop": round(fl / 1e9, 2),
                        "note": "WorldModel.training_step (posterior scan, decoder, losses, full backward, clip, "
                                "AdamW) from the device replay ring; under DP the mask / loss sums and the flat "
                                "gradient are all-reduced (RCCL)"},
            "full_iteration": {"value": round(world * B * H / (wm_s + ac_s), 1), "unit": "imagined latent-steps/s",
                               "ms_per_iteration": round((wm_s + ac_s) * 1e3, 3),
                               "note": "1 WM step + 1 train_Agent epoch per iteration (WM_epochs = AC_epochs = 1)"},
        }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, B, S, H, budget_s=args.cpu_budget)
    print(json.dumps(out), flush=True)
    if world > 1:
        barrier()
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
